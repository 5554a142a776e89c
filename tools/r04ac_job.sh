#!/bin/bash
# GPU-box probe: rocprofv3 kernel trace of bench.py (c2 and natural), per-step timeline.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04ac
mkdir -p $O
for c in testsrc natural; do
  timeout -k 10 200 rocprofv3 --kernel-trace --kernel-include-regex 'mjg::' -d $O/t_$c -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-e2e --content $c --steps 20 --warmup 3 > $O/b_$c.json 2> $O/e_$c.log || exit 1
  f=$(find $O/t_$c -name "*kernel_trace.csv" | head -n 1)
  cp "$f" $O/trace_$c.csv && rm -rf $O/t_$c
  python3 tools/timeline.py $O/trace_$c.csv
done
