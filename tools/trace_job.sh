#!/bin/bash
# GPU-box probe: rocprofv3 kernel trace (per dispatch start/end) of bench.py at two segment
# lengths, to see how k_encode's duration splits into per-frame and per-launch parts and how
# the tail kernels on the second stream overlap it.  Usage: bash tools/trace_job.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for seg in ${SEGS:-30 120}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --kernel-include-regex 'mjg::' -d $O/t$seg -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --seg $seg --steps 10 --warmup 2 > $O/b$seg.json 2> $O/e$seg.log || exit 1
  f=$(find $O/t$seg -name "*kernel_trace.csv" | head -n 1)
  cp "$f" $O/trace_$seg.csv && rm -rf $O/t$seg
done
python3 tools/trace_summary.py $(for s in ${SEGS:-30 120}; do echo $O/trace_$s.csv; done)
