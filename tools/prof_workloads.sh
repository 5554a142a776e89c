#!/bin/bash
# GPU-box job: rocprofv3 kernel stats of bench.py for the given workloads.  Usage: bash tools/prof_workloads.sh TAG c1 c4 ...
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for w in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_bench_$w.json 2> $O/prof_$w.err || exit $?
  f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -n 1)
  cp "$f" $O/kernel_stats_$w.csv && rm -rf $O/prof_$w
  grep mjg $O/kernel_stats_$w.csv | cut -d, -f1-4 | cut -c1-120
done
echo done
