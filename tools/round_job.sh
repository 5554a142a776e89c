#!/bin/bash
# GPU-box job: GPU tests, default bench, other workloads, rocprofv3 stats.  Usage: bash tools/round_job.sh TAG
set -o pipefail
TAG=${1:-r01}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -3 $O/gpu_tests.txt
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
for w in c1 c4 c5; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit $?
  cat $O/bench_$w.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1)
cp "$f" $O/kernel_stats.csv && rm -rf $O/prof
head -n 12 $O/kernel_stats.csv | cut -c1-60,200-
echo done
