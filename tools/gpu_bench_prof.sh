#!/bin/bash
# GPU-box job: bench + rocprofv3 kernel-trace stats.  Usage: bash tools/gpu_bench_prof.sh TAG
set -o pipefail
TAG=${1:-r01}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/prof_bench.json 2> gpurun_out/$TAG/prof.err || exit $?
f=$(find gpurun_out/$TAG/prof -name "*kernel_stats.csv" | head -n 1)
cp "$f" gpurun_out/$TAG/kernel_stats.csv && rm -rf gpurun_out/$TAG/prof
cat gpurun_out/$TAG/bench.json
head -n 12 gpurun_out/$TAG/kernel_stats.csv | cut -c1-60,200-
echo done
