#!/bin/bash
# GPU-box job: GPU tests, the default bench (the driver's command), other workloads, contents.
# Usage: bash tools/r04_bench_job.sh TAG
set -o pipefail
TAG=${1:-r04}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
for w in c1 c4 c5; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  cut -c1-300 $O/bench_$w.json
done
for c in natural noise-patches; do
  timeout -k 10 200 python bench.py --content $c --no-cpu-baseline --no-e2e > $O/bench_c2_$c.json 2> $O/bench_c2_$c.err || { tail -5 $O/bench_c2_$c.err; exit 1; }
  cut -c1-300 $O/bench_c2_$c.json
done
echo done
