#!/bin/bash
# GPU-box job: selected GPU tests (PYTEST_K filter) then selected bench workloads.
# Usage: bash tools/quick_job.sh TAG "pytest -k expr" "c2 c4 ..."
set -o pipefail
TAG=$1; K=$2; WLS=$3
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
  tail -3 $O/gpu_tests.txt
fi
for w in $WLS; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], json.dumps(d['kernel_ms_per_step']), d['roofline']['kernel'], d['roofline']['frac'])"
done
echo done
