#!/bin/bash
# GPU-box job: GPU tests on the in-tree build, then A/B against OLD.so on the listed workloads.
#   bash tools/ab_job.sh OLD.so TAG [workload...]
set -o pipefail
cd "$(dirname "$0")/.."
OLD=$1; TAG=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for w in "$@"; do
  for i in 1 2; do
    for v in old new; do
      if [ $v = old ]; then export MJG_LIBRARY=$OLD; else unset MJG_LIBRARY; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload $w > $O/$w.$v$i.json 2>>$O/err.log || exit $?
      python -c "import json,sys; d=json.load(open('$O/$w.$v$i.json')); print('$w $v$i', d['value'], {k:v for k,v in d['kernel_ms_per_step'].items() if v})"
    done
  done
done
echo done
