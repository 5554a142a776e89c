#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
bash tools/r03e_tailprof.sh $1 "$2" c2 || exit 1
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_oldtail.so; else unset MJG_LIBRARY; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload c2 > $O/c2.$v$i.json 2>>$O/err.log || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/c2.$v$i.json')); print('c2 $v$i', d['value'], {k:v for k,v in d['kernel_ms_per_step'].items() if v})"
  done
done
