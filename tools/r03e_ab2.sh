#!/bin/bash
# GPU tests on the in-tree build, then bench A/B (interleaved) against libmjgpu_v_$2.so
#   Usage: bash tools/r03e_ab2.sh TAG OLDNAME "workloads"
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
for w in $3; do
  for i in 1 2; do
    for v in old new; do
      if [ $v = old ]; then export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_$2.so; else unset MJG_LIBRARY; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload $w > $O/$w.$v$i.json 2>>$O/err.log || exit $?
      python3 -c "import json,sys; d=json.load(open('$O/$w.$v$i.json')); print('$w $v$i', d['value'], d['ms_per_step'], {k:v for k,v in d['kernel_ms_per_step'].items() if v})"
    done
  done
done
echo done
