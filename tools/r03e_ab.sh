#!/bin/bash
# GPU tests on the in-tree build, then kernel A/B (variants.py, one process) and bench A/B
# against libmjgpu_v_oldtail.so.   Usage: bash tools/r03e_ab.sh TAG [workloads]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for w in ${2:-c2 c1}; do
  WL=$w VARIANTS="oldtail=:;new=:" timeout -k 10 300 python3 tools/variants.py > $O/ab_$w.txt 2>&1 || { tail -20 $O/ab_$w.txt; exit 1; }
  grep -E "median|output" $O/ab_$w.txt
done
for w in ${2:-c2 c1}; do
  for i in 1 2; do
    for v in old new; do
      if [ $v = old ]; then export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_oldtail.so; else unset MJG_LIBRARY; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload $w > $O/$w.$v$i.json 2>>$O/err.log || exit $?
      python3 -c "import json,sys; d=json.load(open('$O/$w.$v$i.json')); print('$w $v$i', d['value'], {k:v for k,v in d['kernel_ms_per_step'].items() if v})"
    done
  done
done
echo done
