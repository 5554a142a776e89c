#!/bin/bash
# round 3 session job: GPU tests on the in-tree build, kernel A/B against the round-2 code
# (libmjgpu_v_oldtail.so: 4-kernel tail, 32-bit symbol records, packed row-image stores),
# bench A/B, k_encode breakdown, default bench line with the e2e leg.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for wl in c2 c1; do
  WL=$wl VARIANTS="old=tools/_voldtailsrc:;new=:" timeout -k 10 300 python3 tools/variants.py > $O/ab_$wl.txt 2>&1 || { tail -20 $O/ab_$wl.txt; exit 1; }
  tail -2 $O/ab_$wl.txt
done
for w in c2 c1; do
  for i in 1 2; do
    for v in old new; do
      if [ $v = old ]; then export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_oldtail.so; else unset MJG_LIBRARY; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload $w > $O/$w.$v$i.json 2>>$O/err.log || exit $?
      python3 -c "import json,sys; d=json.load(open('$O/$w.$v$i.json')); print('$w $v$i', d['value'], {k:v for k,v in d['kernel_ms_per_step'].items() if v})"
    done
  done
done
unset MJG_LIBRARY
bash tools/breakdown_job.sh $1/bd c2 > $O/bd.log 2>&1 || { tail -30 $O/bd.log; exit 1; }
tail -12 $O/bd.log
timeout -k 10 300 python bench.py --cpu-seconds 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['kernel_ms_per_step'])); print(json.dumps(d['e2e']))"
