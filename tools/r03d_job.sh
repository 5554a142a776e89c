#!/bin/bash
# round 3 job (tiled k_stuff): GPU tests on the in-tree build; kernel A/B against the round-2
# code (libmjgpu_v_oldtail.so) and the phase ablations (tools/ablate.py) in one process; bench
# A/B old vs new; default bench line with the e2e leg.
#   Usage: [V2=... V1=...] [PROF=1] bash tools/r03d_job.sh TAG  (V2/V1: the c2/c1 VARIANTS)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
WL=c2 VARIANTS="${V2:-oldtail=:;full=:;noemit=:;noexact=:;noscreen=:;nodct=:}" timeout -k 10 400 python3 tools/variants.py > $O/ab_c2.txt 2>&1 || { tail -20 $O/ab_c2.txt; exit 1; }
grep median $O/ab_c2.txt
WL=c1 VARIANTS="${V1:-oldtail=:;full=:}" timeout -k 10 300 python3 tools/variants.py > $O/ab_c1.txt 2>&1 || { tail -20 $O/ab_c1.txt; exit 1; }
grep median $O/ab_c1.txt
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
timeout -k 10 300 python bench.py --cpu-seconds 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['kernel_ms_per_step'])); print(json.dumps(d['e2e']))"
if [ -n "$PROF" ]; then bash tools/driver_prof.sh $1/driver || exit $?; fi
echo done
