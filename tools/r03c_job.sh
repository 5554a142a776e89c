#!/bin/bash
# round 3 session job: GPU tests on the in-tree build; k_encode / tail A/B against the round-2
# code (libmjgpu_v_oldtail.so) and the round-3 changes reverted one at a time, plus the phase
# ablations of the current k_encode (tools/ablate.py), in one process; bench A/B; SQ passes;
# default bench line with the e2e leg.   Usage: bash tools/r03c_job.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
WL=c2 VARIANTS="oldtail=:;full=:;v5=:;nod16=:;noreg0=:;noemit=:;noexact=:;noscreen=:;nodct=:" timeout -k 10 400 python3 tools/variants.py > $O/ab_c2.txt 2>&1 || { tail -20 $O/ab_c2.txt; exit 1; }
grep median $O/ab_c2.txt
WL=c1 VARIANTS="oldtail=:;full=:;v5=:" timeout -k 10 300 python3 tools/variants.py > $O/ab_c1.txt 2>&1 || { tail -20 $O/ab_c1.txt; exit 1; }
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
SET=SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_INSTS_VMEM_RD
for n in v5 full oldtail noemit nodct; do
  export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_$n.so
  timeout -s KILL 120 rocprofv3 --kernel-include-regex 'mjg::k_encode' --pmc $SET -d $O/sq_$n -o run --output-format csv -- python3 tools/pmc_workload.py --workload c2 > $O/sq_$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/sq_$n.log; exit 1; }
  python3 tools/pmc_summary.py $O/sq_$n > $O/sq_$n.json && rm -rf $O/sq_$n || exit 1
  python3 -c "
import json; d = json.load(open('$O/sq_$n.json'))
for k, v in d.items(): print('$n', k[:40], json.dumps({c: round(x) for c, x in v.items()}))"
done
unset MJG_LIBRARY
timeout -k 10 300 python bench.py --cpu-seconds 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['kernel_ms_per_step'])); print(json.dumps(d['e2e']))"

# disk under the e2e leg's temporary files: filesystem and O_DIRECT read rate of a 1.5 GB file
{ df -T /tmp; dd if=/dev/zero of=/tmp/mjg_dd bs=16M count=96 oflag=direct 2>&1 | tail -1; dd if=/tmp/mjg_dd of=/dev/null bs=16M iflag=direct 2>&1 | tail -1; dd if=/tmp/mjg_dd of=/dev/null bs=16M 2>&1 | tail -1; rm -f /tmp/mjg_dd; } > $O/disk.txt 2>&1
cat $O/disk.txt
echo done
