#!/bin/bash
# SQ / TA / TCC counters of the tail kernels, old (libmjgpu_v_oldtail.so) and new (in-tree)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum"
for v in ${2:-old new}; do
  if [ $v = old ]; then export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_oldtail.so; else unset MJG_LIBRARY; fi
  i=0
  for set in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-include-regex 'mjg::' --pmc $set -d $O/${v}_p$i -o run --output-format csv -- python3 tools/pmc_workload.py --workload c2 > $O/${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 $O/${v}_p$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py $O/${v}_p* > $O/summary_$v.json
  python3 -c "
import json; d = json.load(open('$O/summary_$v.json'))
for k, v in d.items():
    if 'encode' not in k: print('$v', k[:30], json.dumps({c: round(x) for c, x in v.items()}))"
done
echo done
