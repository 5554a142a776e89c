#!/bin/bash
# GPU-box job: HEAD breakdown of k_encode on a workload (default c2).
#   1. the gfx950 SQ counter list (rocprofv3 -L, SQ_ lines)
#   2. k_encode time of the full build and of each ablation (tools/ablate.py), one process,
#      interleaved rounds (tools/variants.py)
#   3. one SQ pass (8 counters) per build over tools/pmc_workload.py
# Usage: bash tools/breakdown_job.sh TAG [WORKLOAD]   (ablation .so files built beforehand)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; WL=${2:-c2}
O=gpurun_out/$TAG
mkdir -p $O
NAMES=${NAMES:-noemit noexact noscreen nodct}
timeout -s KILL 60 rocprofv3 -L > $O/counters_all.txt 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+" $O/counters_all.txt | sort -u > $O/sq_counters.txt || true
wc -l < $O/sq_counters.txt
VS=$(python3 tools/ablate.py --variants $NAMES)
WL=$WL VARIANTS="$VS" timeout -k 10 300 python3 tools/variants.py > $O/ablate_$WL.txt 2>&1 || { tail -20 $O/ablate_$WL.txt; exit 1; }
cat $O/ablate_$WL.txt
SET=${SQSET:-SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU}
for n in full $NAMES; do
  if [ $n = full ]; then unset MJG_LIBRARY; else export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_$n.so; fi
  timeout -s KILL 120 rocprofv3 --kernel-include-regex 'mjg::k_encode' --pmc $SET -d $O/sq_$n -o run --output-format csv -- python3 tools/pmc_workload.py --workload $WL > $O/sq_$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/sq_$n.log; exit 1; }
  python3 tools/pmc_summary.py $O/sq_$n > $O/sq_$n.json || exit 1
  python3 -c "
import json; d = json.load(open('$O/sq_$n.json'))
for k, v in d.items(): print('$n', k[:40], json.dumps({c: round(x) for c, x in v.items()}))"
  rm -rf $O/sq_$n
done
unset MJG_LIBRARY
echo done
