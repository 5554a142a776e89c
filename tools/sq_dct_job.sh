#!/bin/bash
# GPU-box job: HBM traffic of the c4 chain at its default DCT stage (profiles/pmc_c4.json), then
# one SQ counter pass per DCT stage of k_encode on a workload (default c2).
# Usage: bash tools/sq_dct_job.sh TAG [WORKLOAD]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; WL=${2:-c2}
O=gpurun_out/$TAG
mkdir -p $O
bash tools/pmc_traffic.sh c4 > $O/traffic.log 2>&1 || { tail -5 $O/traffic.log; exit 1; }
tail -2 $O/traffic.log
SET=SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU
for d in valu mfma; do
  timeout -s KILL 120 rocprofv3 --kernel-include-regex 'mjg::k_encode' --pmc $SET -d $O/sq_$d -o run --output-format csv -- python3 tools/pmc_workload.py --workload $WL --dct $d > $O/sq_$d.log 2>&1 || { echo "pass $d failed"; tail -5 $O/sq_$d.log; exit 1; }
  python3 tools/pmc_summary.py $O/sq_$d > $O/sq_$d.json || exit 1
  python3 -c "
import json; d = json.load(open('$O/sq_$d.json'))
for k, v in d.items(): print('$d', k[:40], json.dumps({c: round(x) for c, x in v.items()}))"
done
echo done
