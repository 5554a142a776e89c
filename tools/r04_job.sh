#!/bin/bash
# GPU-box job (round 4): GPU tests, HEAD per-kernel HBM traffic (tools/pmc_traffic.sh, every
# workload), one SQ pass of k_encode on c2, and the driver's command under rocprofv3
# (tools/driver_prof.sh; its prof.err is checked for the round-3 SIGTERM/SIGSEGV).
# Usage: bash tools/r04_job.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r04}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$2" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
  tail -2 $O/gpu_tests.txt
fi
bash tools/pmc_traffic.sh c2 c1 c4 c5 > $O/pmc_traffic.log 2>&1 || { tail -20 $O/pmc_traffic.log; exit 1; }
cat $O/pmc_traffic.log
cp gpurun_out/pmc_traffic/pmc_*.json $O/
WL=c2 bash tools/gpu_pmc.sh $TAG/sq "SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU" > $O/sq.log 2>&1 || { tail -20 $O/sq.log; exit 1; }
python3 -c "
import json, sys; sys.path.insert(0, '.')
from ffmpeg_distributed_amd import build as B
d = json.load(open('$O/sq/summary.json'))
json.dump({'library_digest': B.source_digest(), 'workload': 'c2 (tools/pmc_workload.py, 3 synced launches)', 'kernels': d}, open('$O/pmc_sq_c2.json', 'w'), indent=1)"
bash tools/driver_prof.sh $TAG/driver > $O/driver.log 2>&1 || { tail -20 $O/driver.log; exit 1; }
tail -3 $O/driver.log | cut -c1-400
echo "prof.err SIGTERM/SIGSEGV/Abort lines: $(grep -c -E 'SIGTERM|SIGSEGV|Abort' $O/driver/prof.err)"
echo done
