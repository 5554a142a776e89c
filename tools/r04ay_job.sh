#!/bin/bash
# GPU-box job: HEAD records after mjg_submit_segments (new library digest): GPU tests, PMC
# traffic for c2 c1 c4 c5 (profiles/pmc_*.json), the c2 SQ pass, the driver-command profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04ay
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && tail -2 $O/gpu_tests.txt &&
bash tools/pmc_traffic.sh c2 c1 c4 c5 &&
WL=c2 bash tools/gpu_pmc.sh r04ay_sq SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU &&
bash tools/driver_prof.sh r04ay_driver
