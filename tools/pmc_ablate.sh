#!/bin/bash
# GPU-box job: SQ counters per k_encode ablation variant (tools/ablate.py, interleaved).
# Usage: bash tools/pmc_ablate.sh TAG VARIANTS   e.g. 0,1,3,5
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; V=$2
mkdir -p gpurun_out/$TAG
n=$(echo $V | tr ',' '\n' | wc -l)
ABLATE=$V timeout -s KILL 240 rocprofv3 --kernel-include-regex 'k_encode' --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d gpurun_out/$TAG/p1 -o run --output-format csv -- python3 tools/ablate.py > gpurun_out/$TAG/p1.log 2>&1 || exit 1
python3 tools/pmc_by_order.py gpurun_out/$TAG/p1 $n 3 | tee gpurun_out/$TAG/summary.txt
