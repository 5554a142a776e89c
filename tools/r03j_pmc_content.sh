#!/bin/bash
# SQ counters of k_encode per content (in-tree build): one --pmc pass per content.
#   Usage: bash tools/r03j_pmc_content.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
for c in testsrc natural noise-patches; do
  PMC_ARGS="--content $c" bash tools/gpu_pmc.sh $1_$c "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES" || exit 1
done
echo done
