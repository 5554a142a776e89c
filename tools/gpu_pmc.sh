#!/bin/bash
# GPU-box job: separate rocprofv3 --pmc passes over tools/pmc_workload.py (k_* kernels only).
# Usage: bash tools/gpu_pmc.sh TAG [counter-set ...]   (each set = one pass)
set -o pipefail
TAG=${1:-pmc}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex 'mjg::' --pmc $set -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 tools/pmc_workload.py > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
