#!/bin/bash
# GPU-box job: separate rocprofv3 --pmc passes over tools/pmc_workload.py (mjg:: kernels only).
# Usage: WL=c4 bash tools/gpu_pmc.sh TAG [counter-set ...]   (each set = one pass, <= 8 SQ counters)
set -o pipefail
TAG=${1:-pmc}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/$TAG
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex 'mjg::' --pmc $set -d gpurun_out/$TAG/p$i -o run --output-format csv -- python3 tools/pmc_workload.py --workload ${WL:-c2} ${PMC_ARGS:-} > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/$TAG/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/$TAG/p* > gpurun_out/$TAG/summary.json
python3 -c "
import json; d = json.load(open('gpurun_out/$TAG/summary.json'))
for k, v in d.items():
    if 'encode' in k or 'scale' in k: print(k[:50], json.dumps({c: round(x) for c, x in v.items()}))"
echo done
