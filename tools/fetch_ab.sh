#!/bin/bash
# GPU-box job: k_encode FETCH_SIZE (raw units) for the in-tree build and for other builds.
# Usage: bash tools/fetch_ab.sh TAG LIB.so ...
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/$TAG
i=0
for lib in "" "$@"; do
  i=$((i+1))
  if [ -n "$lib" ]; then export MJG_LIBRARY=$lib; else unset MJG_LIBRARY; fi
  timeout -s KILL 120 rocprofv3 --kernel-include-regex 'k_encode' --pmc FETCH_SIZE -d gurun_tmp/$TAG/p$i -o run --output-format csv -- python3 tools/pmc_workload.py > gpurun_out/$TAG/p$i.log 2>&1 || exit 1
  python3 - "$lib" gurun_tmp/$TAG/p$i <<'PY'
import sys; sys.path.insert(0, "tools")
from pmc_summary import load
d = load([sys.argv[2]])
for k, v in d.items():
    print(sys.argv[1] or "in-tree", k[:40], "FETCH_SIZE units", round(v["FETCH_SIZE"]), "~GB", round(v["FETCH_SIZE"] * 2047.88 / 1e9, 3))
PY
done
