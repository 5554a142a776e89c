#!/bin/bash
# GPU tests (in-tree build), output equality of the variants (variants.py, one process), then
# the serial per-kernel timings of each.   Usage: bash tools/r03e_job4.sh TAG "v1 v2 ..." [wl]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
VS=$(for v in $2; do printf "%s=:;" $v; done); VS=${VS%;}
WL=${3:-c2} VARIANTS="$VS" timeout -k 10 300 python3 tools/variants.py > $O/var_all.txt 2>&1 || { tail -20 $O/var_all.txt; exit 1; }
grep -E "output|median" $O/var_all.txt
bash tools/r03e_tailprof.sh $1 "$2" ${3:-c2}
