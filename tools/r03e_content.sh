#!/bin/bash
# GPU tests (in-tree build), then variants.py A/B over contents and workloads
#   Usage: bash tools/r03e_content.sh TAG "v1 v2 ..." ["wl:content ..."]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
VS=$(for v in $2; do printf "%s=:;" $v; done); VS=${VS%;}
for wc in ${3:-c2:testsrc c2:natural c2:noise-patches c1:testsrc c4:testsrc}; do
  w=${wc%%:*}; c=${wc##*:}
  ROUNDS=${ROUNDS:-6} WL=$w CONTENT=$c VARIANTS="$VS" timeout -k 10 300 python3 tools/variants.py > $O/var_${w}_$c.txt 2>&1 || { tail -20 $O/var_${w}_$c.txt; exit 1; }
  echo "== $w $c"; grep -E "output|median" $O/var_${w}_$c.txt
done
echo done
