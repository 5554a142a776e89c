#!/bin/bash
# variants equality + serial kernel timings (no GPU tests): Usage: bash tools/r03e_job5.sh TAG "v1 v2" [wl]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
VS=$(for v in $2; do printf "%s=:;" $v; done); VS=${VS%;}
for w in ${3:-c2 c5}; do
  WL=$w VARIANTS="$VS" timeout -k 10 300 python3 tools/variants.py > $O/var_$w.txt 2>&1 || { tail -20 $O/var_$w.txt; exit 1; }
  echo "== $w"; grep -E "output|median" $O/var_$w.txt
done
bash tools/r03e_tailprof.sh $1 "$2" c2
