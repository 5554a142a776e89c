#!/bin/bash
# GPU-box job: tools/variants.py A/B (VARIANTS env) over CASES, no tests.
set -o pipefail
TAG=$1
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for c in $CASES; do
  wl=${c%%:*}; ct=${c##*:}
  WL=$wl CONTENT=$ct timeout -k 10 240 python -u tools/variants.py > $O/ab_${wl}_${ct}.txt 2>&1 || { tail -20 $O/ab_${wl}_${ct}.txt; exit 1; }
  echo "== $wl $ct"; grep -E "median|!=" $O/ab_${wl}_${ct}.txt
done
echo done
