#!/bin/bash
# GPU-box job: tools/variants.py A/B (VARIANTS env) over workloads / contents.
# Usage: VARIANTS="a=...;b=..." bash tools/r04_ab.sh TAG "c2:testsrc c2:natural ..." [tests]
set -o pipefail
TAG=$1; CASES=${2:-c2:testsrc}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$3" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
  tail -2 $O/gpu_tests.txt
fi
for c in $CASES; do
  wl=${c%%:*}; ct=${c##*:}
  WL=$wl CONTENT=$ct timeout -k 10 240 python -u tools/variants.py > $O/ab_${wl}_${ct}.txt 2>&1 || { tail -20 $O/ab_${wl}_${ct}.txt; exit 1; }
  echo "== $wl $ct"; grep -E "median|!=" $O/ab_${wl}_${ct}.txt
done
echo done
