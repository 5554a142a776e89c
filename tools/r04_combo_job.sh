#!/bin/bash
# GPU-box job: GPU tests, a variants.py A/B over CASES, then the phase probe over PCASES.
# Usage: VARIANTS=... CASES=... PCASES=... bash tools/r04_combo_job.sh TAG
set -o pipefail
TAG=$1
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for c in $CASES; do
  wl=${c%%:*}; ct=${c##*:}
  WL=$wl CONTENT=$ct timeout -k 10 240 python -u tools/variants.py > $O/ab_${wl}_${ct}.txt 2>&1 || { tail -20 $O/ab_${wl}_${ct}.txt; exit 1; }
  echo "== $wl $ct"; grep -E "median|!=" $O/ab_${wl}_${ct}.txt
done
for c in $PCASES; do
  wl=${c%%:*}; ct=${c##*:}
  WL=$wl CONTENT=$ct timeout -k 10 120 python -u tools/phase_probe.py ph > $O/phase_${wl}_${ct}.txt 2>&1 || { tail -20 $O/phase_${wl}_${ct}.txt; exit 1; }
  grep -v amdgpu.ids $O/phase_${wl}_${ct}.txt
done
echo done
