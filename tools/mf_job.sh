#!/bin/bash
# GPU-box job: full GPU tests on the in-tree build, then k_encode A/B of the MFMA DCT stage
# (MJG_F_DCT_MFMA, variant names ending in _m) against the VALU passes (tools/variants.py).
# Usage: bash tools/mf_job.sh TAG "WL:CONTENT ..."
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; CASES=${2:-"c2:testsrc c5:testsrc c4:testsrc c2:natural c2:noise-patches"}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
[ -n "$NOTEST" ] || tail -2 $O/gpu_tests.txt
for c in $CASES; do
  IFS=: read wl ct qq <<< "$c"
  echo "== $wl $ct q${qq:-default}"
  Q=${qq:-} WL=$wl CONTENT=$ct VARIANTS="${AB:-valu_v=:;mf_m=:}" timeout -k 10 200 python tools/variants.py > $O/ab_${wl}_${ct}${qq}.txt 2>&1 || { tail -20 $O/ab_${wl}_${ct}${qq}.txt; exit 1; }
  grep median $O/ab_${wl}_${ct}${qq}.txt
done
echo done
