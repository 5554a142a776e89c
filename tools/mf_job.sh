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
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -40 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
for c in $CASES; do
  wl=${c%%:*}; ct=${c##*:}
  echo "== $wl $ct"
  WL=$wl CONTENT=$ct VARIANTS="${AB:-valu=:;mf_m=:}" timeout -k 10 200 python tools/variants.py > $O/ab_${wl}_${ct}.txt 2>&1 || { tail -20 $O/ab_${wl}_${ct}.txt; exit 1; }
  cat $O/ab_${wl}_${ct}.txt
done
echo done
