#!/bin/bash
# GPU-box job: tools/variants.py A/B of prebuilt variant libraries (VARIANTS as for variants.py,
# built beforehand on the CPU with `VARIANTS=... python tools/variants.py --build`) over several
# workloads / contents.  Usage: VARIANTS="head=:;new=abtmp/new:" bash tools/variants_job.sh TAG [WL:CONTENT ...]
# (default c2:testsrc c2:natural c2:noise-patches c1:testsrc c5:testsrc c4:testsrc)
set -o pipefail
TAG=${1:-ab}
shift
CASES=${@:-c2:testsrc c2:natural c2:noise-patches c1:testsrc c5:testsrc c4:testsrc}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for c in $CASES; do
  wl=${c%%:*}; ct=${c##*:}
  echo "## $wl $ct" | tee -a $O/ab.txt
  WL=$wl CONTENT=$ct ROUNDS=${ROUNDS:-6} timeout -k 10 240 python3 tools/variants.py > $O/${wl}_$ct.txt 2>&1 || { tail -5 $O/${wl}_$ct.txt; exit 1; }
  grep -v amdgpu.ids $O/${wl}_$ct.txt | tee -a $O/ab.txt
done
echo done
