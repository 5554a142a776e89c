#!/bin/bash
# GPU-box job: GPU tests, then the phase_clock probe (tools/phase_probe.py) over contents.
set -o pipefail
TAG=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
  tail -2 $O/gpu_tests.txt
fi
for c in ${CASES:-c2:testsrc}; do
  wl=${c%%:*}; ct=${c##*:}
  WL=$wl CONTENT=$ct timeout -k 10 120 python -u tools/phase_probe.py "$@" > $O/phase_${wl}_${ct}.txt 2>&1 || { tail -20 $O/phase_${wl}_${ct}.txt; exit 1; }
  cat $O/phase_${wl}_${ct}.txt
done
echo done
