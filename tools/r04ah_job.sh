#!/bin/bash
# GPU-box probe: bench.py c2 at segment lengths 60 / 120 / 240 / 480 frames (per-launch costs:
# k_encode's drain and the overlap of consecutive launches amortise over more frames).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r04ah
mkdir -p $O
for seg in 60 120 240 480; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --seg $seg --steps 10 --warmup 3 > $O/b_$seg.json 2> $O/e_$seg.log || { tail -5 $O/e_$seg.log; exit 1; }
  python3 -c "
import json; d = json.load(open('$O/b_$seg.json'))
print($seg, d['value'], d['ms_per_step'], round(d['kernel_ms_per_step']['encode'], 4))"
done
