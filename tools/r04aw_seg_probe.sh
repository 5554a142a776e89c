#!/bin/bash
# GPU-box probe: bench.py at 120 (the driver's), 240 and 480 frames per submit, same box,
# interleaved: how much of the step is per-launch ramp and drain in the pipelined regime
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04aw
mkdir -p $O
for r in 1 2; do
  for s in 120 240 480; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --seg $s --pool 960 > $O/b_${s}_$r.json 2> $O/b_${s}_$r.err || { tail -5 $O/b_${s}_$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/b_${s}_$r.json'))
print('seg', $s, $r, d['value'], d['ms_per_step'], round(d['ms_per_step'] * 120 / $s, 4))"
  done
done
