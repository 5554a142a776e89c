#!/bin/bash
# GPU-box job: bench.py (the driver's metric, tail co-running) A/B over variant libraries,
# interleaved rounds.  Usage: LIBS="name ..." ROUNDS=3 ARGS="--workload c2" bash tools/bench_ab.sh TAG
# (name: ffmpeg_distributed_amd/libmjgpu_v_<name>.so; "head" = the in-tree libmjgpu.so)
set -o pipefail
TAG=$1
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 ${ROUNDS:-3}); do
  for n in $LIBS; do
    if [ "$n" = head ]; then unset MJG_LIBRARY; else export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_$n.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e ${ARGS:-} > $O/b_${n}_$r.json 2> $O/b_${n}_$r.err || { tail -5 $O/b_${n}_$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$O/b_${n}_$r.json'))
print('$n', $r, d['value'], d['ms_per_step'], round(d['kernel_ms_per_step']['encode'], 4))"
  done
done
echo done
