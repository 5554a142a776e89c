#!/bin/bash
# GPU-box job: bench.py --segments-per-launch on c1 (-huffman optimal, 250-frame segments, a
# pool of four segments), c5 and the noise-patches content.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04bc
mkdir -p $O
for a in "--workload c1 --pool 1000" "--workload c5" "--content noise-patches"; do
  t=$(echo $a | tr -d ' -')
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --segments-per-launch $a > $O/bench_$t.json 2> $O/bench_$t.err || exit 1
  python3 -c "
import json; d = json.load(open('$O/bench_$t.json')); print('$t', d['value'], d['ms_per_step'], json.dumps(d['segments_per_launch']))" || exit 1
done
