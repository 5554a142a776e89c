#!/bin/bash
# GPU-box job: mjg_submit_segments (several segments per k_encode launch): the driver's bench
# line (with its segments_per_launch leg), and bench.py A/B of this build against the previous
# HEAD library (one segment per submit: the SegList argument's cost).  GPU tests: r04ax run 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04ax
mkdir -p $O
timeout -k 10 300 python bench.py --segments-per-launch > $O/bench.json 2> $O/bench.err && python3 -c "
import json; d = json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], json.dumps(d['segments_per_launch']))" &&
LIBS="head prev" ROUNDS=3 bash tools/bench_ab.sh r04ax_ab_prev &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --content natural --segments-per-launch > $O/bench_nat.json 2> $O/bench_nat.err && python3 -c "
import json; d = json.load(open('$O/bench_nat.json')); print('natural', d['value'], d['ms_per_step'], json.dumps(d['segments_per_launch']))" &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --workload c5 --segments-per-launch > $O/bench_c5.json 2> $O/bench_c5.err && python3 -c "
import json; d = json.load(open('$O/bench_c5.json')); print('c5', d['value'], d['ms_per_step'], json.dumps(d['segments_per_launch']))"
