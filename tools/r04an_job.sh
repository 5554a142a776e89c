#!/bin/bash
# GPU-box job: what costs c1 / c4 against round 3: the counting pass's grid (cg =
# count_grid_full), the tail's wave priority (tp0 = tail_prio=0), both (cgtp0); bench.py.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head cg tp0 cgtp0" ROUNDS=3 ARGS="--workload c1" bash tools/bench_ab.sh r04an_c1 &&
LIBS="head tp0" ROUNDS=3 ARGS="--workload c4" bash tools/bench_ab.sh r04an_c4
