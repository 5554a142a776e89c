#!/bin/bash
# GPU-box job: k_encode's persistent grid at 3 workgroups per CU (tools/patches.py
# enc_grid_per_cu=3) vs HEAD's 4, bench.py c2, natural, c5.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head g3" ROUNDS=3 bash tools/bench_ab.sh r04as_g3 &&
LIBS="head g3" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04as_g3_nat &&
LIBS="head g3" ROUNDS=2 ARGS="--workload c5" bash tools/bench_ab.sh r04as_g3_c5
