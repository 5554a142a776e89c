#!/bin/bash
# GPU-box job: HEAD vs the round-3 build (16deb57) on bench.py, every BASELINE workload line,
# same box, interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head r03" ROUNDS=3 bash tools/bench_ab.sh r04am_c2 &&
LIBS="head r03" ROUNDS=2 ARGS="--workload c1" bash tools/bench_ab.sh r04am_c1 &&
LIBS="head r03" ROUNDS=2 ARGS="--workload c4" bash tools/bench_ab.sh r04am_c4 &&
LIBS="head r03" ROUNDS=2 ARGS="--workload c5" bash tools/bench_ab.sh r04am_c5 &&
LIBS="head r03" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04am_nat
