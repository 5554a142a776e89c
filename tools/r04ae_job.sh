#!/bin/bash
# GPU-box job: the stuffing tail's wave priority 1 / 2 / 3 (tools/patches.py tail_prio) vs HEAD,
# bench.py on c2, natural, c5.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head tp1 tp2 tp3" ROUNDS=3 bash tools/bench_ab.sh r04ae_tp &&
LIBS="head tp1 tp2 tp3" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04ae_tp_nat &&
LIBS="head tp1 tp2 tp3" ROUNDS=2 ARGS="--workload c5" bash tools/bench_ab.sh r04ae_tp_c5
