#!/bin/bash
# GPU-box job: GPU tests at HEAD (two slots, tail stream at the highest priority), then
# bench.py HEAD vs the tail stream at default priority (tools/patches.py stream_prio=normal)
# on c2, natural, c5 and c4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r04ab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ab/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r04ab/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04ab/gpu_tests.txt
LIBS="head tn" ROUNDS=4 bash tools/bench_ab.sh r04ab_prio &&
LIBS="head tn" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04ab_prio_nat &&
LIBS="head tn" ROUNDS=2 ARGS="--workload c5" bash tools/bench_ab.sh r04ab_prio_c5 &&
LIBS="head tn" ROUNDS=2 ARGS="--workload c4" bash tools/bench_ab.sh r04ab_prio_c4
