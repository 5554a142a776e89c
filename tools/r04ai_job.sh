#!/bin/bash
# GPU-box job: GPU tests, then the tail's wave priority raised only for light streams (HEAD)
# vs never (p0: tail_prio=0) vs always (pa: tail_prio_always); bench.py c2, c5, natural, noise.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r04ai
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04ai/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r04ai/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04ai/gpu_tests.txt
LIBS="head p0 pa" ROUNDS=3 bash tools/bench_ab.sh r04ai_c2 &&
LIBS="head p0 pa" ROUNDS=2 ARGS="--workload c5" bash tools/bench_ab.sh r04ai_c5 &&
LIBS="head p0 pa" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04ai_nat &&
LIBS="head p0 pa" ROUNDS=2 ARGS="--content noise-patches" bash tools/bench_ab.sh r04ai_noise
