#!/bin/bash
# GPU-box job: young waves stop taking units near the end of a launch (tools/patches.py
# young_exit=D) vs HEAD: kernel A/B (outputs compared) and bench.py on c2 / natural.
set -o pipefail
cd "$(dirname "$0")/.."
VARIANTS="head=:;ye1=@young_exit=1;ye2=@young_exit=2;ye4=@young_exit=4" CASES="c2:testsrc c2:natural" bash tools/r04_ab_only.sh r04at_young_exit &&
LIBS="head ye2 ye4" ROUNDS=2 bash tools/bench_ab.sh r04at_bench &&
LIBS="head ye2 ye4" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04at_bench_nat
