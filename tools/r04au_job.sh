#!/bin/bash
# GPU-box job: young waves pull dynamic units of S chunks (tools/patches.py young_half=S;
# S = 12 is HEAD's schedule on chunk counters) vs HEAD: kernel A/B (outputs compared) and
# bench.py on c2 / natural.
set -o pipefail
cd "$(dirname "$0")/.."
VARIANTS="head=:;yh12=@young_half=12;yh8=@young_half=8;yh6=@young_half=6;yh4=@young_half=4" CASES="c2:testsrc c2:natural c5:testsrc" bash tools/r04_ab_only.sh r04au_young_half &&
LIBS="head yh12 yh6 yh4" ROUNDS=3 bash tools/bench_ab.sh r04au_bench &&
LIBS="head yh6 yh4" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04au_bench_nat &&
LIBS="head yh6 yh4" ROUNDS=2 ARGS="--workload c5" bash tools/bench_ab.sh r04au_bench_c5
