#!/bin/bash
# GPU-box job: tail co-run probe (bench.py over no-op k_write / k_count_ff variants) and the
# quad-candidate emission A/B on three contents.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head nw nc" ROUNDS=3 bash tools/bench_ab.sh r04p_tail &&
VARIANTS="head=:;q=@quad" CASES="c2:testsrc c2:natural c2:noise-patches" bash tools/r04_ab_only.sh r04p_quad
