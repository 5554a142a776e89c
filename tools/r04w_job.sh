#!/bin/bash
# GPU-box job: bench.py (driver's metric) HEAD vs HEAD without pack_chunk_short (nsp) vs the
# pack64 second fast path (p64); then the kernel A/B of p64.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head nsp p64" ROUNDS=4 bash tools/bench_ab.sh r04w_bench &&
VARIANTS="head=:;p64=@pack64" CASES="c2:testsrc c2:natural c2:noise-patches c5:testsrc" bash tools/r04_ab_only.sh r04w_p64
