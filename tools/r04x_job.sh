#!/bin/bash
# GPU-box job: HEAD validation (GPU tests, PMC traffic, SQ, driver profile; bench lines), then
# the forced two-op screen deposit A/B (tools/patches.py deposit_asm).
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/r04_job.sh r04x && bash tools/r04_bench_job.sh r04y &&
VARIANTS="head=:;da=@deposit_asm" CASES="c2:testsrc c2:natural c5:testsrc" bash tools/r04_ab_only.sh r04x_deposit
