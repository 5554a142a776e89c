#!/bin/bash
# GPU-box job: chunk-parallel coder prototype taken per chunk (tools/patches.py cpc_hybrid=X:
# CPC where the per-lane cost model exceeds X rounds) vs HEAD, outputs compared.
set -o pipefail
cd "$(dirname "$0")/.."
VARIANTS="head=:;h2=@cpc_hybrid=2;h3=@cpc_hybrid=3;h4=@cpc_hybrid=4" CASES="c2:testsrc c2:natural c2:noise-patches c5:testsrc" bash tools/r04_ab_only.sh r04r_hybrid
