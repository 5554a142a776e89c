#!/bin/bash
# GPU-box job: chunk-parallel coder prototype (tools/patches.py cpc) vs HEAD, outputs compared.
set -o pipefail
cd "$(dirname "$0")/.."
VARIANTS="head=:;cpc=@cpc" CASES="c2:testsrc c2:natural c2:noise-patches c5:testsrc" bash tools/r04_ab_only.sh ${TAG:-r04q_cpc}
