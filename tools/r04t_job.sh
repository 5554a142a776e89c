#!/bin/bash
# GPU-box job: short-block pack fast path (tools/patches.py short_pack) vs HEAD, outputs compared.
set -o pipefail
cd "$(dirname "$0")/.."
VARIANTS="head=:;sp=@short_pack;sp64=@short_pack64" CASES="c2:testsrc c2:natural c2:noise-patches c5:testsrc c4:testsrc" bash tools/r04_ab_only.sh r04t_short_pack
