#!/bin/bash
# GPU-box job: emit_block's four-candidate form for chunks with a per-lane block over 6 / 10
# candidates (tools/patches.py quad_adaptive) vs HEAD, kernel A/B on four contents/workloads.
set -o pipefail
cd "$(dirname "$0")/.."
VARIANTS="head=:;qa6=@quad_adaptive=6;qa10=@quad_adaptive=10" CASES="c2:testsrc c2:natural c2:noise-patches c5:testsrc" bash tools/r04_ab_only.sh r04aj_quad_adaptive
