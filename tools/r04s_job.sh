#!/bin/bash
# GPU-box job: stream priorities (tools/patches.py stream_prio) A/B on bench.py, c2 testsrc + natural.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head spt spb" ROUNDS=4 bash tools/bench_ab.sh r04s_prio &&
LIBS="head spt spb" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04s_prio_nat
