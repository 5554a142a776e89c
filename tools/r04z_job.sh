#!/bin/bash
# GPU-box job: the stuffing tail's stream at the highest priority (tools/patches.py
# stream_prio=tailhigh) on bench.py, c2 and natural.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head th" ROUNDS=4 bash tools/bench_ab.sh r04z_tailhigh &&
LIBS="head th" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04z_tailhigh_nat
