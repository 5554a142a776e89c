#!/bin/bash
# GPU-box job: submit queue depth and tail-stream priority on bench.py (c2, natural):
# head = 3 slots; s2 = 2 slots (tools/patches.py slots2); th3 = 3 slots + the tail stream at
# the highest priority (stream_prio=tailhigh); s2th = 2 slots + tailhigh.
set -o pipefail
cd "$(dirname "$0")/.."
LIBS="head s2 th3 s2th" ROUNDS=3 bash tools/bench_ab.sh r04aa_depth &&
LIBS="head s2 th3 s2th" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04aa_depth_nat
