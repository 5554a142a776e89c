#!/bin/bash
# A/B of two libmjgpu builds on the default bench (interleaved runs).  Usage:
#   bash tools/ab_bench.sh OLD.so [bench args...]   (NEW = the in-tree build)
set -o pipefail
cd "$(dirname "$0")/.."
OLD=$1; shift
mkdir -p gpurun_out/ab
for i in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export MJG_LIBRARY=$OLD; else unset MJG_LIBRARY; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab/$v$i.json 2>>gpurun_out/ab/err.log || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/$v$i.json')); print('$v$i', d['value'], d['kernel_ms_per_step'])"
  done
done
