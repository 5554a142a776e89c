#!/bin/bash
# GPU-box probe: k_encode time per block against the resident pool size and the frames per
# launch (c5 8K vs c2 4K).  Usage: bash tools/c5_pool_job.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/c5pool
for args in "--workload c5 --seg 60" "--workload c5 --seg 15" "--seg 30" "--seg 120"; do
  n=$(echo $args | tr ' ' '_')
  timeout -k 10 200 python bench.py --no-cpu-baseline $args > gpurun_out/c5pool/$n.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c5pool/$n.json')); c=d['config']; print('$args', d['value'], d['kernel_ms_per_step']['encode'], 'ps/block', round(d['kernel_ms_per_step']['encode']*1e9/(c['frames_per_step']*((c['width']+15)//16)*((c['height']+15)//16)*6),2))"
done
