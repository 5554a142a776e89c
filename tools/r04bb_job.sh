#!/bin/bash
# GPU-box job: segment lists through k_scale too (-vf scale submits of several segments):
# GPU tests, then HEAD records at the new digest (PMC traffic c2 c1 c4 c5, c2 SQ pass, the
# driver-command profile) and the bench lines with --segments-per-launch (c2, c4, c1).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r04bb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && tail -2 $O/gpu_tests.txt &&
for w in c2 c4 c1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --workload $w --segments-per-launch > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python3 -c "
import json; d = json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['ms_per_step'], json.dumps(d['segments_per_launch']))" || exit 1
done &&
bash tools/pmc_traffic.sh c2 c1 c4 c5 &&
WL=c2 bash tools/gpu_pmc.sh r04bb_sq SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU &&
bash tools/driver_prof.sh r04bb_driver
