#!/bin/bash
# GPU-box job: the round's HEAD records.  GPU tests, the driver's bench command, its rocprofv3
# kernel trace + stats and timeline (tools/driver_prof.sh), PMC HBM traffic per kernel
# (tools/pmc_traffic.sh, before the bench lines that report it), the other BASELINE workloads and
# contents, and an SQ pass of c2 / c1 / c4 (SKIP_PMC=1 / SKIP_SQ=1 leave those passes out).
# Usage: bash tools/head_job.sh TAG
set -o pipefail
TAG=${1:-head}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
# PMC traffic first: the bench lines report it only when profiles/pmc_<workload>.json was counted
# on the library they load (SKIP_PMC=1 when the committed files already carry this digest)
if [ -z "$SKIP_PMC" ]; then
  timeout -k 10 900 bash tools/pmc_traffic.sh > $O/pmc_traffic.log 2>&1 || { tail -5 $O/pmc_traffic.log; exit 1; }
  cp profiles/pmc_c*.json $O/  # pmc_traffic.py writes profiles/ on the box: bring the files back
fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
bash tools/driver_prof.sh ${TAG}_prof > $O/driver_prof.log 2>&1 || exit 1
for w in c1 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
done
for c in natural noise-patches; do
  timeout -k 10 300 python bench.py --content $c --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_$c.json 2> $O/bench_c2_$c.err || exit 1
done
SQ="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY"
SQ2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_BRANCH"
[ -n "$SKIP_SQ" ] && { echo done; exit 0; }
for w in c2 c1 c4; do
  WL=$w timeout -k 10 300 bash tools/gpu_pmc.sh ${TAG}_sq_$w "$SQ" "$SQ2" > $O/sq_$w.log 2>&1 || { tail -5 $O/sq_$w.log; exit 1; }
done
echo done
