#!/bin/bash
# GPU-box job: the stuffing tail's waves at wave priority 3 (tools/patches.py tail_prio) vs HEAD:
# bench.py A/B (c2, natural, c5, c4) and the per-step timeline of both (rocprofv3 kernel trace).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
LIBS="head tp" ROUNDS=4 bash tools/bench_ab.sh r04ad_tp &&
LIBS="head tp" ROUNDS=2 ARGS="--content natural" bash tools/bench_ab.sh r04ad_tp_nat &&
LIBS="head tp" ROUNDS=2 ARGS="--workload c5" bash tools/bench_ab.sh r04ad_tp_c5 &&
LIBS="head tp" ROUNDS=2 ARGS="--workload c4" bash tools/bench_ab.sh r04ad_tp_c4 || exit 1
O=gpurun_out/r04ad
mkdir -p $O
for v in head tp; do
  if [ $v = head ]; then unset MJG_LIBRARY; else export MJG_LIBRARY=$PWD/ffmpeg_distributed_amd/libmjgpu_v_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --kernel-include-regex 'mjg::' -d $O/t_$v -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --no-e2e --steps 20 --warmup 3 > $O/b_$v.json 2> $O/e_$v.log || exit 1
  f=$(find $O/t_$v -name "*kernel_trace.csv" | head -n 1)
  cp "$f" $O/trace_$v.csv && rm -rf $O/t_$v
  echo "== $v"; python3 tools/timeline.py $O/trace_$v.csv
done
