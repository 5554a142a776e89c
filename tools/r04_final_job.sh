#!/bin/bash
# GPU-box job, round-4 HEAD record: GPU tests, per-kernel HBM traffic (every workload) and an SQ
# pass (c2) on the HEAD library, the driver's command under rocprofv3, then the other workloads'
# and contents' bench lines.  Usage: bash tools/r04_final_job.sh TAG
set -o pipefail
TAG=${1:-r04z}
cd "$(dirname "$0")/.."
bash tools/r04_job.sh $TAG || exit 1
O=gpurun_out/$TAG
for w in c1 c4 c5; do
  timeout -k 10 200 python bench.py --workload $w --no-cpu-baseline --no-e2e > $O/bench_$w.json 2> $O/bench_$w.err || { tail -5 $O/bench_$w.err; exit 1; }
  cut -c1-200 $O/bench_$w.json
done
for c in natural noise-patches; do
  timeout -k 10 200 python bench.py --content $c --no-cpu-baseline --no-e2e > $O/bench_c2_$c.json 2> $O/bench_c2_$c.err || { tail -5 $O/bench_c2_$c.err; exit 1; }
  cut -c1-200 $O/bench_c2_$c.json
done
echo final-done
