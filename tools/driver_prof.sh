#!/bin/bash
# GPU-box job: rocprofv3 kernel-trace stats of the exact command the driver runs for
# BENCH (python3 bench.py --gpus 1 --steps 20 --warmup 5), plus a host probe (cores, CPU
# model, cgroup CPU quota, NUMA node of the GPU).  Usage: bash tools/driver_prof.sh TAG
set -o pipefail
TAG=${1:-r02}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p $O
{
  echo "nproc $(nproc)"
  echo "affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
  echo "cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
  lscpu | grep -E "Model name|^CPU\(s\)|Thread|Socket|NUMA" || true
  for d in /sys/class/drm/card*/device/numa_node; do echo "$d $(cat $d)"; done
} > $O/host.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof.err || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1)
cp "$f" $O/kernel_stats.csv && rm -rf $O/prof
grep -E "mjg" $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
cat $O/prof_bench.json
echo done
