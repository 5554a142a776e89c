#!/bin/bash
# GPU-box job: the exact command the driver runs for BENCH (python3 bench.py --gpus 1 --steps 20
# --warmup 5) under rocprofv3 --kernel-trace --stats: the kernel stats CSV, the kernel trace CSV
# and tools/timeline.py's per-step summary of it (timed launches between bench.py's trace
# markers, GPU-busy union per step vs ms_per_step, isolated launches); plus a host probe (cores,
# CPU model, cgroup CPU quota, NUMA node of the GPU).  Usage: bash tools/driver_prof.sh TAG [bench args]
set -o pipefail
TAG=${1:-r05}
shift
ARGS=${@:---gpus 1 --steps 20 --warmup 5}
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
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py $ARGS > $O/prof_bench.json 2> $O/prof.err || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -n 1)
t=$(find $O/prof -name "*kernel_trace.csv" | head -n 1)
cp "$f" $O/kernel_stats.csv && cp "$t" $O/kernel_trace.csv && rm -rf $O/prof
python3 tools/timeline.py $O/kernel_trace.csv $O/prof_bench.json > $O/timeline.txt 2>&1
# keep the trace small enough to come back (gpurun merges <= 64 MiB): the header, mjg kernels, markers
{ head -n 1 $O/kernel_trace.csv; grep -E "mjg::|spin_kernel" $O/kernel_trace.csv; } > $O/kernel_trace.small.csv && mv $O/kernel_trace.small.csv $O/kernel_trace.csv
cat $O/timeline.txt
grep -E "mjg" $O/kernel_stats.csv | cut -d, -f1-4 | cut -c1-140
echo done
