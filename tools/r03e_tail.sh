#!/bin/bash
# serial per-kernel durations (variants.py syncs after every submit, so the tail kernels do not
# co-run with k_encode) under rocprofv3 kernel-trace stats, c2 and c1; per-segment client latency
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for w in c2 c1; do
  WL=$w VARIANTS="cur=:" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- \
    python3 tools/variants.py > $O/var_$w.txt 2>&1 || { tail -20 $O/var_$w.txt; exit 1; }
  f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -n 1)
  cp "$f" $O/serial_stats_$w.csv && rm -rf $O/prof_$w
  grep -E "mjg" $O/serial_stats_$w.csv | cut -d, -f1-4 | cut -c1-150
done
timeout -k 10 200 python3 tools/client_latency.py --n 5 > $O/client_latency.txt 2>&1 || { tail -20 $O/client_latency.txt; exit 1; }
cat $O/client_latency.txt
echo done
