#!/bin/bash
# serial per-kernel durations of two builds (variants.py, one variant per rocprofv3 run)
#   Usage: bash tools/r03e_tailprof.sh TAG "name1 name2" [workload]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
w=${3:-c2}
for v in $2; do
  WL=$w VARIANTS="$v=:" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- \
    python3 tools/variants.py > $O/var_$v.txt 2>&1 || { tail -20 $O/var_$v.txt; exit 1; }
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -n 1)
  cp "$f" $O/stats_${w}_$v.csv && rm -rf $O/prof_$v
  echo "== $v"; python3 -c "
import csv
for r in csv.DictReader(open('$O/stats_${w}_$v.csv')):
    if 'mjg' in r['Name']: print(f\"{r['Name'][:40]:40s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1000:9.2f} min_us={float(r['MinNs'])/1000:9.2f}\")
"
done
echo done
