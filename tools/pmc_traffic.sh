#!/bin/bash
# GPU-box job: HBM traffic per launch of every encoder kernel from rocprofv3 PMC counters.
#   calibration: FETCH_SIZE / WRITE_SIZE of tools/calib_fetch.hip (known byte counts at the
#                access widths the encoder uses: 8 B and 4 B reads, 4 B and 1 B writes)
#   per workload (bench.py --workload): one FETCH_SIZE pass and one WRITE_SIZE pass (the two
#   cannot share a pass: FETCH_SIZE takes 3 TCC counters, WRITE_SIZE 2)
# then tools/pmc_traffic.py writes profiles/pmc_<workload>.json.
# Usage: bash tools/pmc_traffic.sh [WORKLOAD ...]   (default: c2 c1 c4 c5)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
WLS=${@:-c2 c1 c4 c5}
CAL=1565523968
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o $OUT/calib_bin tools/calib_fetch.hip || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $OUT/calib_$c -o run --output-format csv -- $OUT/calib_bin $CAL > $OUT/calib_$c.log 2>&1 || exit 1
done
for w in $WLS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --kernel-include-regex 'mjg::' --pmc $c -d $OUT/${w}_$c -o run --output-format csv -- python3 tools/pmc_workload.py --workload $w > $OUT/${w}_$c.log 2>&1 || exit 1
  done
done
python3 tools/pmc_traffic.py $OUT $CAL $WLS && rm -f $OUT/calib_bin && echo done
