#!/bin/bash
# GPU-box job: HBM traffic of k_encode per launch from rocprofv3 PMC counters.
#   pass 1: FETCH_SIZE of a calibration kernel reading a known byte count with the
#           same 8-byte-per-lane width k_encode uses  -> bytes per FETCH_SIZE unit
#   pass 2: FETCH_SIZE of the bench workload (k_encode)
#   pass 3: WRITE_SIZE of the bench workload
# then tools/pmc_traffic.py writes profiles/pmc_encode_4k_q5.json.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o $OUT/calib_bin tools/calib_fetch.hip || exit 1
timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o run --output-format csv -- $OUT/calib_bin 1565523968 > $OUT/calib.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-include-regex 'mjg::' --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/pmc_workload.py > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-include-regex 'mjg::' --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/pmc_workload.py > $OUT/write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $OUT 1565523968 && rm -f $OUT/calib_bin && echo done
