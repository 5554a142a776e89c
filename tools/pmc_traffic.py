#!/usr/bin/env python3
"""Turn the tools/pmc_traffic.sh counter CSVs into profiles/pmc_encode_4k_q5.json:
per-launch HBM bytes of k_encode = FETCH_SIZE x (calibrated bytes per unit) + WRITE_SIZE x 1024
(WRITE_SIZE is exact for streaming stores per MI355X_MICROARCH.md; the chunk-slot stores
are coalesced 4-byte-per-lane runs, noted as uncalibrated)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402

out, calib_bytes = sys.argv[1], int(sys.argv[2])
cal = load([os.path.join(out, "calib")])
cal_fetch = sum(v["FETCH_SIZE"] for v in cal.values())  # one kernel
per_unit = calib_bytes / cal_fetch
def _enc(d):  # the k_encode instantiation (template arguments in the name)
    return next(v for k, v in d.items() if "k_encode" in k)


fetch = _enc(load([os.path.join(out, "fetch")]))["FETCH_SIZE"]
write = _enc(load([os.path.join(out, "write")]))["WRITE_SIZE"]
frames, W, H = 120, 3840, 2160
res = {
    "kernel": "mjg::k_encode",
    "workload": {"frames_per_launch": frames, "width": W, "height": H, "qscale": 5,
                 "input": "testsrc2-like yuv420p (tools/pmc_workload.py)"},
    "calibration": {"kernel": "tools/calib_fetch.hip (8 B/lane coalesced reads)",
                    "bytes": calib_bytes, "FETCH_SIZE": cal_fetch, "bytes_per_unit": per_unit},
    "FETCH_SIZE": fetch, "WRITE_SIZE": write,
    "read_bytes_per_launch": fetch * per_unit,
    "write_bytes_per_launch": write * 1024,
    "hbm_bytes_per_launch": fetch * per_unit + write * 1024,
    "input_plane_bytes_per_launch": frames * W * H * 3 // 2,
}
res["read_over_input"] = res["read_bytes_per_launch"] / res["input_plane_bytes_per_launch"]
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                    "pmc_encode_4k_q5.json")
for pth in (path, os.path.join(out, "pmc_encode_4k_q5.json")):  # gpurun_out/ travels back
    with open(pth, "w") as f:
        json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
