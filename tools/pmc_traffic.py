#!/usr/bin/env python3
"""Turn the tools/pmc_traffic.sh counter CSVs into profiles/pmc_<workload>.json: per kernel,
HBM bytes per launch = FETCH_SIZE x (calibrated bytes per unit for the kernel's read width)
+ WRITE_SIZE x (calibrated bytes per unit for its write width).

Calibration (tools/calib_fetch.hip) reads / writes a 1.5 GB buffer (past the 256 MiB L3)
with 8 B, 4 B per lane loads and 4 B, 1 B per lane stores; each kernel is assigned the
width of its dominant access (KERNEL_WIDTH).  Usage: pmc_traffic.py OUTDIR CAL_BYTES WL..."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from pmc_summary import load, load_totals  # noqa: E402

# dominant (read, write) access width of each kernel, bytes per lane
KERNEL_WIDTH = {
    "k_encode": (8, 4),       # 8-byte pixel row loads, slot words
    "k_scale": (8, 1),        # 16-byte window loads (4 and 8 B reads calibrate alike), byte stores
    "k_emit_syms": (4, 4),    # symbol record words, slot words
    "k_count_ff": (4, 4),     # slot words
    "k_write": (4, 1),        # slot words in, stuffed bytes out
}


LAUNCHES = 3  # tools/pmc_workload.py --launches default


def _width(name):
    for k, v in KERNEL_WIDTH.items():
        if k in name:
            return v
    return (4, 4)


def main():
    out, cal_bytes, wls = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    calf = load([os.path.join(out, "calib_FETCH_SIZE")])
    calw = load([os.path.join(out, "calib_WRITE_SIZE")])
    per_read = {8: cal_bytes / calf["k_calib_read8"]["FETCH_SIZE"],
                4: cal_bytes / calf["k_calib_read4"]["FETCH_SIZE"]}
    per_write = {4: cal_bytes / calw["k_calib_write4"]["WRITE_SIZE"],
                 1: cal_bytes / calw["k_calib_write1"]["WRITE_SIZE"]}
    import bench
    from ffmpeg_distributed_amd import build as B
    if os.environ.get("MJG_LIBRARY"):  # a variant library (an A/B record): its file's digest
        import hashlib
        with open(os.environ["MJG_LIBRARY"], "rb") as f:
            digest = "file:" + hashlib.sha256(f.read()).hexdigest()
    else:
        if not B.check():  # the counters describe the library the workload loaded: it must be HEAD's
            raise SystemExit("libmjgpu.so is stale against its sources: rebuild before counting")
        digest = B.source_digest()
    for wl in wls:
        W, H, DW, DH, Q, SEG, FULL, HUFF, text = bench.WORKLOADS[wl]
        # per launch = per submit of one segment (the workload syncs LAUNCHES submits); a
        # kernel launched per plane (k_scale: Y, U, V) sums its dispatches of one submit
        fetch = load_totals([os.path.join(out, f"{wl}_FETCH_SIZE")])
        write = load_totals([os.path.join(out, f"{wl}_WRITE_SIZE")])
        kernels = {}
        for name in sorted(set(fetch) | set(write)):
            rw, ww = _width(name)
            f = fetch.get(name, {}).get("FETCH_SIZE", 0.0) / LAUNCHES
            wv = write.get(name, {}).get("WRITE_SIZE", 0.0) / LAUNCHES
            nd = max(fetch.get(name, {}).get("dispatches", 0), write.get(name, {}).get("dispatches", 0))
            kernels[name] = {"FETCH_SIZE": f, "WRITE_SIZE": wv, "read_width": rw, "write_width": ww,
                             "dispatches_per_launch": nd / LAUNCHES,
                             "read_bytes_per_launch": f * per_read[rw],
                             "write_bytes_per_launch": wv * per_write[ww],
                             "hbm_bytes_per_launch": f * per_read[rw] + wv * per_write[ww]}
        in_bytes = SEG * (W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2))
        res = {"library_digest": digest,  # build.source_digest() of the counted library
               "workload": {"name": wl, "text": text, "frames_per_launch": SEG, "width": W, "height": H,
                            "dst_width": DW, "dst_height": DH, "qscale": Q, "huffman": HUFF,
                            "input": "testsrc2-like (tools/pmc_workload.py)"},
               "calibration": {"kernel": "tools/calib_fetch.hip", "bytes": cal_bytes,
                               "fetch_bytes_per_unit": per_read, "write_bytes_per_unit": per_write},
               "input_plane_bytes_per_launch": in_bytes,
               "kernels": kernels}
        dests = [os.path.join(out, f"pmc_{wl}.json")]
        if not os.environ.get("MJG_LIBRARY"):
            dests.append(os.path.join(ROOT, "profiles", f"pmc_{wl}.json"))
        for pth in dests:
            with open(pth, "w") as fo:
                json.dump(res, fo, indent=1)
        print(wl, json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 1) for k, v in kernels.items()}))


if __name__ == "__main__":
    main()
