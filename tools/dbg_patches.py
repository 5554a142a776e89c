#!/usr/bin/env python3
"""Debug: the optimal-Huffman patches case: GPU bytes + coefficients vs the oracle."""
import os
import sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_parity as t  # noqa: E402
import oracle  # noqa: E402
from ffmpeg_distributed_amd.encoder import MjpegEncoder, split_i420  # noqa: E402

w, h, q, full = 200, 72, 2, False
frames = t.rand_frames(w, h, 3, seed=w * 17 + h + q, kind="patches")
os.makedirs(os.path.join(ROOT, "gpurun_out", "dbg"), exist_ok=True)
with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=4, huffman="optimal", debug_coefs=True) as enc:
    enc.submit(frames)
    enc.sync()
    got = enc.fetch_frames() if hasattr(enc, "fetch_frames") else None
    coefs = [enc.debug_coefs(i) for i in range(3)]
with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=4, huffman="optimal") as enc:
    got = enc.encode(frames)
ref = t.oracle_frames(frames, w, h, q, full, huffman="optimal")
for i in range(3):
    open(os.path.join(ROOT, "gpurun_out", "dbg", f"gpu{i}.jpg"), "wb").write(got[i])
    open(os.path.join(ROOT, "gpurun_out", "dbg", f"ref{i}.jpg"), "wb").write(ref[i])
    np.save(os.path.join(ROOT, "gpurun_out", "dbg", f"coef{i}.npy"), coefs[i])
print("saved")
