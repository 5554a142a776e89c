#!/usr/bin/env python3
"""Locate where the fused scale+encode output differs from the unfused one (GPU box): decodes
both JPEGs and prints the MCU rows / columns whose pixels differ."""
import io
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

from ffmpeg_distributed_amd.encoder import MjpegEncoder  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_parity import rand_frames  # noqa: E402

sw, sh, dw, dh, q, full, kind, n, huff = [eval(x) for x in sys.argv[1:10]]
frames = rand_frames(sw, sh, n, seed=sw + dh + q, kind=kind)
with MjpegEncoder(0, sw, sh, dw, dh, qscale=q, full_range=full, max_batch=2, huffman=huff, fused=True) as e:
    got = e.encode(frames)
with MjpegEncoder(0, sw, sh, dw, dh, qscale=q, full_range=full, max_batch=2, huffman=huff) as e:  # k_scale + k_encode
    ref = e.encode(frames)
for i in range(n):
    a = np.asarray(Image.open(io.BytesIO(got[i])).convert("YCbCr")).astype(int)
    b = np.asarray(Image.open(io.BytesIO(ref[i])).convert("YCbCr")).astype(int)
    d = np.abs(a - b).max(axis=2)
    ys, xs = np.nonzero(d)
    print(f"frame {i}: equal={got[i] == ref[i]} sizes {len(got[i])} {len(ref[i])} diff pixels {len(ys)}")
    if len(ys):
        mr = sorted(set((ys // 16).tolist()))
        mc = sorted(set((xs // 16).tolist()))
        print("  MCU rows", mr[:20], "MCU cols", mc[:40])
