#!/usr/bin/env python3
"""Bounded check of the fused scale+encode path on a few sizes (GPU box; run under timeout):
prints per case whether the fused output equals the unfused (k_scale + k_encode) output."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from ffmpeg_distributed_amd.encoder import MjpegEncoder  # noqa: E402
from ffmpeg_distributed_amd.testsrc import testsrc2_i420  # noqa: E402

CASES = [(1040, 530, 520, 265), (1200, 700, 1023, 600), (3840, 2160, 1920, 1080)]
for sw, sh, dw, dh in CASES:
    frames = np.stack([testsrc2_i420(sw, sh, t) for t in range(2)])
    t0 = time.time()
    with MjpegEncoder(0, sw, sh, dw, dh, qscale=3, max_batch=2) as e:  # k_scale + k_encode
        ref = e.encode(frames)
    print(f"{sw}x{sh}->{dw}x{dh} unfused {time.time() - t0:.2f}s", flush=True)
    t0 = time.time()
    with MjpegEncoder(0, sw, sh, dw, dh, qscale=3, max_batch=2, fused=True) as e:
        got = e.encode(frames)
    print(f"{sw}x{sh}->{dw}x{dh} fused {time.time() - t0:.2f}s equal={got == ref}", flush=True)
