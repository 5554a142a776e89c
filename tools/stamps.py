#!/usr/bin/env python3
"""Per-wave start/end clocks of k_encode (diagnostic build, -DMJG_STAMPS): how evenly the
persistent waves finish.  Builds ffmpeg_distributed_amd/libmjgpu_v_stamps.so, encodes
120 4K testsrc2 frames three times, prints the spread of the last launch."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "ffmpeg_distributed_amd", "csrc")
SO = os.path.join(ROOT, "ffmpeg_distributed_amd", "libmjgpu_v_stamps.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                "-DMJG_STAMPS", *sys.argv[1:], "-I", os.path.join(ROOT, "include"), "-o", SO,
                os.path.join(CSRC, "api.hip"), os.path.join(CSRC, "sws_filter.cpp")], check=True)
import torch  # noqa: E402
from ffmpeg_distributed_amd import _lib  # noqa: E402
_lib.LIB_PATH = SO
from ffmpeg_distributed_amd.encoder import MjpegEncoder  # noqa: E402
from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch  # noqa: E402

W, H, N = 3840, 2160, 120
dev = torch.device("cuda", 0)
pool = torch.empty((N, W * H * 3 // 2), dtype=torch.uint8, device=dev)
for i in range(0, N, 20):
    pool[i:i + 20] = testsrc2_i420_torch(W, H, i, 20, dev)
torch.cuda.synchronize()
enc = MjpegEncoder(0, W, H, qscale=5, max_batch=N, timing=True)
for _ in range(3):
    enc.submit(device_ptr=pool.data_ptr(), nframes=N)
    enc.sync()
kt, _ = enc.kernel_times()
L = _lib.load()
L.mjg_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
n = 8192
st = np.zeros(2 * n, np.uint64)
_lib.check(L.mjg_debug_stamps(enc._h, st.ctypes.data, st.size))
st = st.reshape(n, 2).astype(np.int64)
st = st[st[:, 1] > 0]
t0 = st[:, 0].min()
start, end = st[:, 0] - t0, st[:, 1] - t0
dur = end - start
span = end.max()
print(f"waves {len(st)}  k_encode {kt['encode']:.4f} ms  span {span} clk")
for name, v in (("start", start), ("end", end), ("dur", dur)):
    q = np.percentile(v, [0, 10, 50, 90, 99, 100])
    print(f"{name:5s} " + " ".join(f"{x:9.0f}" for x in q) + f"   mean {v.mean():.0f}")
print(f"mean busy fraction of span: {dur.mean() / span:.3f}")
hist = np.histogram(end / span, bins=10, range=(0, 1))[0]
print("end-time histogram (tenths of span):", hist.tolist())
