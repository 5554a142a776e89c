#!/usr/bin/env python3
"""Perf experiment: build k_encode ablation variants (-DMJG_ABLATE=N) and time each on the
same resident 4K frames in one process (interleaved rounds).  Outputs are NOT valid for
N>0; only kernel times matter."""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "ffmpeg_distributed_amd", "csrc")


def build(n, extra=()):
    out = os.path.join(ROOT, "ffmpeg_distributed_amd", f"libmjgpu_ablate{n}.so")
    if "--build" in sys.argv or not os.path.exists(out):
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize", "-fPIC", "-shared",
               f"-DMJG_ABLATE={n}", "-I", os.path.join(ROOT, "include"), "-o", out,
               os.path.join(CSRC, "api.hip"), os.path.join(CSRC, "sws_filter.cpp"), *extra]
        subprocess.run(cmd, check=True, cwd=CSRC)
    return out


def main():
    variants = [int(x) for x in os.environ.get("ABLATE", "0,1,2,3").split(",")]
    libs = {n: build(n) for n in variants}
    if "--build-only" in sys.argv:
        return
    import torch
    from ffmpeg_distributed_amd import _lib
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch
    W, H, N = 3840, 2160, 120
    dev = torch.device("cuda", 0)
    fb = W * H * 3 // 2
    pool = torch.empty((N, fb), dtype=torch.uint8, device=dev)
    for i in range(0, N, 20):
        pool[i:i + 20] = testsrc2_i420_torch(W, H, i, 20, dev)
    torch.cuda.synchronize()
    encs = {}
    for n, path in libs.items():
        _lib._lib = None
        _lib.LIB_PATH = path
        from ffmpeg_distributed_amd.encoder import MjpegEncoder
        encs[n] = MjpegEncoder(0, W, H, qscale=5, max_batch=N, timing=True)
    res = {n: [] for n in libs}
    for rnd in range(6):
        for n, e in encs.items():
            e.kernel_times(reset=True)
            for _ in range(3):
                e.submit(device_ptr=pool.data_ptr(), nframes=N)
                e.sync()
            res[n].append(e.kernel_times()[0]["encode"])
    for n in libs:
        v = sorted(res[n])
        print(f"ABLATE={n}: k_encode median {v[len(v)//2]:.4f} ms  min {v[0]:.4f} ms per {N} frames")


if __name__ == "__main__":
    main()
