#!/usr/bin/env python3
"""Small fixed workload for rocprofv3 PMC passes: 4K testsrc2-like yuv420p, q=5,
`--launches` launches of `--frames` resident frames through k_encode and friends."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=120)
    p.add_argument("--launches", type=int, default=3)
    p.add_argument("--w", type=int, default=3840)
    p.add_argument("--h", type=int, default=2160)
    p.add_argument("--q", type=int, default=5)
    p.add_argument("--dw", type=int, default=None, help="scaled width (-vf scale)")
    p.add_argument("--dh", type=int, default=None)
    a = p.parse_args()
    import torch
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch
    dev = torch.device("cuda", 0)
    fb = a.w * a.h + 2 * ((a.w + 1) // 2) * ((a.h + 1) // 2)
    pool = torch.empty((a.frames, fb), dtype=torch.uint8, device=dev)
    for i in range(0, a.frames, 20):
        k = min(20, a.frames - i)
        pool[i:i + k] = testsrc2_i420_torch(a.w, a.h, i, k, dev)
    torch.cuda.synchronize()
    enc = MjpegEncoder(0, a.w, a.h, dst_w=a.dw, dst_h=a.dh, qscale=a.q, max_batch=a.frames)
    tot = 0
    for _ in range(a.launches):
        enc.submit(device_ptr=pool.data_ptr(), nframes=a.frames)
        tot += int(enc.sync().sum())
    print(f"frames/launch {a.frames} launches {a.launches} mean_jpeg {tot / a.launches / a.frames:.1f}")
    enc.close()


if __name__ == "__main__":
    main()
