#!/usr/bin/env python3
"""Perf experiment: k_encode time per 120 4K frames for one MJG_ENC_WG_PER_CU setting (run
once per setting; the env var is read at mjg_open)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch
    W, H, N = 3840, 2160, 120
    dev = torch.device("cuda", 0)
    pool = torch.empty((N, W * H * 3 // 2), dtype=torch.uint8, device=dev)
    for i in range(0, N, 20):
        pool[i:i + 20] = testsrc2_i420_torch(W, H, i, 20, dev)
    torch.cuda.synchronize()
    e = MjpegEncoder(0, W, H, qscale=5, max_batch=N, timing=True)
    for _ in range(3):
        e.submit(device_ptr=pool.data_ptr(), nframes=N)
        e.sync()
    e.kernel_times(reset=True)
    for _ in range(20):
        e.submit(device_ptr=pool.data_ptr(), nframes=N)
        e.sync()
    print(f"MJG_ENC_WG_PER_CU={os.environ.get('MJG_ENC_WG_PER_CU', 'default')}: "
          f"k_encode {e.kernel_times()[0]['encode']:.4f} ms per {N} frames", flush=True)


if __name__ == "__main__":
    main()
