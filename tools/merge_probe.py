#!/usr/bin/env python3
"""Submit patterns of the c2 workload in one process, each bracketed by a marker kernel
(torch.cuda._sleep: "spin_kernel" in a rocprofv3 kernel trace), to compare how launches of one
or two segments pipeline (merged launches):
  explicit2  mjg_submit_segments of two segments per submit (context of 2 x 120 frames)
  hold       one mjg_submit per segment, library merging, a lone job held even on an idle GPU
  idle       one mjg_submit per segment, library merging, a lone job launched on an idle GPU
  single     one mjg_submit per segment, no merging
Each pattern runs SEGS segments after a 4-segment warmup, synced before and after; prints
frames/s per pattern (rounds interleaved).  usage: merge_probe.py [SEGS] [ROUNDS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    segs = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    import torch
    import bench
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    from ffmpeg_distributed_amd.testsrc import CONTENT
    W, H, _, _, Q, SEG, FULL, HUFF, _ = bench.WORKLOADS["c2"]
    dev = torch.device("cuda", 0)
    npool = 4
    pool = torch.empty((npool * SEG, bench.frame_bytes(W, H)), dtype=torch.uint8, device=dev)
    for i in range(0, npool * SEG, 20):
        pool[i:i + 20] = CONTENT["testsrc"](W, H, i, 20, dev, full_range=FULL)
    torch.cuda.synchronize()
    ptr = [pool[j * SEG].data_ptr() for j in range(npool)]

    def mk(name):
        if name == "explicit2":
            return MjpegEncoder(0, W, H, qscale=Q, max_batch=2 * SEG, merge=False)
        os.environ["MJG_MERGE_HOLD"] = "1" if name == "hold" else "0"
        e = MjpegEncoder(0, W, H, qscale=Q, max_batch=SEG, merge=name != "single")
        os.environ.pop("MJG_MERGE_HOLD")
        return e

    names = ["explicit2", "hold", "idle", "single"]
    encs = {n: mk(n) for n in names}

    def run(name, n, s0):
        e = encs[name]
        if name == "explicit2":
            for s in range(s0, s0 + n, 2):
                e.submit_segments([(ptr[s % npool], SEG), (ptr[(s + 1) % npool], SEG)])
                if e.pending == e.host_depth:
                    e.sync()
        else:
            for s in range(s0, s0 + n):
                e.submit(device_ptr=ptr[s % npool], nframes=SEG)
                if e.pending == e.depth:
                    e.sync()
        while e.pending:
            e.sync()
        torch.cuda.synchronize()

    res = {n: [] for n in names}
    for r in range(rounds):
        for n in names[r % 4:] + names[:r % 4]:
            run(n, 4, 0)
            torch.cuda._sleep(1000)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(n, segs, 4)
            dt = time.perf_counter() - t0
            torch.cuda._sleep(1000)
            torch.cuda.synchronize()
            res[n].append(segs * SEG / dt)
            print(f"round {r} {n:10s} {segs * SEG / dt:10.0f} fps  {dt / segs * 1e3:.4f} ms/segment", flush=True)
    for n in names:
        v = sorted(res[n])
        print(f"{n:10s} median {v[len(v) // 2]:10.0f} fps over {rounds} rounds of {segs} segments")


if __name__ == "__main__":
    main()
