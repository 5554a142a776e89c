#!/usr/bin/env python3
"""Perf A/B of k_encode source variants in ONE process, interleaved rounds (guide §5.4
rule 24).  VARIANTS="name=src:flags;..." where src is a directory holding api.hip & friends
(default: the working tree) or `@patches` (tools/patches.py: the product source with the
named experiment patches applied, e.g. `@no_skip+wide_cost=3`), and flags are extra hipcc
options.  Only kernel times are compared; run tests/test_gpu_parity.py for correctness of
the shipped build."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ffmpeg_distributed_amd", "csrc")


def parse():
    out = []
    for item in os.environ.get("VARIANTS", "cur=:").split(";"):
        name, rest = item.split("=", 1)
        src, _, flags = rest.partition(":")
        if src.startswith("@"):
            src = os.path.join("tools", f"_v{name}src"), src[1:]
        out.append((name, src, flags.split()))
    return out


def build(name, src, flags):
    so = os.path.join(ROOT, "ffmpeg_distributed_amd", f"libmjgpu_v_{name}.so")
    if isinstance(src, tuple):  # (copy dir, patch spec)
        import patches
        src = patches.apply(src[1], os.path.join(ROOT, src[0]))
    else:
        src = os.path.abspath(os.path.join(ROOT, src)) if src else CSRC
    from ffmpeg_distributed_amd import build as B  # the product's compile flags
    base = [a for a in B._command(so) if not a.endswith((".hip", ".cpp"))]
    cmd = base[:1] + [*flags] + base[1:] + [os.path.join(src, "api.hip"), os.path.join(CSRC, "sws_filter.cpp")]
    subprocess.run(cmd, check=True, cwd=src)
    return so


def main():
    vs = parse()
    if "--build" in sys.argv:
        for v in vs:
            build(*v)
        return
    import torch
    import bench
    from ffmpeg_distributed_amd import _lib
    from ffmpeg_distributed_amd.testsrc import CONTENT
    gen = CONTENT[os.environ.get("CONTENT", "testsrc")]
    W, H, DW, DH, Q, N, FULL, HUFF, _ = bench.WORKLOADS[os.environ.get("WL", "c2")]
    Q = int(os.environ.get("Q") or Q)  # quantiser override (A/B at other q)
    dev = torch.device("cuda", 0)
    pool = torch.empty((N, W * H + 2 * ((W + 1) // 2) * ((H + 1) // 2)), dtype=torch.uint8, device=dev)
    for i in range(0, N, 10):
        k = min(10, N - i)
        pool[i:i + k] = gen(W, H, i, k, dev, full_range=FULL)
    torch.cuda.synchronize()
    encs = {}
    for name, _, _ in vs:
        _lib._lib = None
        _lib.LIB_PATH = os.path.join(ROOT, "ffmpeg_distributed_amd", f"libmjgpu_v_{name}.so")
        from ffmpeg_distributed_amd.encoder import MjpegEncoder
        encs[name] = MjpegEncoder(0, W, H, DW, DH, full_range=FULL, qscale=Q, max_batch=N, timing=True,
                                  huffman=HUFF)
    res = {n: [] for n in encs}
    ref = None
    names = list(encs)
    for rnd in range(int(os.environ.get("ROUNDS", "6"))):
        # rotate the order every round: no variant always runs first (or right after another)
        for n in names[rnd % len(names):] + names[:rnd % len(names)]:
            e = encs[n]
            e.kernel_times(reset=True)
            for _ in range(3):
                e.submit(device_ptr=pool.data_ptr(), nframes=N)
                sizes = e.sync()
            if rnd == 0:
                out = e.fetch()
                ref = ref or out
                print(f"{n}: output {'==' if out == ref else '!='} first variant", flush=True)
            res[n].append(e.kernel_times()[0])
    for n, rows in res.items():
        enc = sorted(r["encode"] + r["scale"] + r["huff"] for r in rows)
        tot = sorted(sum(r.values()) for r in rows)
        sc = sorted(r["scale"] for r in rows)
        print(f"{n:12s} scale+huff+encode median {enc[len(enc)//2]:.4f} ms (min {enc[0]:.4f}); "
              f"all kernels median {tot[len(tot)//2]:.4f} ms per {N} frames; scale alone median {sc[len(sc)//2]:.4f}")


if __name__ == "__main__":
    main()
