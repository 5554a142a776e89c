#!/usr/bin/env python3
"""Host read rates of a raw 4K segment file on the GPU box (the input path).

Writes one 120-frame 4K raw I420 segment (1.49 GB), then times reading it into one buffer with
4 threads of positional reads (worker.py's pread path):
  warm      page cache (the dispatcher's usual case: the splitter just wrote the segment)
  cold      after posix_fadvise(DONTNEED) (pages evicted, buffered reads from the device)
  o_direct  O_DIRECT reads (no page cache; 4 KiB-aligned buffer, offsets and lengths)
Tool, not product.  Usage: python tools/read_probe.py [--dir DIR] [--gb 1.49]
"""
from __future__ import annotations

import argparse
import json
import mmap
import os
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor


def timed_read(path, buf, flags=0, threads=4):
    n = len(buf)
    fd = os.open(path, os.O_RDONLY | flags)
    try:
        piece = ((n + threads - 1) // threads + 4095) // 4096 * 4096
        mv = memoryview(buf)

        def one(i):
            off = i * piece
            end = min(n, off + piece)
            while off < end:
                k = os.preadv(fd, [mv[off:end]], off)
                if k <= 0:
                    raise OSError("short read")
                off += k

        t = time.monotonic()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, range(threads)))
        return time.monotonic() - t
    finally:
        os.close(fd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=None)
    ap.add_argument("--gb", type=float, default=1.49)
    a = ap.parse_args()
    n = int(a.gb * 1e9) // 4096 * 4096
    d = tempfile.mkdtemp(prefix="mjg_read_", dir=a.dir)
    path = os.path.join(d, "seg.raw")
    buf = mmap.mmap(-1, n)  # page-aligned (O_DIRECT needs an aligned buffer)
    out = {"bytes": n}
    try:
        blk = os.urandom(1 << 20)
        t = time.monotonic()
        with open(path, "wb") as f:
            for i in range(0, n, len(blk)):
                f.write(blk[: min(len(blk), n - i)])
            f.flush()
            os.fsync(f.fileno())
        out["write_fsync_gbs"] = round(n / (time.monotonic() - t) / 1e9, 2)
        out["warm_gbs"] = [round(n / timed_read(path, buf) / 1e9, 2) for _ in range(3)]
        cold = []
        for _ in range(2):
            fd = os.open(path, os.O_RDONLY)
            os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
            os.close(fd)
            cold.append(round(n / timed_read(path, buf) / 1e9, 2))
        out["cold_gbs"] = cold
        try:
            out["o_direct_gbs"] = [round(n / timed_read(path, buf, os.O_DIRECT) / 1e9, 2) for _ in range(2)]
        except OSError as e:
            out["o_direct_gbs"] = f"unsupported: {e}"
        with open("/proc/mounts") as f:
            out["fs"] = [l.split()[:3] for l in f if " " + os.path.dirname(d.rstrip("/")) in l or l.split()[1] == "/"][:3]
    finally:
        buf.close()
        os.remove(path)
        os.rmdir(d)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
