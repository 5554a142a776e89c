"""The `gpu:N` segment worker: the process the dispatcher starts in place of
`nice -n10 ionice -c3 ffmpeg -f matroska -i pipe: <remote_args> -f matroska pipe:`
(ffmpeg_distributed.py:131-141), with the same contract: one segment on stdin, the
encoded Matroska segment on stdout, ffmpeg-style `Duration:` / `frame= ... speed=Nx`
lines on stderr (parsed at ffmpeg_distributed.py:39-40,62-73), exit code 0 on success.

    python -m ffmpeg_distributed_amd.worker --device N <remote_args...>

remote_args inside the GPU profile (profile.parse) are encoded on GPU N; anything else
runs the reference command line with the real ffmpeg as a child (same output, CPU).

Input: Matroska with V_UNCOMPRESSED I420/Y42B/444P video and YUV4MPEG2 are read natively;
any other codec (the splitter's lossless x264 segments, fd.py:198-202) is decoded by an
`ffmpeg ... -f yuv4mpegpipe` child feeding this process (SURVEY §8f "splitter decode").
A -pix_fmt whose sampling differs from the input's needs a chroma resample, which is not on
the GPU path: the decoded frames then go to the real ffmpeg as y4m (`ffmpeg_fallthrough`).
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import subprocess
import sys
import threading
import time
from fractions import Fraction
from dataclasses import dataclass
from typing import List, Optional

from . import container, profile

DECODE_ARGV = ["ffmpeg", "-v", "error", "-f", "matroska", "-i", "pipe:", "-map", "0:v:0",
               "-f", "yuv4mpegpipe", "-strict", "-1", "pipe:"]
# frames per submit: MJG_WORKER_BATCH, or as many as fit BATCH_BYTES of input (at most 32).
# The three page-locked batch buffers are allocated per segment process, and pinning is a
# large part of its start-up: 4K batches of 32 frames pinned 1.2 GB, of 8 frames 0.3 GB.
BATCH = int(os.environ.get("MJG_WORKER_BATCH", "0"))
BATCH_BYTES = int(os.environ.get("MJG_WORKER_BATCH_BYTES", str(96 << 20)))
# serve mode (and the resident encoder) pins its batches once for many segments.  128 MiB (10 4K
# frames) measured ahead of 256 MiB end to end: a segment's first H2D starts after a smaller
# first read and its last batch drains sooner (per-segment process 3,490-3,649 vs 3,304-3,392 4K
# fps, two clients 3,755-3,790 vs 3,289-3,466; profiles/r05/e2e_batch_ab.txt); every batch holds
# at least 4 frames (an 8K batch of 1 frame leaves the GPU waiting on every sync)
SERVE_BATCH_BYTES = int(os.environ.get("MJG_SERVE_BATCH_BYTES", str(128 << 20)))
MIN_BATCH_FRAMES = 4


def batch_frames(opts, frame_bytes: int) -> int:
    """Frames per page-locked batch: MJG_WORKER_BATCH if set, else what batch_bytes holds,
    clamped to [MIN_BATCH_FRAMES, 32]."""
    return opts.batch or max(MIN_BATCH_FRAMES, min(32, opts.batch_bytes // max(frame_bytes, 1)))
# FFmpeg builds differ in the pix_fmt their CLI hands the mjpeg encoder for yuv420p input
# (yuvj420p: no COM; yuv420p + full range: COM "CS=ITU601"); default = yuvj420p.
COM_ITU601 = os.environ.get("MJG_COM_ITU601", "0") == "1"


def reference_argv(args: List[str]) -> List[str]:
    """The command the reference runs for one segment (fd.py:133-135, without nice/ionice)."""
    return ["ffmpeg", "-f", "matroska", "-i", "pipe:", *args, "-f", "matroska", "pipe:"]


def _hms(t: float) -> str:
    h, r = divmod(max(t, 0.0), 3600)
    m, s = divmod(r, 60)
    return f"{int(h):02d}:{int(m):02d}:{s:05.2f}"


class Progress:
    """ffmpeg-shaped stderr lines so FFMPEGProc's progress regex follows the GPU worker."""

    def __init__(self, err, fps: Fraction, qscale: int):
        self.err, self.fps, self.q = err, fps, qscale
        self.t0 = time.monotonic()
        self.last = 0.0
        self.bytes = 0

    def duration(self, seconds: Optional[float]):
        if seconds is not None:
            self.err.write(f"  Duration: {_hms(seconds)}, start: 0.000000, bitrate: N/A\n")
            self.err.flush()

    def update(self, frames: int, nbytes: int, final: bool = False):
        self.bytes += nbytes
        now = time.monotonic()
        if not final and now - self.last < 0.5:
            return
        self.last = now
        el = max(now - self.t0, 1e-6)
        t = float(frames / self.fps) if self.fps else 0.0
        kb = self.bytes // 1024
        br = (self.bytes * 8 / t / 1000) if t > 0 else 0.0
        self.err.write(f"frame={frames:5d} fps={int(frames / el):3d} q={self.q:.1f} "
                       f"size={kb:8d}KiB time={_hms(t)} bitrate={br:7.1f}kbits/s "
                       f"speed={t / el:.3f}x\n")
        self.err.flush()


# 8: 84 GB/s from the page cache for a 4K segment against 61 GB/s with 4 (r05, bench e2e trace)
READ_THREADS = int(os.environ.get("MJG_READ_THREADS", "8"))
# page-locked batch buffers per encoder context (MJG_WORKER_BUFFERS): the reader fills one
# while two submits are queued and a third waits for the sync
NBUF = max(3, int(os.environ.get("MJG_WORKER_BUFFERS", "4")))
NOUT = 6  # page-locked output buffers: one being filled, up to four queued to the muxer, one in its write
# MJG_WORKER_TRACE=1: one `mjg-trace:` stderr line per segment with where its time went
# (reader, submit, sync, fetch, mux) and the process's CPU / NUMA placement.
TRACE = os.environ.get("MJG_WORKER_TRACE", "0") == "1"


@dataclass(frozen=True)
class Options:
    """Per-segment settings.  A worker process takes them from its environment (the module
    values above); the resident encoder (resident.py) takes them from each request, i.e. from
    the environment of the mjg_client process that sent the segment."""
    batch: int = 0                  # MJG_WORKER_BATCH: frames per submit (0: by bytes)
    batch_bytes: int = 96 << 20     # MJG_WORKER_BATCH_BYTES
    com_itu601: bool = False        # MJG_COM_ITU601
    read_threads: int = 8           # MJG_READ_THREADS
    trace: bool = False             # MJG_WORKER_TRACE
    client_t0: float = 0.0          # trace: the mjg_client's start (MJG_CLIENT_T0, monotonic ns)
    t_accept: float = 0.0           # trace: when the resident encoder accepted the request

    @classmethod
    def from_env(cls, env, batch_bytes: Optional[int] = None, t_accept: float = 0.0) -> "Options":
        """From NAME=VALUE settings (absent names take the defaults above)."""
        try:
            client_t0 = int(env.get("MJG_CLIENT_T0", "0") or 0) / 1e9
        except ValueError:
            client_t0 = 0.0
        return cls(batch=int(env.get("MJG_WORKER_BATCH", "0") or 0),
                   batch_bytes=int(env.get("MJG_WORKER_BATCH_BYTES", "0") or 0) or batch_bytes or (96 << 20),
                   com_itu601=env.get("MJG_COM_ITU601", "0") == "1",
                   read_threads=max(1, int(env.get("MJG_READ_THREADS", "8") or 8)),
                   trace=env.get("MJG_WORKER_TRACE", "0") == "1", client_t0=client_t0, t_accept=t_accept)


def process_options(batch_bytes: Optional[int] = None) -> Options:
    """This process's settings (the module values, read from its environment at import)."""
    return Options(batch=BATCH, batch_bytes=batch_bytes or BATCH_BYTES, com_itu601=COM_ITU601,
                   read_threads=READ_THREADS, trace=TRACE)
# Bind the worker to its GPU's NUMA node (CPUs, and preferred memory for its page-locked
# batches), see bind_numa.  MJG_NUMA_BIND=0 leaves placement to the scheduler.
NUMA_BIND = os.environ.get("MJG_NUMA_BIND", "1") == "1"
_bound_node: Optional[int] = None
_gpu_node = -1


def bind_numa(device: int) -> int:
    """Run the calling thread, and the threads it starts from here on, on the CPUs of
    `device`'s NUMA node and prefer that node for their memory: the segment's positional
    reads copy page-cache pages into page-locked batches that the GPU then reads over PCIe,
    and both the copy and the DMA cross the socket interconnect when the process sits on the
    other node.  Affinity and memory policy are per thread on Linux: threads started later
    (reader, pread pool) inherit them, threads that already exist (the HIP runtime's, which
    the NUMA query itself starts) do not.  When the node's CPUs are not among the allowed
    ones nothing changes (no remote memory preference for a thread that cannot run there).
    Returns the node (-1: unknown / not bound)."""
    global _bound_node, _gpu_node
    if _bound_node is not None:
        return _bound_node
    _bound_node = -1
    from . import _lib
    try:
        node = _gpu_node = _lib.device_numa_node(device)
    except Exception:
        return -1
    if node < 0 or not NUMA_BIND:
        return -1
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _cpulist(f.read().strip()) & os.sched_getaffinity(0)
        if not cpus:
            return -1
        os.sched_setaffinity(0, cpus)
    except OSError:
        return -1
    _prefer_node(node)
    _bound_node = node
    return node


def _prefer_node(node: int) -> None:
    """set_mempolicy(MPOL_PREFERRED, {node}) for the calling thread (x86-64 Linux)."""
    import ctypes
    import platform
    if platform.machine() != "x86_64" or node >= 64:
        return
    try:
        libc = ctypes.CDLL(None, use_errno=True)
        mask = ctypes.c_ulong(1 << node)
        libc.syscall(238, 1, ctypes.byref(mask), ctypes.c_ulong(64))  # SYS_set_mempolicy
    except (OSError, AttributeError):
        pass


def placement() -> str:
    """CPUs this process may run on, the NUMA nodes they span and the cgroup's CPU
    throttling counters (tracing only; Linux /proc and /sys, best effort)."""
    out = []
    try:
        cpus = sorted(os.sched_getaffinity(0))
        out.append(f"cpus={len(cpus)}")
        nodes = {}
        base = "/sys/devices/system/node"
        for d in os.listdir(base):
            if d.startswith("node") and d[4:].isdigit():
                with open(f"{base}/{d}/cpulist") as f:
                    lst = _cpulist(f.read().strip())
                k = len(lst & set(cpus))
                if k:
                    nodes[int(d[4:])] = k
        out.append("nodes=" + ",".join(f"{n}:{k}" for n, k in sorted(nodes.items())))
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            st = dict(line.split() for line in f if line.strip())
        out.append(f"throttled={st.get('nr_throttled', '?')}/{st.get('nr_periods', '?')}"
                   f" throttled_ms={int(st.get('throttled_usec', 0)) // 1000}")
    except (OSError, ValueError):
        pass
    out.append(f"cpu_now={_current_cpu()} gpu_node={_gpu_node} bound={_bound_node}")
    return " ".join(out)


def _cpulist(text: str) -> set:
    cpus = set()
    for part in text.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def _current_cpu() -> int:
    try:
        with open("/proc/thread-self/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[36])
    except (OSError, ValueError, IndexError):
        return -1


def _regular_file_fd(f) -> Optional[int]:
    """The descriptor of a seekable regular file behind `f`, else None (pipes, sockets,
    in-memory streams read sequentially)."""
    import stat
    try:
        fd = f.fileno()
        if stat.S_ISREG(os.fstat(fd).st_mode) and f.seekable():
            return fd
    except (AttributeError, OSError, ValueError):
        pass
    return None


def _pread_exact(fd: int, dest, off: int) -> None:
    got = 0
    while got < len(dest):
        k = os.preadv(fd, [dest[got:]], off + got)
        if k <= 0:
            raise ValueError(f"segment file ends inside a frame at byte {off + got}")
        got += k


class Source:
    """Packed planar frames from stdin: .info (StreamInfo), .read_into(buf, n) -> count."""

    def __init__(self, raw, read_threads: int = READ_THREADS, stderr=None):
        self.child = None
        self.feeder = None
        head = raw.read(4)
        if head.startswith(b"YUV4"):
            self._y4m(container.Y4MReader(raw, head))
            self.duration = None
            return
        if head != b"\x1a\x45\xdf\xa3":
            raise ValueError("input is neither Matroska nor YUV4MPEG2")
        mkv = container.MkvReader(raw, head, record=True)
        tr = next((t for t in mkv.tracks if t.codec.startswith("V_")), None)
        if tr is None:
            raise ValueError("no video track in the segment")
        self.duration = mkv.duration_seconds()
        info = mkv.info(tr.number)
        if tr.codec == "V_UNCOMPRESSED" and tr.colour_space in container.MKV_FOURCC_CHROMA:
            self.info = info
            mkv.stop_recording()
            self._mkv, self._track = mkv, tr.number
            self.read_into = self._read_mkv
            self._fd = _regular_file_fd(raw)
            if self._fd is not None:  # a file (the dispatcher's segment): parallel positional reads
                from concurrent.futures import ThreadPoolExecutor
                self._pool = ThreadPoolExecutor(read_threads)
                self.read_into = self._read_mkv_pread
            return
        # any other codec: ffmpeg decodes, we read its y4m
        self.child = subprocess.Popen(DECODE_ARGV, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                      stderr=_fd_or_none(stderr))
        self.feeder = threading.Thread(target=self._feed, args=(mkv, raw), daemon=True)
        self.feeder.start()
        self._y4m(container.Y4MReader(self.child.stdout))

    def _feed(self, mkv, raw):
        # the decoder gets the exact bytes we consumed: replay them, then the rest
        try:
            self.child.stdin.write(mkv.replay_bytes())
            while True:
                b = raw.read(1 << 20)
                if not b:
                    break
                self.child.stdin.write(b)
        except BrokenPipeError:
            pass
        finally:
            try:
                self.child.stdin.close()
            except BrokenPipeError:
                pass

    def _y4m(self, rd):
        self.info = rd.info
        self.read_into = rd.read_into

    def _read_mkv(self, buf, n):
        fb = self.info.frame_bytes
        mv = memoryview(buf).cast("B")
        for i in range(n):
            try:
                ts = self._mkv.read_frame_into(self._track, mv[i * fb:(i + 1) * fb])
            except ValueError as e:
                raise ValueError(f"V_UNCOMPRESSED {e}") from None
            if ts is None:
                return i
        return n

    def _read_mkv_pread(self, buf, n):
        fb = self.info.frame_bytes
        mv = memoryview(buf).cast("B")
        futs = []

        def pread(off, dest):
            futs.append(self._pool.submit(_pread_exact, self._fd, dest, off))

        try:
            got = self._mkv.frames_into_pread(self._track, [mv[i * fb:(i + 1) * fb] for i in range(n)], pread)
        except ValueError as e:
            raise ValueError(f"V_UNCOMPRESSED {e}") from None
        finally:
            # every positional read has finished before the batch buffer is handed on (or
            # freed on an error path), failed or not; then the first failure is raised
            from concurrent.futures import wait
            wait(futs)
        for f in futs:
            f.result()
        return got

    def close(self, kill: bool = False) -> int:
        """Stop reading: join the pread pool; close the decoder child's output and wait for
        it (kill=True, on an error path: terminate it first).  Returns its exit code."""
        pool = getattr(self, "_pool", None)
        if pool is not None:
            pool.shutdown(wait=True)
            self._pool = None
        if self.child is None:
            return 0
        if kill and self.child.poll() is None:
            self.child.kill()
        try:
            self.child.stdout.close()
        except OSError:
            pass
        rc = self.child.wait()
        self.child = None
        return rc


def _fd_or_none(f):
    try:
        return f.fileno()
    except (AttributeError, OSError, ValueError):
        return None


def passthrough(args: List[str], stdin=None, stdout=None, stderr=None) -> int:
    """Outside the GPU profile: run exactly what the reference runs (on this segment's
    input, output and error streams: the process's own stdin / stdout / stderr unless given;
    in the resident encoder they are the client's descriptors, so ffmpeg's own `Duration:` /
    `frame=` lines reach the dispatcher as they would from the reference's worker)."""
    err = stderr or sys.stderr
    err.flush()  # our own lines before the child's
    try:
        return subprocess.call(reference_argv(args), stdin=_fd_or_none(stdin), stdout=_fd_or_none(stdout),
                               stderr=_fd_or_none(err))
    except FileNotFoundError:
        err.write("ffmpeg not found for a non-GPU profile\n")
        err.flush()
        return 127


def ffmpeg_fallthrough(src: Source, args: List[str], stdout, stderr=None) -> int:
    """The reference command on the CPU for frames already being read: the decoded frames
    go to `ffmpeg -f yuv4mpegpipe -i pipe: <remote_args> -f matroska pipe:` as y4m (its
    stderr is the segment's, see passthrough)."""
    err = stderr or sys.stderr
    argv = ["ffmpeg", "-f", "yuv4mpegpipe", "-i", "pipe:", *args, "-f", "matroska", "pipe:"]
    err.flush()
    try:
        child = subprocess.Popen(argv, stdin=subprocess.PIPE, stdout=stdout, stderr=_fd_or_none(err))
    except FileNotFoundError:
        err.write("ffmpeg not found for a non-GPU profile\n")
        err.flush()
        src.close()
        return 127
    fb = src.info.frame_bytes
    buf = bytearray(fb * 8)
    try:
        child.stdin.write(container.y4m_header(src.info))
        while True:
            n = src.read_into(buf, 8)
            for i in range(n):
                child.stdin.write(b"FRAME\n")
                child.stdin.write(memoryview(buf)[i * fb:(i + 1) * fb])
            if n < 8:
                break
        child.stdin.close()
    except BrokenPipeError:
        pass
    rc = child.wait()
    return rc or src.close()


def run(device: int, args: List[str], stdin=None, stdout=None, stderr=None, cache=None,
        batch_bytes: Optional[int] = None, opts: Optional[Options] = None) -> int:
    """One segment, stdin -> stdout.  `cache` (serve / resident mode): a dict that keeps the
    encoder context and the page-locked batch buffers between segments of the same stream
    shape.  `opts`: the segment's settings (default: this process's, process_options)."""
    t_run = time.monotonic()
    opts = opts or process_options(batch_bytes)
    stdin = stdin or sys.stdin.buffer
    stdout = stdout or sys.stdout.buffer
    stderr = stderr or sys.stderr
    prof, why = profile.try_parse(args)
    if prof is None:
        stderr.write(f"gpu:{device}: {why}; running ffmpeg on the CPU\n")
        stderr.flush()
        return passthrough(args, stdin, stdout, stderr)

    src = Source(stdin, opts.read_threads, stderr)
    info = src.info
    if prof.chroma is not None and prof.chroma != info.chroma:
        stderr.write(f"gpu:{device}: -pix_fmt needs {info.chroma} -> {prof.chroma} chroma resampling; "
                     f"running ffmpeg on the CPU\n")
        stderr.flush()
        return ffmpeg_fallthrough(src, args, stdout, stderr)
    dst_w, dst_h = prof.scale or (info.width, info.height)
    bind_numa(device)  # before the reader threads and the batch buffers
    from .encoder import MjpegEncoder, PinnedBuffer   # GPU work starts here

    batch = batch_frames(opts, info.frame_bytes)

    sar = profile.scaled_sar(info.sar, (info.width, info.height), (dst_w, dst_h))
    key = (info.width, info.height, dst_w, dst_h, info.full_range, prof.qscale, sar,
           opts.com_itu601 and not info.full_range, prof.huffman, info.chroma, prof.rst, batch)
    nbuf = NBUF
    if cache is not None and cache.get("key") == key:
        enc, bufs, obufs = cache["enc"], cache["bufs"], cache["obufs"]
    else:
        if cache is not None:
            release(cache)
        enc = MjpegEncoder(device, info.width, info.height, dst_w, dst_h, full_range=info.full_range,
                           qscale=prof.qscale, sar=sar, max_batch=batch,
                           com_itu601=opts.com_itu601 and not info.full_range, huffman=prof.huffman,
                           chroma=info.chroma, rst=prof.rst)
        bufs = [PinnedBuffer(batch * enc.frame_bytes) for _ in range(nbuf)]
        # page-locked output buffers: the packets are DMA'd into one (enc.fetch_into) and the
        # muxer writes them from it; regrown when a submit's JPEGs do not fit
        obufs = [None] * NOUT
        if cache is not None:
            cache.update(key=key, enc=enc, bufs=bufs, obufs=obufs)
    prog = Progress(stderr, info.fps, prof.qscale)
    prog.duration(src.duration)
    mkv = container.MkvWriter(stdout, dst_w, dst_h, info.fps, sar)

    # NBUF page-locked batches: the reader fills one while two are queued on the GPU (the
    # encoder takes a second submit before the first is synced, so its kernels run back to
    # back); a batch returns to the reader as soon as its submit is synced (the H2D has read
    # it), before the packets are fetched, so the reader never waits on the fetch.
    fb = enc.frame_bytes
    free: "queue.Queue[int]" = queue.Queue()
    full: "queue.Queue" = queue.Queue()
    abort = threading.Event()
    for i in range(nbuf):
        free.put(i)

    tr = {"read": 0.0, "submit": 0.0, "sync": 0.0, "fetch": 0.0, "mux": 0.0, "wait": 0.0}
    t_seg = time.monotonic()

    def reader():
        try:
            while True:
                i = free.get()
                if i < 0 or abort.is_set():
                    return
                t0 = time.monotonic()
                n = src.read_into(bufs[i].array, batch)
                tr["read"] += time.monotonic() - t0
                full.put((i, n))
                if n < batch:
                    full.put(None)
                    return
        except BaseException as e:   # surfaced by the main loop
            full.put(e)

    th = threading.Thread(target=reader, daemon=True)
    th.start()
    frames = 0
    queued: "list" = []  # buffer index and frame count per submit, oldest first
    # the muxer thread writes each synced submit's packets while the main thread keeps the
    # GPU fed (a 4K segment's 120 JPEGs are ~20 MB of writes)
    outq: "queue.Queue" = queue.Queue(maxsize=4)
    ofree: "queue.Queue[int]" = queue.Queue()  # output buffers the muxer has written
    for i in range(NOUT):
        ofree.put(i)
    mux_err: list = []

    def muxer():
        nonlocal frames
        while True:
            try:
                item = outq.get(timeout=0.1)
            except queue.Empty:
                if abort.is_set():  # error path: the main thread may not be able to post None
                    return
                continue
            if item is None:
                return
            packets, m, ob = item
            if mux_err:
                ofree.put(ob)
                continue  # drain after a failure
            try:
                t0 = time.monotonic()
                for p in packets:
                    mkv.write_frame(p)
                mkv.flush_pending()  # the packets leave buffer `ob` before it is reused
                tr["mux"] += time.monotonic() - t0
                frames += m
                prog.update(frames, sum(len(p) for p in packets))
            except BaseException as e:  # surfaced by the main thread
                mux_err.append(e)
            ofree.put(ob)

    mt = threading.Thread(target=muxer, daemon=True)
    mt.start()

    def drain_one():
        j, m = queued.pop(0)
        t0 = time.monotonic()
        enc.sync()
        free.put(j)  # consumed by its H2D: back to the reader before the fetch
        t1 = time.monotonic()
        while True:  # a written output buffer (the muxer returns them); abort: error path
            try:
                ob = ofree.get(timeout=0.1)
                break
            except queue.Empty:
                if mux_err:
                    raise mux_err[0]
        need = enc.last_total
        if obufs[ob] is None or obufs[ob].nbytes < need:
            if obufs[ob] is not None:
                obufs[ob].free()
            obufs[ob] = PinnedBuffer(max(need + need // 2, 1 << 20))
        packets = enc.fetch_into(obufs[ob])  # one DMA into page-locked memory, no copy
        tr["sync"] += t1 - t0
        tr["fetch"] += time.monotonic() - t1
        if mux_err:
            raise mux_err[0]
        outq.put((packets, m, ob))

    failed = True
    try:
        while True:
            t0 = time.monotonic()
            item = full.get()
            tr["wait"] += time.monotonic() - t0
            if item is None:
                break
            if isinstance(item, BaseException):
                raise item
            i, n = item
            if n:
                if len(queued) == enc.host_depth:  # host submits: one launch each
                    drain_one()
                t0 = time.monotonic()
                enc.submit(bufs[i].array[: n * fb], n)
                tr["submit"] += time.monotonic() - t0
                queued.append((i, n))
            else:
                free.put(i)
        while queued:
            drain_one()
        outq.put(None)
        mt.join()
        if mux_err:
            raise mux_err[0]
        mkv.close()
        prog.update(frames, 0, final=True)
        failed = False
        if opts.trace:
            hand = ""  # the resident's hand-off: client start -> accept -> worker.run
            if opts.t_accept:
                hand += f"handoff={t_run - opts.t_accept:.4f} "
                if opts.client_t0:
                    hand += f"client={opts.t_accept - opts.client_t0:.4f} "
            stderr.write(f"mjg-trace: frames={frames} total={time.monotonic() - t_seg:.4f} "
                         f"setup={t_seg - t_run:.4f} {hand}"
                         + " ".join(f"{k}={v:.4f}" for k, v in tr.items()) + f" {placement()}\n")
            stderr.flush()
    finally:
        # Nothing is freed while a reader could still write into a batch buffer: stop the
        # reader thread (it finishes at most the read in flight, whose positional reads it
        # waits for), killing a decoder child whose pipe it may be blocked on; then close
        # the source, and only then the encoder and the page-locked buffers.
        abort.set()
        free.put(-1)
        if mt.is_alive():  # error path: let the muxer finish what it holds, then stop
            try:  # never block here: a full queue means the muxer is inside a write, and it
                outq.put_nowait(None)  # sees `abort` once that write returns
            except queue.Full:
                pass
            mt.join(timeout=5.0)
        th.join(timeout=5.0)
        if th.is_alive():
            src.close(kill=True)
            th.join(timeout=5.0)
        stuck = th.is_alive()  # blocked on a stdin pipe that never delivers: leak, never free
        # the muxer's packets are views into the page-locked output buffers: one still inside
        # a write (a stdout pipe that does not drain) keeps them, so they are leaked, not freed
        mux_stuck = mt.is_alive()
        rc = src.close(kill=failed)
        if (failed or stuck or mux_stuck) and cache is not None:  # a submit may still be queued: start afresh
            for k in ("key", "enc", "bufs", "obufs"):
                cache.pop(k, None)
            cache = None
        if cache is None:
            enc.close()
            if not stuck:
                for b in bufs:
                    b.free()
            if not mux_stuck:
                for b in obufs:
                    if b is not None:
                        b.free()
    if rc:
        stderr.write(f"decoder exited with {rc}\n")
        return 1
    return 0


def release(cache) -> None:
    """Close the encoder context and free the batch buffers a serve cache holds."""
    enc, bufs = cache.pop("enc", None), cache.pop("bufs", None) or []
    obufs = [b for b in (cache.pop("obufs", None) or []) if b is not None]
    cache.pop("key", None)
    if enc is not None:
        enc.close()
    for b in bufs + obufs:
        b.free()


SERVE_DONE = "mjg-serve: segment done rc="


def serve(device: int, args: List[str], requests=None, stderr=None) -> int:
    """Persistent worker (dispatcher --persistent-gpu-workers): one process per `-H gpu:N`
    entry encodes segment after segment, keeping its HIP context, encoder and page-locked
    buffers, so a segment no longer pays process start + HIP init + allocation (~0.5 s).
    Each request line on stdin is a JSON array `[INPUT, OUTPUT]` (dispatcher.serve_request:
    any path survives, tabs and newlines included); the segment runs exactly as `run`
    runs it for one process (same output bytes, same ffmpeg-style stderr lines), then
    `mjg-serve: segment done rc=N` on stderr ends it.  EOF on stdin ends the server."""
    requests = requests or sys.stdin
    stderr = stderr or sys.stderr
    cache: dict = {}
    try:
        for line in requests:
            line = line.rstrip("\n")
            if not line:
                continue
            try:
                src, dst = json.loads(line)
                with open(src, "rb") as fin, open(dst, "wb") as fout:
                    rc = run(device, args, stdin=fin, stdout=fout, stderr=stderr, cache=cache,
                             batch_bytes=SERVE_BATCH_BYTES)
            except Exception as e:
                stderr.write(f"gpu:{device}: {type(e).__name__}: {e}\n")
                rc = 1
            stderr.write(f"{SERVE_DONE}{rc}\n")
            stderr.flush()
    finally:
        release(cache)
    return 0


def main(argv=None) -> int:
    # no -h/--help and no abbreviations: every other argument is ffmpeg's (remote_args), and
    # argparse would read `-huffman default` as `-h uffman`
    ap = argparse.ArgumentParser(prog="ffmpeg_distributed_amd.worker", add_help=False, allow_abbrev=False)
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--serve", action="store_true")
    ns, rest = ap.parse_known_args(argv)
    if ns.serve:
        return serve(ns.device, rest)
    try:
        return run(ns.device, rest)
    except Exception as e:  # the dispatcher re-queues the segment on a nonzero exit
        sys.stderr.write(f"gpu:{ns.device}: {type(e).__name__}: {e}\n")
        return 1


if __name__ == "__main__":
    sys.exit(main())
