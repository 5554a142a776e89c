"""Resident per-GPU encoder behind `mjg_client` (csrc/mjg_client.c).

The dispatcher starts one worker process per segment (ffmpeg_distributed.py:131-141).  For
a `gpu:N` host that process is `mjg_client`: a small native program that hands its stdin,
stdout and stderr to this resident encoder over a Unix socket (SCM_RIGHTS) and exits with
the segment's exit code.  This process keeps the HIP runtime, the encoder contexts and the
page-locked batch buffers between segments, so a segment costs what `worker.run` costs in
`--serve` mode, while the dispatcher still sees exactly the reference's per-segment process
contract: segment on stdin, Matroska on stdout, ffmpeg-style progress on stderr, exit code.

    python -m ffmpeg_distributed_amd.resident --device N --socket NAME [--idle SECONDS]

mjg_client starts it (stdio on its log file, in the caller's process group) when no encoder listens on
NAME, an abstract-namespace socket.  Each connection is one request (wire format in
mjg_client.c): an encode request carries the remote_args, the client's MJG_* environment
and its three descriptors; `worker.run` encodes the segment from them on a thread of its
own (segments of concurrent clients overlap on the GPU), the copies of the descriptors are
closed, then the exit code goes back (an 'A' byte acknowledges the request first: a client
whose connection closes before it, queued while the encoder shut its socket at the idle
timeout, connects again).  Peers with another uid are refused (and the client refuses an
encoder of another uid).  The encoder exits after `idle` seconds without a request, or on a
shutdown request.
"""
from __future__ import annotations

import argparse
import array
import errno
import io
import os
import socket
import struct
import sys
import threading
import time
from typing import Dict, List, Tuple

from . import worker

MAGIC = b"MJG2"                      # r05: the ACK byte is part of the protocol (mjg_client.c)
KIND_ENCODE, KIND_SHUTDOWN = 0, 1
HEADER = struct.Struct("<4sIIII")   # magic, total bytes, kind, nargs, nenv
MAX_REQUEST = 1 << 20
ACK = b"A"                           # request read: the client no longer retries the connection
MAX_IDLE_CACHES = 4                  # encoder contexts kept between segments


def encode_request(kind: int, args: List[str], env: Dict[str, str]) -> bytes:
    """The wire form mjg_client sends (for tests and Python clients)."""
    parts = [a.encode("utf-8", "surrogateescape") + b"\0" for a in args]
    parts += [f"{k}={v}".encode("utf-8", "surrogateescape") + b"\0" for k, v in env.items()]
    body = b"".join(parts)
    return HEADER.pack(MAGIC, HEADER.size + len(body), kind, len(args), len(env)) + body


def parse_request(data: bytes) -> Tuple[int, List[str], Dict[str, str]]:
    if len(data) < HEADER.size:
        raise ValueError("short request")
    magic, total, kind, nargs, nenv = HEADER.unpack_from(data)
    if magic != MAGIC or total != len(data) or kind not in (KIND_ENCODE, KIND_SHUTDOWN):
        raise ValueError("malformed request")
    parts = data[HEADER.size:].split(b"\0")
    if parts[-1] != b"" or len(parts) - 1 != nargs + nenv:
        raise ValueError("malformed request strings")
    strs = [p.decode("utf-8", "surrogateescape") for p in parts[:-1]]
    env = {}
    for kv in strs[nargs:]:
        k, sep, v = kv.partition("=")
        if not sep:
            raise ValueError("malformed environment entry")
        env[k] = v
    return kind, strs[:nargs], env


def recv_request(conn: socket.socket) -> Tuple[bytes, List[int]]:
    """One request's bytes and the descriptors that came with it."""
    data, fds = b"", []
    total = None
    while total is None or len(data) < total:
        chunk, anc, flags, _ = conn.recvmsg(65536, socket.CMSG_SPACE(8 * 4))
        for level, typ, cdata in anc:
            if level == socket.SOL_SOCKET and typ == socket.SCM_RIGHTS:
                a = array.array("i")
                a.frombytes(cdata[: len(cdata) - len(cdata) % a.itemsize])
                fds.extend(a)
        if flags & socket.MSG_CTRUNC:
            for fd in fds:
                os.close(fd)
            raise ValueError("descriptors truncated")
        if not chunk:
            for fd in fds:
                os.close(fd)
            raise EOFError("client closed the connection")
        data += chunk
        if total is None and len(data) >= HEADER.size:
            total = HEADER.unpack_from(data)[1]
            if total > MAX_REQUEST or total < HEADER.size:
                for fd in fds:
                    os.close(fd)
                raise ValueError("request size")
    return data, fds


def peer_uid(conn: socket.socket) -> int:
    pid, uid, gid = struct.unpack("3i", conn.getsockopt(socket.SOL_SOCKET, socket.SO_PEERCRED,
                                                        struct.calcsize("3i")))
    return uid


class Resident:
    """The accept loop, a thread per request and a pool of worker.run caches (each an
    encoder context + its page-locked batches, reused LIFO so one client at a time always
    finds the context of its stream shape)."""

    def __init__(self, device: int, sock: socket.socket, idle: float, run=None):
        self.device, self.sock, self.idle = device, sock, idle
        self.run = run or worker.run
        self.lock = threading.Lock()
        self.active = 0
        self.last = time.monotonic()
        self.free_caches: List[dict] = []
        self.stop = threading.Event()
        self.threads: List[threading.Thread] = []

    def _take_cache(self) -> dict:
        with self.lock:
            return self.free_caches.pop() if self.free_caches else {}

    def _give_cache(self, cache: dict):
        with self.lock:
            self.free_caches.append(cache)
            extra = self.free_caches[:-MAX_IDLE_CACHES] if len(self.free_caches) > MAX_IDLE_CACHES else []
            del self.free_caches[:len(extra)]
        for c in extra:
            worker.release(c)

    def handle(self, conn: socket.socket, t_accept: float = 0.0):
        fds: List[int] = []
        rc = 1
        try:
            if peer_uid(conn) != os.getuid():
                return
            data, fds = recv_request(conn)
            kind, args, env = parse_request(data)
            conn.sendall(ACK)  # read, nothing of the segment touched yet (see mjg_client.c)
            if kind == KIND_SHUTDOWN:
                self.stop.set()
                rc = 0
            elif len(fds) != 3:
                rc = 1
            else:
                rc = self._encode(args, env, fds, t_accept)
                fds = []  # closed by _encode
            conn.sendall(struct.pack("<i", rc))
        except (OSError, ValueError, EOFError) as e:
            sys.stderr.write(f"resident gpu:{self.device}: request failed: {type(e).__name__}: {e}\n")
        finally:
            for fd in fds:
                os.close(fd)
            conn.close()
            with self.lock:
                self.active -= 1
                self.last = time.monotonic()

    def _encode(self, args: List[str], env: Dict[str, str], fds: List[int], t_accept: float = 0.0) -> int:
        fin = os.fdopen(fds[0], "rb")
        fout = os.fdopen(fds[1], "wb")
        ferr = io.TextIOWrapper(os.fdopen(fds[2], "wb"), encoding="utf-8", errors="replace",
                                line_buffering=True)
        cache = self._take_cache()
        rc = 1
        try:
            opts = worker.Options.from_env(env, worker.SERVE_BATCH_BYTES, t_accept=t_accept)
            rc = self.run(self.device, args, stdin=fin, stdout=fout, stderr=ferr, cache=cache, opts=opts)
        except Exception as e:  # a failed segment: the dispatcher re-queues it
            try:
                ferr.write(f"gpu:{self.device}: {type(e).__name__}: {e}\n")
            except (OSError, ValueError):
                pass
            rc = 1
        finally:
            # the segment's output and messages are complete before the exit code goes back
            for f in (fout, ferr, fin):
                try:
                    f.close()
                except (OSError, ValueError):
                    rc = rc or 1
            self._give_cache(cache)
        return rc

    def serve(self) -> int:
        self.sock.settimeout(0.5)
        try:
            while not self.stop.is_set():
                try:
                    conn, _ = self.sock.accept()
                    t_accept = time.monotonic()
                except socket.timeout:
                    with self.lock:
                        if self.active == 0 and time.monotonic() - self.last > self.idle:
                            break
                    continue
                conn.settimeout(None)
                with self.lock:
                    self.active += 1
                t = threading.Thread(target=self.handle, args=(conn, t_accept), daemon=True)
                self.threads = [x for x in self.threads if x.is_alive()] + [t]
                t.start()
        finally:
            self.sock.close()  # no new clients; the running segments finish
            for t in self.threads:
                t.join()
            with self.lock:
                caches, self.free_caches = self.free_caches, []
            for c in caches:
                worker.release(c)
        return 0


def shutdown(client: str, device: int, timeout: float = 30.0) -> bool:
    """Ask the resident encoder of `device` to exit (`mjg_client --shutdown`) and wait until its
    socket refuses connections; True when none runs any more."""
    import subprocess
    subprocess.run([client, "--device", str(device), "--shutdown"], timeout=timeout)
    name = subprocess.run([client, "--device", str(device), "--socket-name"], capture_output=True,
                          text=True, timeout=timeout).stdout.strip()
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        try:
            s.connect("\0" + name)
        except OSError:
            return True
        finally:
            s.close()
        time.sleep(0.1)
    return False


def listen(name: str) -> socket.socket:
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.bind("\0" + name)
    s.listen(64)
    return s


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="ffmpeg_distributed_amd.resident")
    ap.add_argument("--device", type=int, required=True)
    ap.add_argument("--socket", required=True)
    ap.add_argument("--idle", type=float, default=30.0)
    a = ap.parse_args(argv)
    try:
        sock = listen(a.socket)  # first: clients connect (and queue) while the runtime starts
    except OSError as e:
        if e.errno == errno.EADDRINUSE:
            return 0  # another encoder for this device won the race
        raise
    worker.bind_numa(a.device)  # main thread, before any request thread exists
    sys.stderr.write(f"resident gpu:{a.device}: listening on @{a.socket} (pid {os.getpid()})\n")
    sys.stderr.flush()
    return Resident(a.device, sock, a.idle).serve()


if __name__ == "__main__":
    sys.exit(main())
