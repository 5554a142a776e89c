"""The per-segment `gpu:N` process as a thin client (csrc/mjg_client.c) of the resident
per-GPU encoder (resident.py), on the CPU: the hand-off protocol (request wire format,
descriptors over SCM_RIGHTS), the reference's process contract as the dispatcher sees it
(ffmpeg_distributed.py:131-141: stdin segment -> stdout, stderr progress, exit code), and the
client starting an encoder when none listens.  The encode itself is a stub here; the GPU
test (tests/test_gpu_worker.py) runs the real one through the same path."""
import os
import subprocess
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ffmpeg_distributed_amd import build as B  # noqa: E402
from ffmpeg_distributed_amd import dispatcher as D  # noqa: E402
from ffmpeg_distributed_amd import resident as R  # noqa: E402


@pytest.fixture(scope="module")
def client():
    if not os.path.exists(B.LIB):
        pytest.skip("libmjgpu.so not built")
    return B.build_client()


def socket_name(client, dev="0"):
    return subprocess.run([client, "--device", dev, "--socket-name"], check=True, capture_output=True,
                          text=True).stdout.strip()


def test_request_roundtrip():
    args = ["-c:v", "mjpeg", "-vf", "scale=1920:1080:flags=bicubic", "tab\there", "ünï"]
    env = {"MJG_WORKER_TRACE": "1", "MJG_COM_ITU601": "0"}
    k, a, e = R.parse_request(R.encode_request(R.KIND_ENCODE, args, env))
    assert (k, a, e) == (R.KIND_ENCODE, args, env)
    data = R.encode_request(R.KIND_SHUTDOWN, [], {})
    assert R.parse_request(data) == (R.KIND_SHUTDOWN, [], {})
    for bad in (data[:10], b"XXXX" + data[4:], data + b"x", data[:-1] + b"y"):
        with pytest.raises(ValueError):
            R.parse_request(bad)


def test_options_from_request_env():
    from ffmpeg_distributed_amd import worker
    o = worker.Options.from_env({"MJG_WORKER_TRACE": "1", "MJG_WORKER_BATCH": "3",
                                 "MJG_COM_ITU601": "1"}, 256 << 20)
    assert o.trace and o.batch == 3 and o.com_itu601 and o.batch_bytes == 256 << 20 and o.read_threads == 8
    assert worker.Options.from_env({}) == worker.Options()


def test_batch_frames():
    """Page-locked batch sizing (r05): the resident encoder's 128 MiB default holds 10 4K
    frames; an 8K batch never drops below MIN_BATCH_FRAMES; MJG_WORKER_BATCH wins."""
    from ffmpeg_distributed_amd import worker
    o = worker.Options.from_env({}, worker.SERVE_BATCH_BYTES)
    assert worker.SERVE_BATCH_BYTES == 128 << 20
    assert worker.batch_frames(o, 3840 * 2160 * 3 // 2) == 10
    assert worker.batch_frames(o, 7680 * 4320 * 3 // 2) == worker.MIN_BATCH_FRAMES == 4
    assert worker.batch_frames(o, 64 * 64 * 3 // 2) == 32
    assert worker.batch_frames(worker.Options.from_env({"MJG_WORKER_BATCH": "3"}), 3840 * 2160 * 3 // 2) == 3


def fake_run(dev, args, stdin, stdout, stderr, cache, opts):
    """Stands in for worker.run: the segment's bytes, prefixed, with ffmpeg-style progress."""
    data = stdin.read()
    cache["n"] = cache.get("n", 0) + 1
    if data == b"boom":
        raise ValueError("bad segment")
    stderr.write("  Duration: 00:00:02.00, start: 0.000000, bitrate: N/A\n")
    stderr.write(f"frame=   50 fps= 25 q=5.0 size=N/A time=00:00:02.00 bitrate=N/A speed=1.00x\n")
    stdout.write(b"GPU" + str(dev).encode() + b":" + data + (b":trace" if opts.trace else b"")
                 + b":%d" % cache["n"])
    return 7 if data == b"rc7" else 0


def run_segment(argv, src, dst):
    seen = []
    with open(src, "rb") as fi, open(dst, "wb") as fo:
        p = D.FFMPEGProc(argv, stdin=fi, stdout=fo, update_callback=lambda *a: seen.append(a))
        rc = p.run()
    return rc, p, seen


def test_client_hands_segment_to_resident_encoder(client, tmp_path, monkeypatch):
    """The dispatcher's per-segment process for gpu:0 is mjg_client; the resident encoder
    reads the client's stdin, writes its stdout and stderr, and the client exits with the
    segment's code.  One encoder context (cache) serves consecutive segments."""
    name = socket_name(client)
    srv = R.Resident(0, R.listen(name), idle=60, run=fake_run)
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    try:
        argv = D.worker_argv("gpu:0", ["-c:v", "mjpeg", "-q:v", "5"], resident=True)
        assert argv[:3] == [client, "--device", "0"] and argv[-5:] == ["--", "-c:v", "mjpeg", "-q:v", "5"]
        for i, body in enumerate([b"seg-a", b"seg-b"]):
            (tmp_path / f"in{i}").write_bytes(body)
            rc, p, seen = run_segment(argv, tmp_path / f"in{i}", tmp_path / f"out{i}")
            assert rc == 0 and (tmp_path / f"out{i}").read_bytes() == b"GPU0:" + body + b":%d" % (i + 1)
            assert p.duration == 2.0 and seen and seen[0][:3] == (50, 25, 2.0)
        (tmp_path / "rc").write_bytes(b"rc7")
        assert run_segment(argv, tmp_path / "rc", tmp_path / "out_rc")[0] == 7
        (tmp_path / "boom").write_bytes(b"boom")
        rc, p, _ = run_segment(argv, tmp_path / "boom", tmp_path / "out_boom")
        assert rc == 1 and "gpu:0: ValueError: bad segment" in p.stderr
        monkeypatch.setenv("MJG_WORKER_TRACE", "1")  # the client's MJG_* settings travel
        rc, _, _ = run_segment(argv, tmp_path / "in0", tmp_path / "out_t")
        assert rc == 0 and (tmp_path / "out_t").read_bytes().startswith(b"GPU0:seg-a:trace")
    finally:
        assert subprocess.run([client, "--device", "0", "--shutdown"]).returncode == 0
        th.join(10)
    assert not th.is_alive()
    assert subprocess.run([client, "--device", "0", "--shutdown"]).returncode == 0  # none runs: 0


def test_concurrent_clients_share_one_encoder(client, tmp_path):
    """Two TaskThreads on the same GPU (-H gpu:0 -H gpu:0): both segments are served at once,
    each with an encoder context of its own."""
    name = socket_name(client)
    gate = threading.Barrier(2, timeout=10)

    def slow_run(dev, args, stdin, stdout, stderr, cache, opts):
        gate.wait()  # both requests are inside run() together
        return fake_run(dev, args, stdin, stdout, stderr, cache, opts)

    srv = R.Resident(0, R.listen(name), idle=60, run=slow_run)
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    try:
        argv = D.worker_argv("gpu:0", [], resident=True)
        res = {}
        for i in range(2):
            (tmp_path / f"in{i}").write_bytes(b"x%d" % i)
        ts = [threading.Thread(target=lambda i=i: res.__setitem__(i, run_segment(argv, tmp_path / f"in{i}",
                                                                                   tmp_path / f"out{i}")[0]))
              for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(20)
        assert res == {0: 0, 1: 0}
        assert sorted((tmp_path / f"out{i}").read_bytes() for i in range(2)) == [b"GPU0:x0:1", b"GPU0:x1:1"]
    finally:
        subprocess.run([client, "--device", "0", "--shutdown"])
        th.join(10)


def test_client_starts_an_encoder_when_none_listens(client, tmp_path):
    """No encoder listening: the client starts `python -m ffmpeg_distributed_amd.resident`
    (a new session whose stdio is its log, so the dispatcher still sees EOF when the client
    exits), hands over the segment and relays its exit code.  Without a GPU the encode fails
    loudly (no CPU path): exit 1 and the error on the segment's stderr."""
    from ffmpeg_distributed_amd.container import MkvWriter
    from fractions import Fraction
    seg = tmp_path / "seg.mkv"
    with open(seg, "wb") as f:
        w = MkvWriter(f, 16, 16, Fraction(25), codec="V_UNCOMPRESSED", colour_space=b"I420")
        w.write_frame(bytes(16 * 16 * 3 // 2))
        w.close()
    argv = [client, "--device", "7", "--python", sys.executable, "--idle", "20", "--",
            "-c:v", "mjpeg", "-q:v", "5", "-dct", "int", "-huffman", "default", "-bitexact"]
    name = socket_name(client, "7")
    t0 = time.monotonic()
    try:
        rc, p, _ = run_segment(argv, seg, tmp_path / "out.mkv")
        assert time.monotonic() - t0 < 60
        assert rc == 1 and "gpu:7:" in p.stderr, p.stderr
        # the encoder stays for the next segment
        assert subprocess.run(["python3", "-c", f"import socket; s = socket.socket(socket.AF_UNIX); "
                               f"s.connect('\\0{name}')"]).returncode == 0
    finally:
        assert subprocess.run([client, "--device", "7", "--shutdown"]).returncode == 0
    for _ in range(100):  # the encoder exits after the shutdown request
        r = subprocess.run(["python3", "-c", f"import socket; s = socket.socket(socket.AF_UNIX); "
                            f"s.connect('\\0{name}')"], capture_output=True)
        if r.returncode != 0:
            break
        time.sleep(0.1)
    assert r.returncode != 0


def test_worker_argv_resident_switch(client, monkeypatch):
    args = ["-q:v", "5"]
    assert D.worker_argv("gpu:2", args, resident=False) == [sys.executable, "-m", "ffmpeg_distributed_amd.worker",
                                                            "--device", "2", *args]
    monkeypatch.setenv("MJG_RESIDENT", "0")
    assert D.worker_argv("gpu:2", args)[:3] == [sys.executable, "-m", "ffmpeg_distributed_amd.worker"]
    monkeypatch.setenv("MJG_RESIDENT", "1")
    assert D.worker_argv("gpu:2", args) == [client, "--device", "2", "--python", sys.executable, "--", *args]
    assert D.server_argv("gpu:2", args)[-1] == "--serve"


def test_resident_passthrough_progress_reaches_the_client(client, tmp_path, monkeypatch):
    """A non-GPU profile in the resident encoder runs the real worker.run, which runs the
    reference's ffmpeg command (here the tests/shims stand-in) on the segment's descriptors:
    ffmpeg's own Duration / frame= lines and its output reach the client's stderr / stdout,
    not the encoder's log (worker.passthrough inherited the resident's stderr)."""
    monkeypatch.setenv("PATH", os.path.join(ROOT, "tests", "shims") + os.pathsep + os.environ["PATH"])
    name = socket_name(client)
    srv = R.Resident(0, R.listen(name), idle=60)  # run = worker.run
    th = threading.Thread(target=srv.serve, daemon=True)
    th.start()
    try:
        argv = D.worker_argv("gpu:0", ["-c:v", "libx264", "-crf", "18"], resident=True)
        (tmp_path / "in").write_bytes(b"SEGMENT")
        rc, p, seen = run_segment(argv, tmp_path / "in", tmp_path / "out")
        assert rc == 0, p.stderr
        assert (tmp_path / "out").read_bytes() == b"ENC[SEGMENT]"
        assert p.duration == 10.0 and [s[0] for s in seen] == [50, 100]
        assert "gpu:0: " in p.stderr and "running ffmpeg on the CPU" in p.stderr
        monkeypatch.setenv("PATH", "/nonexistent")  # no ffmpeg: the message is the segment's too
        rc, p, _ = run_segment(argv, tmp_path / "in", tmp_path / "out2")
        assert rc == 127 and "ffmpeg not found" in p.stderr
    finally:
        subprocess.run([client, "--device", "0", "--shutdown"])
        th.join(10)


def test_client_reconnects_when_a_connection_closes_before_the_ack(client, tmp_path):
    """An encoder that closes a queued connection unread (its idle exit racing a client) ends
    that connection before the 'A' acknowledgement: nothing of the segment was read, so the
    client connects again and the segment is encoded once, with exit code 0."""
    name = socket_name(client)
    sock = R.listen(name)
    dropped = []

    def serve():
        conn, _ = sock.accept()  # the first connection: closed unread
        dropped.append(1)
        conn.close()
        R.Resident(0, sock, idle=60, run=fake_run).serve()

    th = threading.Thread(target=serve, daemon=True)
    th.start()
    try:
        argv = D.worker_argv("gpu:0", ["-q:v", "5"], resident=True)
        (tmp_path / "in").write_bytes(b"seg")
        rc, p, _ = run_segment(argv, tmp_path / "in", tmp_path / "out")
        assert rc == 0 and dropped == [1], p.stderr
        assert (tmp_path / "out").read_bytes() == b"GPU0:seg:1"
    finally:
        subprocess.run([client, "--device", "0", "--shutdown"])
        th.join(10)


def test_client_log_is_private(client):
    """The encoder's log lives in a 0700 directory of this user (no symlink followed)."""
    import stat
    d = f"/tmp/mjg-{os.getuid()}"
    subprocess.run([client, "--device", "0", "--socket-name"], check=True, capture_output=True)
    if os.path.exists(d):
        st = os.lstat(d)
        assert stat.S_ISDIR(st.st_mode) and st.st_uid == os.getuid() and (st.st_mode & 0o077) == 0
