"""The N>1 path on the CPU: two gloo ranks run the same sharding / timed-region / max
reduction code bench.py runs over RCCL, and the dispatcher drives two `gpu:N` hosts
(worker stubbed) so segments are split across devices with no collective."""
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from ffmpeg_distributed_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    done = []
    segs = shard.segments_for_rank(12, rank, world)
    # rank 1 is slower: the job time must be its time, seen identically by both ranks
    dt = shard.timed_region(lambda s: (done.append(segs[s]), time.sleep(0.01 * (1 + rank))),
                            1, len(segs) - 1, dist.barrier, lambda: None)
    mx = shard.max_over_ranks(dt, dist)
    q.put((rank, segs, done, dt, mx))
    dist.barrier()
    dist.destroy_process_group()


def test_two_gloo_ranks_shard_and_reduce():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    all_segs = sorted(s for _, segs, _, _, _ in res for s in segs)
    assert all_segs == list(range(12))                     # every segment exactly once
    assert all(done == segs for _, segs, done, _, _ in res)
    mx = {r[4] for r in res}
    assert len(mx) == 1 and mx.pop() == pytest.approx(max(r[3] for r in res))
    # the closing barrier makes the fast rank wait: both see at least the slow rank's work
    slow_work = (len(res[1][1]) - 1) * 0.02
    assert min(r[3] for r in res) >= slow_work * 0.95


@pytest.mark.parametrize("n,world", [(0, 1), (1, 8), (300, 8), (7, 3)])
def test_round_robin_partition(n, world):
    parts = [shard.segments_for_rank(n, r, world) for r in range(world)]
    assert sorted(s for p in parts for s in p) == list(range(n))
    assert max(map(len, parts)) - min(map(len, parts)) <= 1


def test_single_rank_max_is_identity():
    assert shard.max_over_ranks(1.25) == 1.25


STUB_WORKER = r"""
import sys, time
dev = sys.argv[sys.argv.index("--device") + 1]
data = sys.stdin.read()
time.sleep(0.2)
sys.stderr.write("  Duration: 00:00:02.00, start: 0.000000, bitrate: N/A\n")
sys.stderr.write("frame=   50 fps= 25 q=5.0 size=N/A time=00:00:02.00 bitrate=N/A speed=1.00x\n")
sys.stdout.write("GPU" + dev + "[" + data + "]")
"""


def test_dispatcher_spreads_segments_over_gpu_hosts(tmp_path, monkeypatch):
    """-H gpu:0 -H gpu:1: every segment is encoded exactly once, by one of the two
    device workers, pulled dynamically from the shared queue; no collective involved."""
    import sys
    from ffmpeg_distributed_amd import dispatcher as D
    here = os.path.dirname(os.path.abspath(__file__))
    monkeypatch.setenv("PATH", os.path.join(here, "shims") + os.pathsep + os.environ["PATH"])
    monkeypatch.setenv("SHIM_SEGMENTS", "6")
    monkeypatch.chdir(tmp_path)
    stub = tmp_path / "stub_worker.py"
    stub.write_text(STUB_WORKER)
    real = D.worker_argv

    def argv(host, args, resident=None):
        a = real(host, args, resident=False)
        assert a[:3] == [sys.executable, "-m", "ffmpeg_distributed_amd.worker"]
        return [sys.executable, str(stub)] + a[3:]

    monkeypatch.setattr(D, "worker_argv", argv)
    (tmp_path / "input.mp4").write_text("RAW")
    D.encode(["gpu:0", "gpu:1"], "input.mp4", "out.mkv", 2, "-c:v mjpeg -q:v 5", "-an",
             tmp_dir="segs", keep_tmp=True)
    outs = sorted(os.listdir(tmp_path / "segs" / "out"))
    assert outs == [f"{i:08d}.mkv" for i in range(6)]
    bodies = [(tmp_path / "segs" / "out" / o).read_text() for o in outs]
    assert all(b.startswith(("GPU0[SEG", "GPU1[SEG")) for b in bodies)
    assert {b[:4] for b in bodies} == {"GPU0", "GPU1"}
    assert (tmp_path / "out.mkv").read_text() == "|".join(bodies)


STUB_SERVER = r"""
import json, os, sys, time
dev = sys.argv[sys.argv.index("--device") + 1]
assert sys.argv[-1] == "--serve"
with open(os.environ["STUB_LOG"], "a") as log:
    log.write(f"start {dev}\n")
for line in sys.stdin:
    src, dst = json.loads(line)
    data = open(src).read()
    time.sleep(0.05)
    if data.startswith("SEG2:") and not os.path.exists("crashed"):
        open("crashed", "w").close()
        os._exit(3)                      # the server dies mid-segment
    rc = 0
    if data.startswith("SEG4:") and not os.path.exists("failed"):
        open("failed", "w").close()
        rc = 1                           # one segment fails, the server lives on
    else:
        with open(dst, "w") as f:
            f.write("GPU" + dev + "[" + data + "]")
    sys.stderr.write("  Duration: 00:00:02.00, start: 0.000000, bitrate: N/A\n")
    sys.stderr.write("frame=   50 fps= 25 q=5.0 size=N/A time=00:00:02.00 bitrate=N/A speed=1.00x\n")
    sys.stderr.write(f"mjg-serve: segment done rc={rc}\n")
    sys.stderr.flush()
"""


def test_dispatcher_persistent_gpu_workers(tmp_path, monkeypatch):
    """-P: one long-lived worker per gpu:N entry takes segment after segment over its request
    pipe; a segment it fails is re-queued like a failed per-segment worker, and a server that
    dies fails its segment and is started again."""
    import sys
    from ffmpeg_distributed_amd import dispatcher as D
    here = os.path.dirname(os.path.abspath(__file__))
    monkeypatch.setenv("PATH", os.path.join(here, "shims") + os.pathsep + os.environ["PATH"])
    monkeypatch.setenv("SHIM_SEGMENTS", "8")
    monkeypatch.setenv("STUB_LOG", str(tmp_path / "starts.log"))
    monkeypatch.chdir(tmp_path)
    stub = tmp_path / "stub_server.py"
    stub.write_text(STUB_SERVER)
    real = D.worker_argv

    def argv(host, args, resident=None):
        a = real(host, args, resident=False)
        assert a[:3] == [sys.executable, "-m", "ffmpeg_distributed_amd.worker"]
        return [sys.executable, str(stub)] + a[3:]

    monkeypatch.setattr(D, "worker_argv", argv)
    (tmp_path / "input.mp4").write_text("RAW")
    D.encode(["gpu:0", "gpu:1"], "input.mp4", "out.mkv", 2, "-c:v mjpeg -q:v 5", "-an",
             tmp_dir="segs", keep_tmp=True, persistent_gpu_workers=True)
    outs = sorted(os.listdir(tmp_path / "segs" / "out"))
    assert outs == [f"{i:08d}.mkv" for i in range(8)]
    bodies = [(tmp_path / "segs" / "out" / o).read_text() for o in outs]
    assert all(b.startswith(("GPU0[SEG", "GPU1[SEG")) for b in bodies)
    assert [b[5:9] for b in bodies] == [f"SEG{i}" for i in range(8)]
    assert (tmp_path / "out.mkv").read_text() == "|".join(bodies)
    starts = (tmp_path / "starts.log").read_text().split("\n")[:-1]
    assert sorted(set(starts)) == ["start 0", "start 1"]
    assert len(starts) == 3  # one server per host, plus the restart after the crash


def test_worker_serve_protocol(tmp_path, monkeypatch):
    """worker.serve: one request line per segment, the segment's files opened for run(),
    the done line carries run()'s exit code (an exception is a failed segment, rc 1)."""
    import io
    import json
    from ffmpeg_distributed_amd import worker
    calls = []

    def fake_run(dev, args, stdin, stdout, stderr, cache, batch_bytes=None):
        data = stdin.read()
        calls.append((dev, args, data, id(cache)))
        if data == b"boom":
            raise ValueError("bad segment")
        stdout.write(b"out:" + data)
        stderr.write("frame=    1 fps=  1 q=5.0 size=N/A time=00:00:00.04 bitrate=N/A speed=1.00x\n")
        return 0 if data != b"rc7" else 7

    monkeypatch.setattr(worker, "run", fake_run)
    reqs = []
    for i, body in enumerate([b"a", b"boom", b"rc7", b"b"]):
        (tmp_path / f"in{i}").write_bytes(body)
        reqs.append(json.dumps([f"{tmp_path}/in{i}", f"{tmp_path}/out{i}"]) + "\n")
    err = io.StringIO()
    assert worker.serve(2, ["-q:v", "5"], requests=io.StringIO("".join(reqs)), stderr=err) == 0
    done = [l for l in err.getvalue().splitlines() if l.startswith(worker.SERVE_DONE)]
    assert [int(l[len(worker.SERVE_DONE):]) for l in done] == [0, 1, 7, 0]
    assert "ValueError: bad segment" in err.getvalue()
    assert (tmp_path / "out0").read_bytes() == b"out:a" and (tmp_path / "out3").read_bytes() == b"out:b"
    assert len({c[3] for c in calls}) == 1 and all(c[:2] == (2, ["-q:v", "5"]) for c in calls)


def test_serve_request_survives_any_path(tmp_path, monkeypatch):
    """Paths with tabs, newlines and quotes go through the one-line serve protocol intact."""
    import io
    from ffmpeg_distributed_amd import dispatcher as D, worker
    seen = []

    def fake_run(dev, args, stdin, stdout, stderr, cache, batch_bytes=None):
        seen.append(stdin.read())
        stdout.write(b"ok")
        return 0

    monkeypatch.setattr(worker, "run", fake_run)
    d = tmp_path / "a\tb\nc 'q\""
    d.mkdir()
    (d / "in.mkv").write_bytes(b"payload")
    req = D.serve_request(str(d / "in.mkv"), str(d / "out.mkv"))
    assert req.count("\n") == 1 and req.endswith("\n")
    err = io.StringIO()
    assert worker.serve(0, [], requests=io.StringIO(req), stderr=err) == 0
    assert seen == [b"payload"] and (d / "out.mkv").read_bytes() == b"ok"
    assert err.getvalue().strip().endswith(worker.SERVE_DONE + "0")


def test_ffmpegproc_stop_is_prompt_while_child_is_silent():
    """stop() ends the stderr follow loop within a poll period even when the child writes
    nothing (fd.py:61-68 polls with a timeout); the child itself is not killed (fd.py:56-57)."""
    import sys
    import threading
    from ffmpeg_distributed_amd import dispatcher as D
    p = D.FFMPEGProc([sys.executable, "-c", "import time, sys; sys.stderr.write('hello\\n'); "
                      "sys.stderr.flush(); time.sleep(30)"])
    t = threading.Thread(target=p.run)
    t0 = time.monotonic()
    t.start()
    time.sleep(0.5)
    p.stop()
    t.join(5)
    try:
        assert not t.is_alive()
        assert time.monotonic() - t0 < 4
        assert "hello" in p.stderr
    finally:
        p.proc.kill()
        p.proc.wait()


def test_gpu_server_stop_fails_the_running_segment(tmp_path):
    """A stop event set while a persistent server works on a segment closes the server and
    fails the segment instead of waiting for it."""
    import sys
    import threading
    from ffmpeg_distributed_amd import dispatcher as D
    stub = tmp_path / "silent.py"
    stub.write_text("import sys, time\nfor line in sys.stdin:\n    time.sleep(60)\n")
    srv = D.GpuServer("gpu:0")
    srv._start = lambda args: (setattr(srv, "args", list(args)), setattr(srv, "proc", __import__("subprocess").Popen(
        [sys.executable, str(stub)], stdin=-1, stdout=-3, stderr=-1, universal_newlines=True, bufsize=1)),
        setattr(srv, "feed", D._LineFeed(srv.proc.stderr)))
    stop = threading.Event()
    threading.Timer(0.3, stop.set).start()
    t0 = time.monotonic()
    rc = srv.run_task(D.Task(str(tmp_path / "i"), str(tmp_path / "o"), []), stop=stop)
    assert rc == 1 and time.monotonic() - t0 < 5 and srv.proc is None
