"""The gpu:N worker end to end on the GPU: a segment in (YUV4MPEG2 or raw Matroska), a
V_MJPEG Matroska segment out, every packet byte-identical to the CPU oracle's encode
of the same frame (oracle/mjpeg_oracle.c restating ffmpeg's mjpeg/swscale path)."""
import io
import json
from fractions import Fraction

import numpy as np
import pytest

from ffmpeg_distributed_amd import container, profile, worker
from ffmpeg_distributed_amd.encoder import split_i420
from ffmpeg_distributed_amd.testsrc import testsrc2_i420 as make_testsrc
from oracle import oracle

pytestmark = pytest.mark.gpu

ARGS = "-c:v mjpeg -q:v {q} -dct int -huffman default -bitexact".split()


def _args(q, scale=None, huffman="default"):
    a = [x.format(q=q) for x in ARGS]
    if huffman is None:  # no -huffman: FFmpeg's default, optimal
        a = a[:6] + a[8:]
    else:
        a[7] = huffman
    return (["-vf", f"scale={scale[0]}:{scale[1]}:flags=bicubic"] if scale else []) + a


def _run(data, args, monkeypatch, batch=None):
    if batch:
        monkeypatch.setattr(worker, "BATCH", batch)
    out, err = io.BytesIO(), io.StringIO()
    rc = worker.run(0, args, stdin=io.BytesIO(data), stdout=out, stderr=err)
    assert rc == 0, err.getvalue()
    r = container.MkvReader(io.BytesIO(out.getvalue()))
    return r, [d for _, d in r.frames(1)], err.getvalue()


def _y4m(frames, w, h, extra=""):
    b = io.BytesIO()
    b.write(f"YUV4MPEG2 W{w} H{h} F25:1 Ip A1:1 C420jpeg{extra}\n".encode())
    for f in frames:
        b.write(b"FRAME\n" + f.tobytes())
    return b.getvalue()


@pytest.mark.parametrize("w,h,scale,q,n,batch", [
    (160, 96, None, 5, 11, 4),            # batches of 4 with a ragged tail
    (176, 100, (96, 54), 3, 6, 32),       # downscale, odd chroma height
    (64, 48, (130, 74), 9, 5, 2),         # upscale
])
def test_worker_y4m_matches_oracle(w, h, scale, q, n, batch, monkeypatch):
    frames = [make_testsrc(w, h, i) for i in range(n)]
    r, packets, err = _run(_y4m(frames, w, h), _args(q, scale), monkeypatch, batch)
    dw, dh = scale or (w, h)
    info = r.info(1)
    assert (info.width, info.height, info.codec, info.fps) == (dw, dh, "V_MJPEG", Fraction(25))
    assert len(packets) == n
    for i, f in enumerate(frames):
        y, u, v = split_i420(f, w, h)
        sar = profile.scaled_sar((1, 1), (w, h), (dw, dh))
        ref = oracle.encode_frame(y, u, v, dw, dh, full_range=False, qscale=q, sar=sar)
        assert packets[i] == ref, f"frame {i}"
    assert f"frame={n:5d}" in err


def test_worker_raw_mkv_full_range(monkeypatch):
    w, h, n = 96, 64, 7
    frames = [make_testsrc(w, h, 3 + i) for i in range(n)]
    buf = io.BytesIO()
    wr = container.MkvWriter(buf, w, h, Fraction(30000, 1001), codec="V_UNCOMPRESSED",
                             colour_space=b"I420", colour_range=2)
    for f in frames:
        wr.write_frame(f.tobytes())
    wr.close()
    r, packets, _ = _run(buf.getvalue(), _args(4), monkeypatch, 3)
    assert r.info(1).fps == Fraction(30000, 1001)
    for i, f in enumerate(frames):
        y, u, v = split_i420(f, w, h)
        assert packets[i] == oracle.encode_frame(y, u, v, full_range=True, qscale=4, sar=(1, 1))


@pytest.mark.parametrize("huffman", ["optimal", None])
def test_worker_huffman_optimal(huffman, monkeypatch):
    """-huffman optimal, explicit or by default (no -huffman, as BASELINE configs[0] runs)."""
    w, h, n, q = 144, 80, 5, 5
    frames = [make_testsrc(w, h, 7 + i) for i in range(n)]
    r, packets, _ = _run(_y4m(frames, w, h), _args(q, huffman=huffman), monkeypatch, 2)
    for i, f in enumerate(frames):
        y, u, v = split_i420(f, w, h)
        ref = oracle.encode_frame(y, u, v, full_range=False, qscale=q, sar=(1, 1), huffman="optimal")
        assert packets[i] == ref, f"frame {i}"


@pytest.mark.parametrize("fourcc,chroma,extra", [
    (b"Y42B", "422", ["-slices", "4"]),                       # 4:2:2 + RST layout
    (b"444P", "444", ["-thread_type", "slice", "-pix_fmt", "yuvj444p"]),
    (b"I420", "420", ["-threads", "1", "-slices", "2", "-huffman", "optimal"]),  # slices force default
])
def test_worker_raw_mkv_422_444_rst(fourcc, chroma, extra, monkeypatch):
    """Raw 4:2:2 / 4:4:4 Matroska segments and slice-threaded remote_args:
    the worker keeps the input sampling and writes the RST layout."""
    from ffmpeg_distributed_amd.encoder import i420_frame_bytes
    w, h, n, q = 112, 72, 5, 4
    fb = i420_frame_bytes(w, h, chroma)
    rng = np.random.default_rng(4)
    frames = [np.clip(rng.normal(128, 40, fb), 0, 255).astype(np.uint8) for _ in range(n)]
    buf = io.BytesIO()
    wr = container.MkvWriter(buf, w, h, Fraction(25), codec="V_UNCOMPRESSED", colour_space=fourcc,
                             colour_range=1)
    for f in frames:
        wr.write_frame(f.tobytes())
    wr.close()
    args = [x.format(q=q) for x in ARGS[:6]] + ["-bitexact"] + extra
    r, packets, _ = _run(buf.getvalue(), args, monkeypatch, 2)
    assert len(packets) == n
    for i, f in enumerate(frames):
        y, u, v = split_i420(f, w, h, chroma)
        ref = oracle.encode_frame(y, u, v, full_range=False, qscale=q, sar=(1, 1), chroma=chroma, rst=True)
        assert packets[i] == ref, f"frame {i}"


def test_worker_serve_reuses_context_across_segments(tmp_path):
    """worker.serve (dispatcher -P): segments of one shape share the encoder context and
    batch buffers, a segment of another shape gets a new one; every packet still equals
    the oracle's encode of its frame."""
    segs = [(96, 64, 5, 3), (96, 64, 5, 9), (80, 48, 5, 4), (96, 64, 5, 2)]
    reqs, want = [], []
    for i, (w, h, q, n) in enumerate(segs):
        frames = [make_testsrc(w, h, 11 * i + k) for k in range(n)]
        buf = io.BytesIO()
        wr = container.MkvWriter(buf, w, h, Fraction(25), codec="V_UNCOMPRESSED", colour_space=b"I420")
        for f in frames:
            wr.write_frame(f.tobytes())
        wr.close()
        (tmp_path / f"in{i}.mkv").write_bytes(buf.getvalue())
        reqs.append(json.dumps([f"{tmp_path}/in{i}.mkv", f"{tmp_path}/out{i}.mkv"]) + "\n")
        want.append([oracle.encode_frame(*split_i420(f, w, h), full_range=False, qscale=q, sar=(1, 1))
                     for f in frames])
    err = io.StringIO()
    assert worker.serve(0, _args(5), requests=io.StringIO("".join(reqs)), stderr=err) == 0
    assert err.getvalue().count(worker.SERVE_DONE + "0") == len(segs), err.getvalue()
    for i in range(len(segs)):
        r = container.MkvReader(io.BytesIO((tmp_path / f"out{i}.mkv").read_bytes()))
        assert [d for _, d in r.frames(1)] == want[i], f"segment {i}"


def _raw_mkv(frames, w, h):
    buf = io.BytesIO()
    wr = container.MkvWriter(buf, w, h, Fraction(25), codec="V_UNCOMPRESSED", colour_space=b"I420")
    for f in frames:
        wr.write_frame(f.tobytes())
    wr.close()
    return buf.getvalue()


def test_worker_serve_segment_failing_mid_stream(tmp_path, monkeypatch):
    """A segment that fails mid-stream (its file ends inside a frame after several batches
    were submitted) reports rc 1; the reader thread and its positional reads are stopped
    before the batch buffers are freed, and the next segments come out byte-exact."""
    monkeypatch.setattr(worker, "BATCH", 2)
    w, h, q = 96, 64, 5
    good = [[make_testsrc(w, h, 5 * i + k) for k in range(7)] for i in range(3)]
    bad = _raw_mkv([make_testsrc(w, h, 100 + k) for k in range(9)], w, h)
    (tmp_path / "bad.mkv").write_bytes(bad[: len(bad) - w * h])  # last frame cut short
    reqs = [json.dumps([str(tmp_path / "in0.mkv"), str(tmp_path / "out0.mkv")]),
            json.dumps([str(tmp_path / "bad.mkv"), str(tmp_path / "outbad.mkv")]),
            json.dumps([str(tmp_path / "in1.mkv"), str(tmp_path / "out1.mkv")]),
            json.dumps([str(tmp_path / "in2.mkv"), str(tmp_path / "out2.mkv")])]
    for i, frames in enumerate(good):
        (tmp_path / f"in{i}.mkv").write_bytes(_raw_mkv(frames, w, h))
    err = io.StringIO()
    assert worker.serve(0, _args(q), requests=io.StringIO("\n".join(reqs) + "\n"), stderr=err) == 0
    done = [l for l in err.getvalue().splitlines() if l.startswith(worker.SERVE_DONE)]
    assert [int(l[len(worker.SERVE_DONE):]) for l in done] == [0, 1, 0, 0], err.getvalue()
    assert "ends inside a frame" in err.getvalue()
    for i, frames in enumerate(good):
        r = container.MkvReader(io.BytesIO((tmp_path / f"out{i}.mkv").read_bytes()))
        want = [oracle.encode_frame(*split_i420(f, w, h), full_range=False, qscale=q, sar=(1, 1)) for f in frames]
        assert [d for _, d in r.frames(1)] == want, f"segment {i}"


def test_resident_client_segments_match_oracle(tmp_path):
    """The dispatcher's per-segment process for -H gpu:0 is mjg_client, which hands the
    segment to the GPU's resident encoder (started on first use): every packet equals the
    oracle's encode, a failing segment exits 1 with its error on stderr, and the next segment
    of another shape comes out byte-exact too (fd.py:131-141 contract)."""
    import subprocess
    import sys
    from ffmpeg_distributed_amd import build, dispatcher as D
    client = build.build_client()
    cases = [(96, 64, 5, 3), (96, 64, 5, 9), (80, 48, 5, 4)]
    argv = D.worker_argv("gpu:0", _args(5), resident=True)
    assert argv[0] == client
    try:
        for i, (w, h, q, n) in enumerate(cases):
            frames = [make_testsrc(w, h, 13 * i + k) for k in range(n)]
            (tmp_path / f"in{i}.mkv").write_bytes(_raw_mkv(frames, w, h))
            seen = []
            with open(tmp_path / f"in{i}.mkv", "rb") as fi, open(tmp_path / f"out{i}.mkv", "wb") as fo:
                p = D.FFMPEGProc(argv, stdin=fi, stdout=fo, update_callback=lambda *a: seen.append(a))
                assert p.run() == 0, p.stderr
            assert seen and seen[-1][0] == n  # the final progress line counts every frame
            r = container.MkvReader(io.BytesIO((tmp_path / f"out{i}.mkv").read_bytes()))
            want = [oracle.encode_frame(*split_i420(f, w, h), full_range=False, qscale=q, sar=(1, 1)) for f in frames]
            assert [d for _, d in r.frames(1)] == want, f"segment {i}"
            if i == 0:
                bad = _raw_mkv([make_testsrc(96, 64, 50 + k) for k in range(4)], 96, 64)
                (tmp_path / "bad.mkv").write_bytes(bad[: len(bad) - 100])
                with open(tmp_path / "bad.mkv", "rb") as fi, open(tmp_path / "outbad.mkv", "wb") as fo:
                    p = D.FFMPEGProc(argv, stdin=fi, stdout=fo)
                    assert p.run() == 1 and "ends inside a frame" in p.stderr
    finally:
        subprocess.run([client, "--device", "0", "--shutdown"], timeout=60)
        _wait_resident_gone(client, "0")


def _wait_resident_gone(client, dev, timeout=30.0):
    """The resident encoder has exited (its socket refuses connections)."""
    import socket
    import subprocess
    import time
    name = subprocess.run([client, "--device", dev, "--socket-name"], capture_output=True, text=True).stdout.strip()
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout:
        s = socket.socket(socket.AF_UNIX)
        try:
            s.connect("\0" + name)
        except OSError:
            return
        finally:
            s.close()
        time.sleep(0.2)
    raise AssertionError("resident encoder still running after its shutdown")
