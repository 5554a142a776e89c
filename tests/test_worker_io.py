"""Host side of the gpu:N worker: remote_args profile parsing, the native Matroska /
YUV4MPEG2 segment I/O, the decoder-child replay and the passthrough to real ffmpeg.
No GPU (the encode itself is covered by test_gpu_worker.py)."""
import io
import json
import os
import subprocess
import sys
import tempfile
import textwrap
from fractions import Fraction

import numpy as np
import pytest

from ffmpeg_distributed_amd import container, profile, worker
from ffmpeg_distributed_amd.testsrc import testsrc2_i420 as make_testsrc

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
NORTH_STAR = "-vf scale=1920:1080:flags=bicubic -c:v mjpeg -q:v 5 -dct int -huffman default -bitexact"


# ------------------------------------------------------------------ profile
def test_profile_north_star():
    p = profile.parse(NORTH_STAR)
    assert p.scale == (1920, 1080) and p.qscale == 5 and p.sws_flags == ("bicubic",)
    p = profile.parse("-c:v mjpeg -q:v 2 -dct int -huffman default -flags +bitexact -an")
    assert p.scale is None and p.qscale == 2 and p.huffman == "default"


@pytest.mark.parametrize("args,huff", [
    ("-c:v mjpeg -q:v 5 -dct int -huffman optimal -bitexact", "optimal"),
    ("-c:v mjpeg -q:v 5 -dct int -bitexact", "optimal"),  # FFmpeg's default mode
    ("-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact", "default"),
])
def test_profile_huffman_modes(args, huff):
    assert profile.parse(args).huffman == huff


@pytest.mark.parametrize("extra,rst", [
    ("", False),                                   # default: frame threading, no DRI/RST
    ("-threads 8", False),
    ("-slices 1", False),
    ("-slices 4", True),                           # slice_context_count = -slices
    ("-threads 1 -slices 2", True),
    ("-thread_type slice", True),                  # -threads auto (> 1) slice threads
    ("-thread_type slice -threads 4", True),
    ("-thread_type slice -threads 1", False),
    ("-thread_type slice+frame -threads 4", False),  # frame threading wins for encoders
    ("-thread_type frame", False),
])
def test_profile_slice_threading(extra, rst):
    p = profile.parse("-c:v mjpeg -q:v 5 -dct int -bitexact " + extra)
    assert p.rst == rst
    assert p.huffman == ("default" if rst else "optimal")   # slices force default tables


@pytest.mark.parametrize("pf,chroma", [("yuvj420p", "420"), ("yuvj422p", "422"), ("yuvj444p", "444")])
def test_profile_pix_fmt(pf, chroma):
    assert profile.parse(f"-c:v mjpeg -q:v 5 -dct int -bitexact -pix_fmt {pf}").chroma == chroma
    assert profile.parse("-c:v mjpeg -q:v 5 -dct int -bitexact").chroma is None


@pytest.mark.parametrize("q,expect", [(1, 2), (2, 2), (3, 3), (5, 5), (31, 31), (40, 31), (4.5, 5), (4.4, 4), (7.9, 8)])
def test_profile_qscale_mapping(q, expect):
    # update_qscale: lambda = q*118 (truncated), qscale = (lambda*139 + 8192) >> 14
    assert profile.effective_qscale(q) == expect


def test_boundary_flag_substitutions():
    """The substitutions INTEGRATION.md documents: every accepted -vf scale flag set (plain
    bicubic, BASELINE's own form; no flags= at all; bicubic+accurate_rnd+bitexact) is encoded
    by swscale's bitexact + accurate_rnd C path -- the encoder is always opened with
    sws_bitexact (the worker never passes another value) -- and -q:v goes through
    update_qscale with the qmin = 2 / qmax = 31 clip."""
    import inspect
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    base = "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact"
    for vf, flags in [("scale=1920:1080:flags=bicubic", ("bicubic",)),
                      ("scale=1920:1080", ("bicubic",)),
                      ("scale=w=1920:h=1080:flags=bicubic+accurate_rnd+bitexact",
                       ("bicubic", "accurate_rnd", "bitexact"))]:
        p = profile.parse(f"-vf {vf} {base}")
        assert p.scale == (1920, 1080) and p.sws_flags == flags
    assert inspect.signature(MjpegEncoder).parameters["sws_bitexact"].default is True
    with open(os.path.join(ROOT, "ffmpeg_distributed_amd", "worker.py")) as f:
        assert "sws_bitexact" not in f.read()
    for vf in ("scale=1920:1080:flags=bilinear", "scale=1920:1080:flags=bicubic+neighbor",
               "scale=1920:1080:flags=accurate_rnd"):
        assert profile.try_parse(f"-vf {vf} {base}")[0] is None
    # q < 2 clips to qmin 2; fractional -q:v truncates lambda first
    assert [profile.effective_qscale(q) for q in (0.5, 1, 1.9, 2, 2.5, 3, 31, 40)] == [2, 2, 2, 2, 3, 3, 31, 31]
    assert profile.parse("-c:v mjpeg -q:v 1 -dct int -bitexact").qscale == 2


@pytest.mark.parametrize("args", [
    "-c:v libx264 -crf 18",
    "-c:v mjpeg -q:v 5 -dct int -huffman zigzag -bitexact",
    "-c:v mjpeg -q:v 5 -huffman default -bitexact",                  # default dct is not int
    "-c:v mjpeg -q:v 5 -dct int -huffman default",                   # no -bitexact
    "-c:v mjpeg -b:v 10M -dct int -huffman default -bitexact",       # rate control
    "-vf scale=1920:-2 -c:v mjpeg -q:v 5 -dct int -huffman default -bitexact",
    "-vf scale=1280:720:flags=lanczos -c:v mjpeg -q:v 5 -dct int -huffman default -bitexact",
    "-vf scale=1280:720,hflip -c:v mjpeg -q:v 5 -dct int -huffman default -bitexact",
    "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact -pix_fmt gray",
    "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact -thread_type auto",
    "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact -slices many",
    # -fflags is a muxer flag: it does not make the encoder bitexact (the Lavc COM remains)
    "-c:v mjpeg -q:v 5 -dct int -huffman default -fflags +bitexact",
    # codec flags other than bitexact change the bitstream (+gray: flat chroma)
    "-c:v mjpeg -q:v 5 -dct int -huffman default -flags +gray+bitexact",
    "-c:v mjpeg -q:v 5 -dct int -huffman default -flags +bitexact+qscale",
    # bitexact switched off again
    "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact -flags -bitexact",
    "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact -fflags +genpts",
])
def test_profile_rejects_outside_gpu_path(args):
    prof, why = profile.try_parse(args)
    assert prof is None and why


@pytest.mark.parametrize("args", [
    "-c:v mjpeg -q:v 5 -dct int -flags +bitexact",
    "-c:v mjpeg -q:v 5 -dct int -flags:v bitexact",
    "-c:v mjpeg -q:v 5 -dct int -bitexact -fflags +bitexact",
    "-c:v mjpeg -q:v 5 -dct int -fflags +bitexact -flags +bitexact",
])
def test_profile_codec_bitexact_spellings(args):
    prof, why = profile.try_parse(args)
    assert prof is not None, why


# ------------------------------------------------------------------ matroska
def _mjpeg_like(i):
    return bytes([0xFF, 0xD8]) + bytes([i & 0xFF]) * (100 + 37 * i) + bytes([0xFF, 0xD9])


@pytest.mark.parametrize("fps", [Fraction(25), Fraction(30000, 1001), Fraction(60)])
def test_mkv_roundtrip(fps):
    buf = io.BytesIO()
    w = container.MkvWriter(buf, 1920, 1080, fps, sar=(4, 3))
    frames = [_mjpeg_like(i) for i in range(150)]      # > 1 s: several clusters
    for f in frames:
        w.write_frame(f)
    w.close()
    raw = buf.getvalue()
    assert raw[:4] == b"\x1a\x45\xdf\xa3" and raw.count(b"\x1f\x43\xb6\x75") >= 2
    r = container.MkvReader(io.BytesIO(raw))
    got = list(r.frames(1))
    assert [d for _, d in got] == frames
    assert [t for t, _ in got] == [round(Fraction(1000 * i) / fps) for i in range(150)]
    info = r.info(1)
    assert (info.width, info.height, info.codec) == (1920, 1080, "V_MJPEG")
    assert info.fps == fps
    assert info.sar == (4, 3)


def test_ebml_sizes():
    assert container._size_bytes(0) == b"\x80"
    assert container._size_bytes(126) == b"\xfe"
    assert container._size_bytes(127) == b"\x40\x7f"        # 0x7f alone would mean "unknown"
    assert container._size_bytes(16382) == b"\x7f\xfe"
    assert container._size_bytes(16383) == b"\x20\x3f\xff"
    for n in (0, 1, 126, 127, 300, 1 << 20, (1 << 28) + 5):
        v, ln = container._read_vint(io.BytesIO(container._size_bytes(n)), False)
        assert v == n and ln == len(container._size_bytes(n))


def _i420(w, h, n, seed=0):
    return np.stack([make_testsrc(w, h, seed + i) for i in range(n)])


def _y4m(frames, w, h, fps="25:1", extra=" Ip A1:1 C420jpeg XYSCSS=420JPEG"):
    out = io.BytesIO()
    out.write(f"YUV4MPEG2 W{w} H{h} F{fps}{extra}\n".encode())
    for f in frames:
        out.write(b"FRAME\n")
        out.write(f.tobytes())
    return out.getvalue()


def test_y4m_reader():
    w, h = 70, 38                                       # odd chroma: cw = 35, ch = 19
    fr = _i420(w, h, 5)
    data = _y4m(fr, w, h, "30000:1001", " Ip A16:15 C420mpeg2 XCOLORRANGE=FULL")
    rd = container.Y4MReader(io.BytesIO(data))
    assert (rd.info.width, rd.info.height, rd.info.fps, rd.info.sar, rd.info.full_range) == \
        (w, h, Fraction(30000, 1001), (16, 15), True)
    buf = np.zeros((8, fr.shape[1]), np.uint8)
    assert rd.read_into(buf, 3) == 3 and rd.read_into(buf[3:], 5) == 2
    np.testing.assert_array_equal(buf[:5], fr)


def test_y4m_rejects_unsupported_sampling():
    for c in (b"C411", b"Cmono", b"C444alpha", b"C420p10"):
        with pytest.raises(ValueError):
            container.Y4MReader(io.BytesIO(b"YUV4MPEG2 W16 H16 F25:1 " + c + b"\n"))


@pytest.mark.parametrize("tag,chroma,cw,ch", [(b"C422", "422", 35, 38), (b"C444", "444", 70, 38),
                                              (b"C420paldv", "420", 35, 19)])
def test_y4m_reader_422_444(tag, chroma, cw, ch):
    w, h = 70, 38
    rng = np.random.default_rng(1)
    fb = w * h + 2 * cw * ch
    fr = rng.integers(0, 256, (3, fb), dtype=np.uint8)
    rd = container.Y4MReader(io.BytesIO(_y4m(fr, w, h, extra=" Ip A1:1 " + tag.decode())))
    assert rd.info.chroma == chroma and rd.info.frame_bytes == fb
    buf = np.zeros((3, fb), np.uint8)
    assert rd.read_into(buf, 3) == 3
    np.testing.assert_array_equal(buf, fr)
    # the writer's header reads back to the same stream description
    hdr = container.y4m_header(rd.info)
    assert container.Y4MReader(io.BytesIO(hdr)).info == rd.info


@pytest.mark.parametrize("fourcc,chroma", [(b"Y42B", "422"), (b"444P", "444")])
def test_source_reads_uncompressed_mkv_422_444(fourcc, chroma):
    w, h = 48, 32
    fb = container.StreamInfo(w, h, chroma=chroma).frame_bytes
    fr = np.random.default_rng(2).integers(0, 256, (5, fb), dtype=np.uint8)
    src = worker.Source(io.BytesIO(_mkv_raw(fr, w, h, colour=fourcc)))
    assert src.child is None and src.info.chroma == chroma and src.info.frame_bytes == fb
    buf = np.zeros((8, fb), np.uint8)
    assert src.read_into(buf, 8) == 5
    np.testing.assert_array_equal(buf[:5], fr)


def _mkv_raw(frames, w, h, codec="V_UNCOMPRESSED", colour=b"I420", rng=1):
    buf = io.BytesIO()
    wr = container.MkvWriter(buf, w, h, Fraction(25), codec=codec, colour_space=colour, colour_range=rng)
    for f in frames:
        wr.write_frame(f.tobytes())
    wr.close()
    return buf.getvalue()


def test_source_reads_uncompressed_mkv():
    w, h = 48, 32
    fr = _i420(w, h, 7)
    src = worker.Source(io.BytesIO(_mkv_raw(fr, w, h, rng=2)))
    assert src.child is None and src.info.full_range and (src.info.width, src.info.height) == (w, h)
    buf = np.zeros((4, fr.shape[1]), np.uint8)
    out = []
    while True:
        n = src.read_into(buf, 4)
        out.extend(buf[:n].copy())
        if n < 4:
            break
    np.testing.assert_array_equal(np.stack(out), fr)


FAKE_DECODER = textwrap.dedent("""
    import sys
    sys.path.insert(0, {root!r})
    from ffmpeg_distributed_amd import container
    r = container.MkvReader(sys.stdin.buffer)
    i = r.info(1)
    o = sys.stdout.buffer
    o.write(b"YUV4MPEG2 W%d H%d F25:1 Ip A1:1 C420jpeg XCOLORRANGE=LIMITED\\n" % (i.width, i.height))
    for _, d in r.frames(1):
        o.write(b"FRAME\\n" + d[::-1][::-1])
""")


def test_source_decoder_child_gets_every_byte(monkeypatch, tmp_path):
    """Non-raw codecs go through a decoder child; the bytes the Matroska probe already
    consumed must be replayed to it (here the 'codec' is raw I420 under another name)."""
    w, h = 64, 48
    fr = _i420(w, h, 40)
    script = tmp_path / "fake_decoder.py"
    script.write_text(FAKE_DECODER.format(root=ROOT))
    monkeypatch.setattr(worker, "DECODE_ARGV", [sys.executable, str(script)])
    src = worker.Source(io.BytesIO(_mkv_raw(fr, w, h, codec="V_MPEG4/ISO/AVC", colour=b"")))
    assert src.child is not None and not src.info.full_range
    buf = np.zeros((64, fr.shape[1]), np.uint8)
    n = src.read_into(buf, 64)
    assert n == 40
    np.testing.assert_array_equal(buf[:40], fr)
    assert src.close() == 0


def test_worker_passthrough_runs_reference_command(tmp_path):
    """remote_args outside the GPU profile: exactly the reference's worker ffmpeg runs."""
    log = tmp_path / "shim.log"
    env = dict(os.environ, PATH=os.path.join(HERE, "shims") + os.pathsep + os.environ["PATH"],
               SHIM_LOG=str(log), PYTHONPATH=ROOT)
    args = ["-c:v", "libx264", "-crf", "18"]
    p = subprocess.run([sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", "0", *args],
                       input=b"SEGMENT", capture_output=True, env=env, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout == b"ENC[SEGMENT]"
    calls = [json.loads(l) for l in open(log)]
    assert calls == [{"prog": "ffmpeg", "argv": worker.reference_argv(args)[1:], "host": "localhost"}]
    assert b"running ffmpeg on the CPU" in p.stderr


def test_worker_pix_fmt_resample_falls_through_to_ffmpeg(tmp_path):
    """-pix_fmt asking for another chroma sampling than the input's is not on the GPU path:
    the frames read so far (and the rest) go to the real ffmpeg as y4m, with the
    remote_args unchanged."""
    log = tmp_path / "shim.log"
    env = dict(os.environ, PATH=os.path.join(HERE, "shims") + os.pathsep + os.environ["PATH"],
               SHIM_LOG=str(log), PYTHONPATH=ROOT)
    w, h = 16, 8
    fr = np.full((3, w * h + 2 * 8 * 4), 0x41, np.uint8)      # ASCII-safe: the shim reads text
    fr[:, :7] = np.arange(3)[:, None] + 0x30
    data = _y4m(fr, w, h, extra=" Ip A1:1 C420jpeg")
    args = ["-c:v", "mjpeg", "-q:v", "5", "-dct", "int", "-bitexact", "-pix_fmt", "yuvj444p"]
    p = subprocess.run([sys.executable, "-m", "ffmpeg_distributed_amd.worker", "--device", "0", *args],
                       input=data, capture_output=True, env=env, timeout=60)
    assert p.returncode == 0, p.stderr
    calls = [json.loads(l) for l in open(log)]
    assert calls == [{"prog": "ffmpeg", "argv": ["-f", "yuv4mpegpipe", "-i", "pipe:", *args, "-f",
                                                 "matroska", "pipe:"], "host": "localhost"}]
    body = p.stdout[len(b"ENC["):-1]
    rd = container.Y4MReader(io.BytesIO(body))
    assert (rd.info.width, rd.info.height, rd.info.chroma) == (w, h, "420")
    buf = np.zeros_like(fr)
    assert rd.read_into(buf, 3) == 3
    np.testing.assert_array_equal(buf, fr)


def test_progress_lines_parse_with_dispatcher_regex():
    from ffmpeg_distributed_amd import dispatcher as D
    err = io.StringIO()
    pr = worker.Progress(err, Fraction(25), 5)
    pr.duration(12.5)
    pr.update(250, 123456, final=True)
    lines = err.getvalue().splitlines()
    assert D.parse_duration(lines[0]) == pytest.approx(12.5)
    f, fps, t, speed = D.parse_progress(lines[1])
    assert f == 250 and t == pytest.approx(10.0) and speed > 0


def test_scaled_sar_follows_vf_scale():
    assert profile.scaled_sar((1, 1), (3840, 2160), (1920, 1080)) == (1, 1)
    assert profile.scaled_sar((1, 1), (176, 100), (96, 54)) == (99, 100)
    assert profile.scaled_sar((0, 0), (176, 100), (96, 54)) == (0, 0)
    assert profile.scaled_sar((4, 3), (720, 576), (1280, 720)) == (15, 16)


@pytest.mark.parametrize("num,den,mx", [(1, 1, 65535), (100000, 70001, 65535), (355, 113, 100),
                                        (2**40 + 1, 2**39, 65535), (-6, 4, 10), (65536, 65535, 65535)])
def test_av_reduce_bounds_and_accuracy(num, den, mx):
    n, d = profile.av_reduce(num, den, mx)
    assert abs(n) <= mx and 0 < d <= mx
    x = Fraction(num, den)
    if abs(x.numerator) <= mx and x.denominator <= mx:
        assert Fraction(n, d) == x                       # exact when it fits
    assert abs(Fraction(n, d) - x) <= abs(x) / mx


def test_mkv_without_display_size_means_square_pixels():
    buf = io.BytesIO()
    w = container.MkvWriter(buf, 320, 240, Fraction(25))
    w.write_frame(b"x")
    w.close()
    assert container.MkvReader(io.BytesIO(buf.getvalue())).info(1).sar == (1, 1)


@pytest.mark.parametrize("args", [
    "-c:v mjpeg -q:v 5 -dct int -huffman default -bitexact",
    "-vf scale=1920:1080:flags=bicubic -c:v mjpeg -q:v 3 -dct int -huffman optimal -bitexact",
    "-c:v mjpeg -q:v 5 -dct int -h -hide_banner --help -devi 1",
])
def test_worker_cli_passes_every_ffmpeg_argument(args, monkeypatch):
    """`python -m ffmpeg_distributed_amd.worker --device N <remote_args>` (the dispatcher's
    gpu:N argv) hands remote_args to run() unchanged: -huffman is not argparse's -h, and
    no prefix of --device is taken as --device."""
    seen = {}
    monkeypatch.setattr(worker, "run", lambda dev, rest: seen.update(dev=dev, rest=rest) or 0)
    assert worker.main(["--device", "3", *args.split()]) == 0
    assert seen == {"dev": 3, "rest": args.split()}


def test_source_reads_raw_mkv_frames_in_place():
    """Raw V_UNCOMPRESSED segments go from the stream straight into the page-locked batch
    buffer (MkvReader.read_frame_into): same frames as the block iterator, across clusters
    and a ragged last batch; a wrong-sized block is an error, not a silent truncation."""
    w, h, n = 48, 32, 70   # 30 fps: three 1 s clusters
    frames = [np.random.default_rng(i).integers(0, 256, w * h * 3 // 2, dtype=np.uint8) for i in range(n)]
    buf = io.BytesIO()
    wr = container.MkvWriter(buf, w, h, Fraction(30), codec="V_UNCOMPRESSED", colour_space=b"I420")
    for f in frames:
        wr.write_frame(f.tobytes())
    wr.close()
    data = buf.getvalue()
    src = worker.Source(io.BytesIO(data))
    assert src._mkv._raw.recorded is None  # no copy of the input kept for a decoder
    fb = src.info.frame_bytes
    out = np.zeros((16, fb), np.uint8)
    got = []
    while True:
        k = src.read_into(out, 16)
        got += [out[i].copy() for i in range(k)]
        if k < 16:
            break
    assert len(got) == n and all((a == b).all() for a, b in zip(got, frames))
    ref = [d for _, d in container.MkvReader(io.BytesIO(data)).frames(1)]
    assert [bytes(g) for g in got] == ref

    bad = io.BytesIO()
    wr = container.MkvWriter(bad, w, h, Fraction(30), codec="V_UNCOMPRESSED", colour_space=b"I420")
    wr.write_frame(frames[0].tobytes()[:-1])
    wr.close()
    src = worker.Source(io.BytesIO(bad.getvalue()))
    with pytest.raises(ValueError, match="V_UNCOMPRESSED frame of"):
        src.read_into(np.zeros((1, fb), np.uint8), 1)


def test_source_parallel_reads_from_a_file(tmp_path):
    """A segment that is a regular file (the dispatcher's stdin, or worker --serve): block
    headers parsed in order, payloads fetched by parallel positional reads into the batch
    buffer; same frames as the sequential reader, across clusters and ragged batches."""
    w, h, n = 40, 24, 75
    frames = [np.random.default_rng(100 + i).integers(0, 256, w * h * 3 // 2, dtype=np.uint8)
              for i in range(n)]
    path = tmp_path / "seg.mkv"
    with open(path, "wb") as f:
        wr = container.MkvWriter(f, w, h, Fraction(25), codec="V_UNCOMPRESSED", colour_space=b"I420")
        for fr in frames:
            wr.write_frame(fr.tobytes())
        wr.close()
    for batch in (1, 7, 32):
        with open(path, "rb") as fin:
            src = worker.Source(fin)
            assert src.read_into == src._read_mkv_pread
            out = np.zeros((batch, src.info.frame_bytes), np.uint8)
            got = []
            while True:
                k = src.read_into(out, batch)
                got += [out[i].copy() for i in range(k)]
                if k < batch:
                    break
            assert src.close() == 0
        assert len(got) == n and all((a == b).all() for a, b in zip(got, frames)), batch

    bad = tmp_path / "bad.mkv"
    with open(bad, "wb") as f:
        wr = container.MkvWriter(f, w, h, Fraction(25), codec="V_UNCOMPRESSED", colour_space=b"I420")
        wr.write_frame(frames[0].tobytes())
        wr.write_frame(frames[1].tobytes()[:-3])
        wr.close()
    with open(bad, "rb") as fin:
        src = worker.Source(fin)
        with pytest.raises(ValueError, match="V_UNCOMPRESSED frame of"):
            src.read_into(np.zeros((2, src.info.frame_bytes), np.uint8), 2)
        src.close()
