"""Parse the reference's `remote_args` (ffmpeg_distributed.py:190 shlex-splits them and
:134 passes them to the worker ffmpeg) into the GPU encode profile, or report why the
arguments fall outside it (the worker then runs the real ffmpeg unchanged).

Supported profile (BASELINE north star, plus FFmpeg's default -huffman optimal):
    [-vf scale=W:H[:flags=bicubic...]] -c:v mjpeg -q:v N -dct int [-huffman default|optimal] -bitexact
plus
  - the slice-threaded (RST) layout: -slices N (N > 1), or -thread_type slice with -threads
    other than 1 (mpegvideo's slice_context_count > 1: DRI + one restart interval per MCU
    row; mjpegenc.c then forces -huffman default);
  - -pix_fmt yuvj420p / yuvj422p / yuvj444p (the output sampling; the worker checks it
    against the input's, since a chroma resample is not on the GPU path);
  - options that do not change the video bitstream: -an -sn -dn -y -threads N
    -thread_type frame -f matroska -map 0:v[:0].
"""
from __future__ import annotations

import shlex
from math import gcd
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple, Union


@dataclass
class Profile:
    qscale: int                      # effective mpegvideo qscale (update_qscale mapping)
    q_arg: float                     # the -q:v value as given
    scale: Optional[Tuple[int, int]] = None   # -vf scale=W:H
    sws_flags: Tuple[str, ...] = ("bicubic",)
    huffman: str = "optimal"         # mjpegenc.c "huffman" option, default optimal
    rst: bool = False                # slice threading: DRI + RST per MCU row
    chroma: Optional[str] = None     # "420"/"422"/"444" from -pix_fmt (None: the input's)


class Unsupported(ValueError):
    pass


def effective_qscale(q: float) -> int:
    """mpegvideo_enc.c update_qscale for a fixed -q:v: lambda = q*FF_QP2LAMBDA(118),
    qscale = (lambda*139 + 128*64) >> 14, clipped to [qmin=2, qmax=31]."""
    lam = int(q * 118)
    return max(2, min(31, (lam * 139 + 128 * 64) >> 14))


_FLAGS_OK = {"bicubic", "accurate_rnd", "bitexact", "full_chroma_int", "full_chroma_inp"}


def _parse_scale(vf: str) -> Tuple[Tuple[int, int], Tuple[str, ...]]:
    if "," in vf or ";" in vf or not vf.startswith("scale="):
        raise Unsupported(f"filter graph {vf!r} (only a single scale=W:H is GPU-accelerated)")
    parts = vf[len("scale="):].split(":")
    kv, pos = {}, []
    for p in parts:
        if "=" in p:
            k, v = p.split("=", 1)
            kv[k] = v
        else:
            pos.append(p)
    w = kv.pop("w", kv.pop("width", pos[0] if len(pos) > 0 else None))
    h = kv.pop("h", kv.pop("height", pos[1] if len(pos) > 1 else None))
    flags = tuple(f for f in kv.pop("flags", "bicubic").replace("+", " ").split() if f)
    if kv:
        raise Unsupported(f"scale options {sorted(kv)}")
    try:
        W, H = int(w), int(h)
    except (TypeError, ValueError):
        raise Unsupported(f"scale size {w}:{h} (explicit positive W:H required)")
    if W <= 0 or H <= 0:
        raise Unsupported(f"scale size {W}:{H}")
    if not flags or flags[0] != "bicubic" or any(f not in _FLAGS_OK for f in flags):
        raise Unsupported(f"scale flags {flags}")
    return (W, H), flags


def _flag_ops(v: str) -> List[Tuple[str, str]]:
    """An AVOption flags string (`+a-b`, `a+b`, `a`) as (op, name) pairs; op '' replaces the
    whole set (libavutil opt.c set_string_flags: a leading name without +/- starts from 0)."""
    out, op, name = [], "", ""
    for ch in v:
        if ch in "+-":
            if name:
                out.append((op, name))
            op, name = ch, ""
        else:
            name += ch
    if name:
        out.append((op, name))
    if not out:
        raise Unsupported(f"flags {v!r}")
    return out


def _apply_flag(cur: bool, ops: List[Tuple[str, str]]) -> bool:
    for op, _ in ops:
        cur = op != "-"
    return cur


def parse(args: Union[str, Sequence[str]]) -> Profile:
    """Profile for `remote_args`, or raise Unsupported(reason)."""
    a: List[str] = shlex.split(args) if isinstance(args, str) else list(args)
    codec = q = dct = huff = None
    bitexact = False
    slices = 0
    threads: Optional[int] = None     # None: auto (0)
    thread_type = "slice+frame"       # AVCodecContext default: FF_THREAD_FRAME | FF_THREAD_SLICE
    chroma = None
    scale = None
    flags: Tuple[str, ...] = ("bicubic",)
    i = 0

    def val():
        nonlocal i
        if i + 1 >= len(a):
            raise Unsupported(f"{a[i]} without a value")
        i += 1
        return a[i]

    while i < len(a):
        o = a[i]
        if o in ("-c:v", "-codec:v", "-vcodec", "-c", "-codec"):
            codec = val()
        elif o in ("-q:v", "-qscale:v", "-q", "-qscale"):
            try:
                q = float(val())
            except ValueError:
                raise Unsupported(f"{o} {a[i]}")
        elif o == "-dct":
            dct = val()
        elif o == "-huffman":
            huff = val()
        elif o == "-bitexact":
            bitexact = True
        elif o in ("-flags", "-flags:v"):
            # AVCodecContext.flags: the only codec flag on the GPU path is bitexact; any other
            # (+gray, +qscale, ...) changes the bitstream, so it is not accepted silently
            v = val()
            ops = _flag_ops(v)
            if any(name != "bitexact" for _, name in ops):
                raise Unsupported(f"{o} {v} (only bitexact is GPU-accelerated)")
            bitexact = _apply_flag(bitexact, ops)
        elif o == "-fflags":
            # AVFormatContext.fflags: a muxer flag (format-level bitexact, no Lavf version
            # strings); it never reaches the encoder, so it does not count as codec bitexact
            v = val()
            if any(name != "bitexact" for _, name in _flag_ops(v)):
                raise Unsupported(f"-fflags {v}")
        elif o in ("-vf", "-filter:v"):
            scale, flags = _parse_scale(val())
        elif o in ("-an", "-sn", "-dn", "-y"):
            pass
        elif o in ("-threads", "-threads:v"):
            v = val()
            try:
                threads = None if v == "auto" else int(v)
            except ValueError:
                raise Unsupported(f"{o} {v}")
            if threads == 0:
                threads = None
        elif o in ("-thread_type", "-thread_type:v"):
            thread_type = val()
            if any(t not in ("slice", "frame") for t in thread_type.split("+")):
                raise Unsupported(f"-thread_type {thread_type}")
        elif o in ("-slices", "-slices:v"):
            try:
                slices = int(val())
            except ValueError:
                raise Unsupported(f"-slices {a[i]}")
        elif o in ("-pix_fmt", "-pix_fmt:v"):
            pf = val()
            if pf not in PIX_FMT_CHROMA:
                raise Unsupported(f"-pix_fmt {pf} (GPU path writes yuvj420p/422p/444p)")
            chroma = PIX_FMT_CHROMA[pf]
        elif o == "-f":
            if val() != "matroska":
                raise Unsupported(f"-f {a[i]}")
        elif o == "-map":
            if val() not in ("0:v", "0:v:0", "0"):
                raise Unsupported(f"-map {a[i]}")
        else:
            raise Unsupported(f"option {o}")
        i += 1
    if codec != "mjpeg":
        raise Unsupported(f"codec {codec!r}")
    if q is None:
        raise Unsupported("no -q:v (rate control modes are not GPU-accelerated)")
    if dct != "int":
        raise Unsupported(f"-dct {dct!r} (only the integer jfdctint is bit-exact reproducible)")
    if huff is None:
        huff = "optimal"  # mjpegenc.c: the "huffman" AVOption defaults to HUFFMAN_TABLE_OPTIMAL
    if huff not in ("default", "optimal"):
        raise Unsupported(f"-huffman {huff!r}")
    if not bitexact:
        raise Unsupported("no -bitexact (the Lavc COM segment is build-specific)")
    rst = uses_slices(slices, threads, thread_type)
    if rst:
        huff = "default"  # mjpegenc.c: slice_context_count > 1 forces HUFFMAN_TABLE_DEFAULT
    return Profile(qscale=effective_qscale(q), q_arg=q, scale=scale, sws_flags=flags, huffman=huff,
                   rst=rst, chroma=chroma)


PIX_FMT_CHROMA = {"yuvj420p": "420", "yuvj422p": "422", "yuvj444p": "444"}


def uses_slices(slices: int, threads: Optional[int], thread_type: str) -> bool:
    """Whether the mjpeg encoder runs with slice_context_count > 1 (mpegvideo.c
    ff_mpv_init_context: nb_slices = -slices if set, else the thread count when slice
    threading is active; the frame-threading encoder, preferred whenever "frame" is in
    -thread_type, gives each frame a single-threaded context).  The layout then does not
    depend on the slice count (a restart interval per MCU row either way); -threads auto
    counts as more than one thread.  A one-MCU-row picture still gets no RST (the slice
    count is clipped to mb_height), which the encoder handles."""
    if slices:
        return slices > 1
    if threads == 1:
        return False
    return "frame" not in thread_type.split("+")


def av_reduce(num: int, den: int, max_v: int) -> Tuple[int, int]:
    """libavutil av_reduce: the best rational approximation of num/den with both terms
    <= max_v (continued-fraction convergents, then the best semiconvergent)."""
    a0n, a0d, a1n, a1d = 0, 1, 1, 0
    sign = (num < 0) != (den < 0)
    num, den = abs(num), abs(den)
    g = gcd(num, den)
    if g:
        num, den = num // g, den // g
    if num <= max_v and den <= max_v:
        a1n, a1d, den = num, den, 0
    while den:
        x = num // den
        next_den = num - den * x
        a2n, a2d = x * a1n + a0n, x * a1d + a0d
        if a2n > max_v or a2d > max_v:
            if a1n:
                x = (max_v - a0n) // a1n
            if a1d:
                x = min(x, (max_v - a0d) // a1d)
            if den * (2 * x * a1d + a0d) > num * a1d:
                a1n, a1d = x * a1n + a0n, x * a1d + a0d
            break
        a0n, a0d, a1n, a1d = a1n, a1d, a2n, a2d
        num, den = den, next_den
    return (-a1n if sign else a1n), a1d


def scaled_sar(sar: Tuple[int, int], src: Tuple[int, int], dst: Tuple[int, int]) -> Tuple[int, int]:
    """Sample aspect ratio after the scale filter (vf_scale config_props: an unknown SAR
    stays unknown, otherwise SAR * (out_h*in_w)/(out_w*in_h), reduced), then the 16-bit
    reduction the JFIF APP0 writer applies (mjpegenc_common.c jpeg_put_comments)."""
    if sar[0] <= 0 or sar[1] <= 0:
        return (0, 0)
    n, d = av_reduce(dst[1] * src[0] * sar[0], dst[0] * src[1] * sar[1], 2**31 - 1)
    if n > 65535 or d > 65535:
        n, d = av_reduce(n, d, 65535)
    return n, d


def try_parse(args) -> Tuple[Optional[Profile], Optional[str]]:
    try:
        return parse(args), None
    except Unsupported as e:
        return None, str(e)
