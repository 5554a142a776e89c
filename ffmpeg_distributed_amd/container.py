"""Native segment I/O for the gpu:N worker (worker-side demux/mux
in-process).  The reference's worker reads a Matroska segment on stdin and writes a
Matroska segment on stdout (ffmpeg_distributed.py:133-135); its output must stay
readable by the ffmpeg concat demuxer the reference runs at :216-227.

  Y4MReader   YUV4MPEG2 raw 4:2:0 / 4:2:2 / 4:4:4 frames (what `ffmpeg -f yuv4mpegpipe` emits)
  y4m_header  the matching writer's stream header
  MkvReader   Matroska with V_UNCOMPRESSED I420 / Y42B / 444P video (a `-c copy` split of
              raw video) or V_MJPEG (used by the tests to read our own output back)
  MkvWriter   Matroska with one V_MJPEG video track, one keyframe SimpleBlock per frame
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from fractions import Fraction
from typing import BinaryIO, Iterator, List, Optional, Tuple

# ------------------------------------------------------------------------- EBML
EBML = 0x1A45DFA3
SEGMENT = 0x18538067
INFO = 0x1549A966
TRACKS = 0x1654AE6B
TRACK_ENTRY = 0xAE
VIDEO = 0xE0
CLUSTER = 0x1F43B675
BLOCK_GROUP = 0xA0
SIMPLE_BLOCK = 0xA3
BLOCK = 0xA1
TIMESTAMP = 0xE7
MASTERS = {EBML, SEGMENT, INFO, TRACKS, TRACK_ENTRY, VIDEO, CLUSTER, BLOCK_GROUP, 0x55B0}
UNKNOWN = object()


def _id_bytes(eid: int) -> bytes:
    n = (eid.bit_length() + 7) // 8
    return eid.to_bytes(n, "big")


def _size_bytes(n: int) -> bytes:
    for length in range(1, 9):
        if n < (1 << (7 * length)) - 1:
            return ((1 << (7 * length)) | n).to_bytes(length, "big")
    raise ValueError(n)


def element(eid: int, payload: bytes) -> bytes:
    return _id_bytes(eid) + _size_bytes(len(payload)) + payload


def uint_el(eid: int, v: int) -> bytes:
    n = max(1, (v.bit_length() + 7) // 8)
    return element(eid, v.to_bytes(n, "big"))


def str_el(eid: int, s: str) -> bytes:
    return element(eid, s.encode())


def float_el(eid: int, v: float) -> bytes:
    return element(eid, struct.pack(">d", v))


def _read_vint(f: BinaryIO, keep_marker: bool):
    b = f.read(1)
    if not b:
        return None, 0
    first = b[0]
    length = 1
    mask = 0x80
    while length <= 8 and not first & mask:
        length += 1
        mask >>= 1
    if length > 8:
        raise ValueError("bad EBML vint")
    rest = f.read(length - 1)
    if len(rest) != length - 1:
        raise EOFError
    v = first if keep_marker else first & (mask - 1)
    for x in rest:
        v = (v << 8) | x
    if not keep_marker and v == (1 << (7 * length)) - 1:
        return UNKNOWN, length
    return v, length


# ------------------------------------------------------------------------- Y4M
@dataclass
class StreamInfo:
    width: int
    height: int
    fps: Fraction = Fraction(25, 1)
    sar: Tuple[int, int] = (0, 0)       # (0, 0): unknown
    full_range: bool = False
    codec: str = "rawvideo"
    frame_bytes: int = 0
    chroma: str = "420"                 # planar sampling: "420", "422", "444"

    def __post_init__(self):
        if not self.frame_bytes:
            hs, vs = {"420": (1, 1), "422": (1, 0), "444": (0, 0)}[self.chroma]
            cw, ch = (self.width + hs) >> hs, (self.height + vs) >> vs
            self.frame_bytes = self.width * self.height + 2 * cw * ch


# Matroska V_UNCOMPRESSED ColourSpace fourccs (libavformat/raw.c ff_raw_pix_fmt_tags)
MKV_FOURCC_CHROMA = {b"I420": "420", b"": "420", b"Y42B": "422", b"444P": "444"}


def y4m_chroma(tag: str) -> str:
    """Sampling of a YUV4MPEG2 'C' tag (yuv4mpegdec.c: 420jpeg/420paldv/420mpeg2/420, 422, 444)."""
    for c in ("420", "422", "444"):
        if tag == c or (c == "420" and tag in ("420jpeg", "420paldv", "420mpeg2")):
            return c
    raise ValueError(f"y4m colorspace C{tag}: only 8-bit 4:2:0 / 4:2:2 / 4:4:4")


def y4m_header(info: "StreamInfo") -> bytes:
    """YUV4MPEG2 stream header for `info` (yuv4mpegenc.c field order)."""
    c = {"420": "420jpeg", "422": "422", "444": "444"}[info.chroma]
    a = f"A{info.sar[0]}:{info.sar[1]}" if info.sar != (0, 0) else "A0:0"
    x = " XCOLORRANGE=FULL" if info.full_range else ""
    fps = info.fps
    return (f"YUV4MPEG2 W{info.width} H{info.height} F{fps.numerator}:{fps.denominator} Ip {a} "
            f"C{c}{x}\n").encode()


class Y4MReader:
    """YUV4MPEG2: 'YUV4MPEG2 W H F A I C X...\\n' then ('FRAME[params]\\n' + I420)*."""

    def __init__(self, f: BinaryIO, head: bytes = b""):
        self.f = f
        line = head + self._readline()
        if not line.startswith(b"YUV4MPEG2"):
            raise ValueError("not a YUV4MPEG2 stream")
        w = h = None
        fps, sar, full, chroma = Fraction(25), (0, 0), False, "420"
        for tok in line.split()[1:]:
            t, v = tok[:1], tok[1:].decode()
            if t == b"W":
                w = int(v)
            elif t == b"H":
                h = int(v)
            elif t == b"F":
                n, d = v.split(":")
                fps = Fraction(int(n), int(d))
            elif t == b"A":
                n, d = v.split(":")
                sar = (int(n), int(d))
            elif t == b"C":
                chroma = y4m_chroma(v)
            elif t == b"X" and v.upper().startswith("COLORRANGE="):
                full = v.split("=", 1)[1].upper() == "FULL"
        if not w or not h:
            raise ValueError("y4m header without W/H")
        self.info = StreamInfo(w, h, fps, sar, full, chroma=chroma)

    def _readline(self) -> bytes:
        out = bytearray()
        while True:
            c = self.f.read(1)
            if not c or c == b"\n":
                return bytes(out)
            out += c

    def read_into(self, buf, nframes: int) -> int:
        """Read up to nframes into buf (a writable uint8 buffer); returns frames read."""
        mv = memoryview(buf).cast("B")
        fb = self.info.frame_bytes
        for i in range(nframes):
            tag = self.f.read(5)
            if len(tag) < 5:
                return i
            if tag != b"FRAME":
                raise ValueError("y4m: expected FRAME")
            while self.f.read(1) not in (b"\n", b""):
                pass
            dst = mv[i * fb:(i + 1) * fb]
            got = 0
            while got < fb:
                n = self.f.readinto(dst[got:])
                if not n:
                    raise EOFError("truncated y4m frame")
                got += n
        return nframes


# ------------------------------------------------------------------------- MKV read
@dataclass
class MkvTrack:
    number: int = 0
    codec: str = ""
    width: int = 0
    height: int = 0
    default_duration: int = 0          # ns
    colour_space: bytes = b""
    display: Tuple[int, int] = (0, 0)
    colour_range: int = 0              # Colour/Range: 1 broadcast, 2 full


class MkvReader:
    """Streaming Matroska reader (no seeking): track list, then frames of track 1."""

    def __init__(self, f: BinaryIO, head: bytes = b"", record: bool = False):
        import io
        self._raw = _Prefixed(f, head, record)
        self.f = io.BufferedReader(self._raw)
        self.tracks: List[MkvTrack] = []
        self._pending: List[Tuple[int, bytes]] = []
        self._cluster_ts = 0
        self.timescale = 1000000
        self._in_track: Optional[MkvTrack] = None
        self._eof = False
        self.duration: Optional[float] = None     # Info/Duration, timescale units
        # headers up to the first Cluster's start (its blocks are left to the frame readers:
        # an 8K block is 50 MB, not something to read -- and record -- while parsing headers)
        while True:
            eid, _ = _read_vint(self.f, True)
            if eid is None:
                self._eof = True
                break
            size, _ = _read_vint(self.f, False)
            if eid == CLUSTER and self.tracks:
                self._in_track = None
                break
            if not self._element(eid, size) or (self.tracks and self._in_track is None and self._pending):
                break

    def _step(self) -> bool:
        eid, _ = _read_vint(self.f, True)
        if eid is None:
            self._eof = True
            return False
        size, _ = _read_vint(self.f, False)
        return self._element(eid, size)

    def _element(self, eid: int, size) -> bool:
        if eid in MASTERS:
            if eid == TRACK_ENTRY:
                self._in_track = MkvTrack()
                self.tracks.append(self._in_track)
            return True
        if size is UNKNOWN:
            raise ValueError(f"unknown-size leaf element {eid:#x}")
        data = self.f.read(size)
        if len(data) != size:
            self._eof = True
            return False
        tr = self.tracks[-1] if self.tracks else None
        if eid == 0x2AD7B1:
            self.timescale = int.from_bytes(data, "big")
        elif eid == 0xD7 and tr:
            tr.number = int.from_bytes(data, "big")
        elif eid == 0x86 and tr:
            tr.codec = data.rstrip(b"\0").decode()
        elif eid == 0x23E383 and tr:
            tr.default_duration = int.from_bytes(data, "big")
        elif eid == 0xB0 and tr:
            tr.width = int.from_bytes(data, "big")
        elif eid == 0xBA and tr:
            tr.height = int.from_bytes(data, "big")
        elif eid == 0x54B0 and tr:
            tr.display = (int.from_bytes(data, "big"), tr.display[1])
        elif eid == 0x54BA and tr:
            tr.display = (tr.display[0], int.from_bytes(data, "big"))
        elif eid == 0x2EB524 and tr:
            tr.colour_space = data
        elif eid == TIMESTAMP:
            self._cluster_ts = int.from_bytes(data, "big")
        elif eid in (SIMPLE_BLOCK, BLOCK):
            self._in_track = None
            tn, n = _vint_from(data, 0)
            rel = struct.unpack(">h", data[n:n + 2])[0]
            flags = data[n + 2]
            if flags & 0x06:
                raise ValueError("laced Matroska blocks are not supported")
            self._pending.append((tn, self._cluster_ts + rel, data[n + 3:]))
        elif eid == 0x4489:
            self.duration = struct.unpack(">d" if size == 8 else ">f", data)[0]
        elif eid == 0x55B9 and tr:
            tr.colour_range = int.from_bytes(data, "big")
        return True

    def read_frame_into(self, track: int, dest) -> Optional[int]:
        """The next block of `track` read straight into `dest` (a writable buffer of exactly
        the block's payload size: one copy, no intermediate bytes); returns its timestamp
        (timescale units), or None at the end of the stream."""
        while True:
            while self._pending:
                tn, ts, data = self._pending.pop(0)
                if tn == track:
                    if len(data) != len(dest):
                        raise ValueError(f"frame of {len(data)} bytes, expected {len(dest)}")
                    dest[:] = data
                    return ts
            if self._eof:
                return None
            eid, _ = _read_vint(self.f, True)
            if eid is None:
                self._eof = True
                return None
            size, _ = _read_vint(self.f, False)
            if eid not in (SIMPLE_BLOCK, BLOCK) or size is UNKNOWN:
                if not self._element(eid, size):
                    return None
                continue
            self._in_track = None
            first = self.f.read(1)
            if not first:
                self._eof = True
                return None
            vlen = 1
            while vlen <= 8 and not first[0] & (0x80 >> (vlen - 1)):
                vlen += 1
            rest = self.f.read(vlen - 1 + 3)
            if len(rest) != vlen + 2:
                self._eof = True
                return None
            tn, _ = _vint_from(first + rest, 0)
            rel = struct.unpack(">h", rest[vlen - 1:vlen + 1])[0]
            if rest[vlen + 1] & 0x06:
                raise ValueError("laced Matroska blocks are not supported")
            payload = size - vlen - 3
            if tn != track:
                if len(self.f.read(payload)) != payload:
                    self._eof = True
                    return None
                continue
            if payload != len(dest):
                raise ValueError(f"frame of {payload} bytes, expected {len(dest)}")
            if self.f.readinto(dest) != payload:
                self._eof = True
                return None
            return self._cluster_ts + rel

    def _held(self) -> int:
        """Bytes this reader holds past its logical position (may refill from the stream)."""
        return len(self.f.peek(1))

    def frames_into_pread(self, track: int, dests, pread) -> int:
        """Like read_frame_into over `dests`, for a stream backed by a regular file: block
        headers are parsed here, each payload is skipped and handed to `pread(file_offset,
        dest)` (positional reads, which the caller runs in parallel).  Returns how many of
        `dests` got a block; the caller waits for the reads."""
        outer = self._raw.f
        n = 0
        while n < len(dests):
            if self._pending:
                if self.read_frame_into(track, dests[n]) is None:
                    return n
                n += 1
                continue
            if self._eof:
                return n
            eid, _ = _read_vint(self.f, True)
            if eid is None:
                self._eof = True
                return n
            size, _ = _read_vint(self.f, False)
            if eid not in (SIMPLE_BLOCK, BLOCK) or size is UNKNOWN:
                if not self._element(eid, size):
                    return n
                continue
            self._in_track = None
            first = self.f.read(1)
            if not first:
                self._eof = True
                return n
            vlen = 1
            while vlen <= 8 and not first[0] & (0x80 >> (vlen - 1)):
                vlen += 1
            rest = self.f.read(vlen - 1 + 3)
            if len(rest) != vlen + 2:
                self._eof = True
                return n
            tn, _ = _vint_from(first + rest, 0)
            if rest[vlen + 1] & 0x06:
                raise ValueError("laced Matroska blocks are not supported")
            payload = size - vlen - 3
            if tn == track and payload != len(dests[n]):
                raise ValueError(f"frame of {payload} bytes, expected {len(dests[n])}")
            held = self._held()
            off = outer.tell() - held  # file offset of the payload
            if payload <= held:
                self.f.read(payload)
            else:
                self.f.read(held)
                outer.seek(payload - held, 1)
            if tn == track:
                pread(off, dests[n])
                n += 1
        return n

    def stop_recording(self) -> None:
        """No decoder child will need the bytes read so far (raw frames are read natively)."""
        self._raw.recorded = None

    def replay_bytes(self) -> bytes:
        """Every byte taken from the underlying stream so far (record=True), so a
        decoder child can be handed the whole input; stops recording."""
        out = bytes(self._raw.recorded)
        self._raw.recorded = None
        return out

    def frames(self, track: int = 1) -> Iterator[Tuple[int, bytes]]:
        """(timestamp in timescale units, payload) of every block of `track`."""
        while True:
            while self._pending:
                tn, ts, data = self._pending.pop(0)
                if tn == track:
                    yield ts, data
            if self._eof or not self._step():
                while self._pending:
                    tn, ts, data = self._pending.pop(0)
                    if tn == track:
                        yield ts, data
                return

    def info(self, track: int = 1) -> StreamInfo:
        tr = next(t for t in self.tracks if t.number == track)
        fps = Fraction(10 ** 9, tr.default_duration) if tr.default_duration else Fraction(25)
        sar = (1, 1)     # matroskadec: display size defaults to the pixel size
        if tr.display != (0, 0) and tr.width and tr.height:
            s = Fraction(tr.display[0] * tr.height, tr.display[1] * tr.width)
            sar = (s.numerator, s.denominator)
        chroma = MKV_FOURCC_CHROMA.get(tr.colour_space, "420") if tr.codec == "V_UNCOMPRESSED" else "420"
        return StreamInfo(tr.width, tr.height, fps.limit_denominator(1001), sar,
                          full_range=tr.colour_range == 2, codec=tr.codec, chroma=chroma)

    def duration_seconds(self) -> Optional[float]:
        return None if self.duration is None else self.duration * self.timescale / 1e9


def _vint_from(buf: bytes, pos: int):
    first = buf[pos]
    length, mask = 1, 0x80
    while not first & mask:
        length += 1
        mask >>= 1
    v = first & (mask - 1)
    for x in buf[pos + 1:pos + length]:
        v = (v << 8) | x
    return v, length


class _Prefixed:
    """Raw stream that first returns `head` (bytes already peeked), then `f`;
    optionally keeps a copy of everything it returned."""

    def __init__(self, f, head, record=False):
        self.f, self.head = f, head
        self.recorded = bytearray() if record else None

    def readable(self):
        return True

    def readinto(self, b):
        if self.head:
            n = min(len(b), len(self.head))
            b[:n] = self.head[:n]
            if self.recorded is not None:
                self.recorded += self.head[:n]
            self.head = self.head[n:]
            return n
        if self.recorded is None and hasattr(self.f, "readinto"):
            return self.f.readinto(b)  # straight into the caller's buffer
        data = self.f.read(len(b))
        b[:len(data)] = data
        if self.recorded is not None:
            self.recorded += data
        return len(data)

    @property
    def closed(self):
        return False


# ------------------------------------------------------------------------- MKV write
class MkvWriter:
    """One video track (V_MJPEG by default); every frame a keyframe SimpleBlock; clusters of <= 1 s written
    with known sizes as they fill (the stream is a pipe, so the Segment size is unknown)."""

    def __init__(self, f: BinaryIO, width: int, height: int, fps: Fraction,
                 sar: Tuple[int, int] = (0, 0), app: str = "ffmpeg_distributed_amd",
                 codec: str = "V_MJPEG", colour_space: bytes = b"", colour_range: int = 0):
        self.f = f
        self.fps = Fraction(fps)
        self.n = 0
        self._cluster: List[bytes] = []
        self._cluster_ts = 0
        ebml = element(EBML, uint_el(0x4286, 1) + uint_el(0x42F7, 1) + uint_el(0x42F2, 4) +
                       uint_el(0x42F3, 8) + str_el(0x4282, "matroska") + uint_el(0x4287, 4) +
                       uint_el(0x4285, 2))
        info = element(INFO, uint_el(0x2AD7B1, 1000000) + str_el(0x4D80, app) + str_el(0x5741, app))
        video = uint_el(0xB0, width) + uint_el(0xBA, height)
        if sar[0] > 0 and sar[1] > 0 and sar[0] != sar[1]:
            dw = Fraction(width * sar[0], sar[1])
            video += uint_el(0x54B0, round(dw)) + uint_el(0x54BA, height)
        if colour_space:
            video += element(0x2EB524, colour_space)
        if colour_range:
            video += element(0x55B0, uint_el(0x55B9, colour_range))
        track = element(TRACK_ENTRY, uint_el(0xD7, 1) + uint_el(0x73C5, 1) + uint_el(0x83, 1) +
                        uint_el(0x9C, 0) + str_el(0x86, codec) +
                        uint_el(0x23E383, round(Fraction(10 ** 9) / self.fps)) + element(VIDEO, video))
        f.write(ebml + _id_bytes(SEGMENT) + b"\x01\xff\xff\xff\xff\xff\xff\xff" + info +
                element(TRACKS, track))

    def _ts_ms(self, i: int) -> int:
        return round(Fraction(1000 * i) / self.fps)

    def write_frame(self, jpeg: bytes):
        ts = self._ts_ms(self.n)
        if self._cluster and (ts - self._cluster_ts >= 1000 or len(self._cluster) >= 256):
            self._flush()
        if not self._cluster:
            self._cluster_ts = ts
            self._cluster_bytes = 0
        rel = ts - self._cluster_ts
        # the SimpleBlock's header (ID, size, track 1, timecode, keyframe flag); the JPEG is
        # written after it as its own piece: no per-frame copy of the payload
        body = 4 + len(jpeg)
        head = _id_bytes(SIMPLE_BLOCK) + _size_bytes(body) + b"\x81" + struct.pack(">hB", rel, 0x80)
        self._cluster.append((head, jpeg))
        self._cluster_bytes += len(head) + len(jpeg)
        self.n += 1

    def flush_pending(self):
        """End the current cluster now and write it (its packets may live in a buffer the
        caller reuses next: the worker's page-locked output buffers).  Clusters then follow the
        submits (at most 1 s / 256 frames still holds)."""
        self._flush()

    def _flush(self):
        if self._cluster:
            ts = uint_el(TIMESTAMP, self._cluster_ts)
            pieces = [_id_bytes(CLUSTER) + _size_bytes(len(ts) + self._cluster_bytes) + ts]
            for head, jpeg in self._cluster:
                pieces.append(head)
                pieces.append(jpeg)
            self.f.writelines(pieces)
            self._cluster = []

    def close(self):
        self._flush()
        self.f.flush()
