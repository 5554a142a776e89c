"""Deterministic synthetic video in the spirit of lavfi `testsrc2` (the reference
benchmark input, BASELINE.json configs): 75% colour bars, luma/chroma ramps, a moving
box, a moving checkerboard patch and a frame-counter bar.  FFmpeg is not available on
this pool, so this is *synthetic data of the same shape and character*, not
testsrc2's exact pixels.  One integer formula, evaluated by numpy (CPU) or torch
(any device) with identical results.
"""
from __future__ import annotations

import numpy as np

# BT.601 limited-range 75% bars: white, yellow, cyan, green, magenta, red, blue, black
_BARS = np.array([[180, 128, 128], [162, 44, 142], [131, 156, 44], [112, 72, 58],
                  [84, 184, 198], [65, 100, 212], [35, 212, 114], [16, 128, 128]], np.int32)


def _plane(xp, w, h, t, comp, sub, full_range, device=None):
    """One plane (comp 0=Y, 1=U, 2=V) of frame t; sub=1 for 2x subsampled chroma."""
    W, H = w, h
    pw, ph = (W + sub) >> sub, (H + sub) >> sub
    if xp is np:
        ys = np.arange(ph, dtype=np.int32)[:, None] << sub
        xs = np.arange(pw, dtype=np.int32)[None, :] << sub
        bars = _BARS[:, comp]
        where, mn, mx = np.where, np.minimum, np.maximum
    else:
        import torch
        ys = (torch.arange(ph, dtype=torch.int32, device=device)[:, None] << sub)
        xs = (torch.arange(pw, dtype=torch.int32, device=device)[None, :] << sub)
        bars = torch.as_tensor(_BARS[:, comp], device=device)
        where, mn, mx = torch.where, torch.minimum, torch.maximum
    top = (ys < (3 * H) // 4)
    bar_idx = (xs * 8) // W
    v_bars = bars[bar_idx.reshape(-1)].reshape(1, -1) + 0 * ys
    if comp == 0:
        ramp = 16 + (xs * 219) // max(W - 1, 1) + 0 * ys
    elif comp == 1:
        ramp = 16 + (xs * 224) // max(W - 1, 1) + 0 * ys
    else:
        ramp = 16 + ((H - 1 - ys) * 224) // max(H - 1, 1) + 0 * xs
    v = where(top, v_bars, ramp)
    if comp == 0:  # low-amplitude moving diagonal texture over the bars (AC content)
        saw = (xs + 2 * ys + 3 * t) % 48
        v = where(top, v + (mn(saw, 48 - saw) - 12) // 2, v)
    # moving box
    bs = max(H // 6, 8)
    bx = (t * 13 * max(W // 256, 1)) % max(W - bs, 1)
    by = (t * 7 * max(H // 256, 1)) % max(H - bs, 1)
    inbox = (xs >= bx) & (xs < bx + bs) & (ys >= by) & (ys < by + bs)
    boxval = [(200 + 3 * t) % 220 + 16, (60 + 5 * t) % 224 + 16, (180 + 11 * t) % 224 + 16][comp]
    v = where(inbox, boxval + 0 * v, v)
    # moving checkerboard patch (high-frequency detail: long AC runs, 0xFF stuffing)
    cs = max(H // 8, 16)
    cx = (W // 2 + t * 5) % max(W - cs, 1)
    cy = H // 8
    incb = (xs >= cx) & (xs < cx + cs) & (ys >= cy) & (ys < cy + cs)
    cell = max(1, cs // 16)
    chk = (((xs - cx) // cell + (ys - cy) // cell) & 1)
    chkval = (16 + 219 * chk) if comp == 0 else (128 + (2 * chk - 1) * (56 if comp == 1 else -56))
    v = where(incb, chkval + 0 * v, v)
    # frame counter bar along the bottom (binary digits of t)
    fb = max(H // 32, 4)
    inbar = ys >= H - fb
    bit = (t >> mn(((xs * 16) // W), 15 + 0 * xs)) & 1
    if comp == 0:
        v = where(inbar, 16 + 219 * bit, v)
    else:
        v = where(inbar, 128 + 0 * v, v)
    if full_range:
        # limited -> full range the way a yuvj source would carry it
        if comp == 0:
            v = ((v - 16) * 255 + 109) // 219
        else:
            v = ((v - 128) * 127 + 56) // 112 + 128
    v = mn(mx(v, 0 * v), 255 + 0 * v)
    return v


def testsrc2_i420(w: int, h: int, t: int, full_range: bool = False) -> np.ndarray:
    """One packed I420 frame (numpy uint8)."""
    planes = [_plane(np, w, h, int(t), c, 0 if c == 0 else 1, full_range) for c in range(3)]
    return np.concatenate([p.astype(np.uint8).reshape(-1) for p in planes])


def testsrc2_i420_torch(w: int, h: int, t0: int, n: int, device, full_range: bool = False):
    """n consecutive frames [t0, t0+n) as a (n, frame_bytes) uint8 torch tensor on device."""
    import torch
    frames = []
    for t in range(t0, t0 + n):
        planes = [_plane(torch, w, h, t, c, 0 if c == 0 else 1, full_range, device=device)
                  for c in range(3)]
        frames.append(torch.cat([p.to(torch.uint8).reshape(-1) for p in planes]))
    return torch.stack(frames)


# ----------------------------------------------------------------- content sensitivity
# Benchmark content beside testsrc2 (bench.py --content): the entropy coder's share of the
# encode grows with the coded bits, so throughput depends on content.  Neither is a parity
# input (the parity tests draw their own content); both are seeded and deterministic.

def _fractal(torch, h, w, seed, device, octaves, amp0, decay):
    """Value noise summed over octaves: a random grid of cell 2^k px, bicubic-upsampled,
    amplitude amp0 * decay^(octave) -- a 1/f-like spectrum with natural-image statistics."""
    import torch.nn.functional as F
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    acc = torch.zeros((1, 1, h, w), dtype=torch.float32, device=device)
    amp = amp0
    for cell in octaves:
        gh, gw = h // cell + 3, w // cell + 3
        grid = torch.randn((1, 1, gh, gw), generator=g, device=device)
        up = F.interpolate(grid, size=(gh * cell, gw * cell), mode="bicubic", align_corners=False)
        acc += amp * up[:, :, cell:cell + h, cell:cell + w]
        amp *= decay
    return acc[0, 0]


def natural_i420_torch(w: int, h: int, t0: int, n: int, device, full_range: bool = False):
    """n frames of fractal (1/f) value noise: smooth regions, textures and soft edges at every
    scale, about the coded size of camera footage at q=5 (several times testsrc2's)."""
    import torch
    cw, ch = (w + 1) // 2, (h + 1) // 2
    frames = []
    scale = max(1, w // 480)
    oct_y = [c * scale for c in (256, 128, 64, 32, 16, 8, 4)] + [2, 1]
    oct_c = [c * scale for c in (128, 64, 32, 16, 8)]
    for t in range(t0, t0 + n):
        y = 118 + _fractal(torch, h, w, 1000 + t, device, oct_y, 38.0, 0.75)
        u = 128 + _fractal(torch, ch, cw, 2000 + t, device, oct_c, 16.0, 0.7)
        v = 128 + _fractal(torch, ch, cw, 3000 + t, device, oct_c, 16.0, 0.7)
        lo, hi = (0, 255) if full_range else (16, 235)
        planes = [y.clamp(lo, hi), u.clamp(lo, 240 if not full_range else 255),
                  v.clamp(lo, 240 if not full_range else 255)]
        frames.append(torch.cat([p.round().to(torch.uint8).reshape(-1) for p in planes]))
    return torch.stack(frames)


def noise_patches_i420_torch(w: int, h: int, t0: int, n: int, device, full_range: bool = False,
                             frac: float = 0.125):
    """testsrc2 frames with a seeded `frac` of their 16x16 macroblocks replaced by uniform
    noise (Y and the co-sited 8x8 chroma): worst-case blocks (~40 nonzero coefficients,
    long codes, 0xFF stuffing) scattered among cheap ones."""
    import torch
    base = testsrc2_i420_torch(w, h, t0, n, device, full_range)
    mbw, mbh = w // 16, h // 16
    cw, ch = (w + 1) // 2, (h + 1) // 2
    g = torch.Generator(device=device)
    for i in range(n):
        g.manual_seed(7000 + t0 + i)
        sel = (torch.rand((mbh, mbw), generator=g, device=device) < frac)
        my = sel.repeat_interleave(16, 0).repeat_interleave(16, 1)
        mc = sel.repeat_interleave(8, 0).repeat_interleave(8, 1)
        f = base[i]
        y = f[: w * h].view(h, w)
        u = f[w * h: w * h + cw * ch].view(ch, cw)
        v = f[w * h + cw * ch:].view(ch, cw)
        for p, m in ((y, my), (u, mc), (v, mc)):
            hh, ww = m.shape
            noise = torch.randint(0, 256, (hh, ww), generator=g, device=device, dtype=torch.uint8)
            sub = p[:hh, :ww]
            sub[m] = noise[m]
    return base


CONTENT = {"testsrc": testsrc2_i420_torch, "natural": natural_i420_torch,
           "noise-patches": noise_patches_i420_torch}


def write_raw_segment(path: str, w: int, h: int, fps, frames: int, distinct: int = 8,
                      full_range: bool = False) -> int:
    """A raw V_UNCOMPRESSED I420 Matroska segment of `frames` testsrc2-like frames (cycling
    `distinct` of them), the splitter's `-c copy` of raw video.  Returns
    its size in bytes."""
    import os
    from fractions import Fraction
    from .container import MkvWriter
    pool = [testsrc2_i420(w, h, t, full_range=full_range).tobytes() for t in range(min(distinct, max(frames, 1)))]
    with open(path, "wb") as f:
        wr = MkvWriter(f, w, h, Fraction(fps), codec="V_UNCOMPRESSED", colour_space=b"I420",
                       colour_range=2 if full_range else 0)
        for i in range(frames):
            wr.write_frame(pool[i % len(pool)])
        wr.close()
    return os.path.getsize(path)
