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
