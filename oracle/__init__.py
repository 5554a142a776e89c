"""CPU oracle for the MJPEG segment-encode hot path -- TEST INFRASTRUCTURE ONLY.

Restates FFmpeg's mjpeg encoder (-dct int, -huffman default, -bitexact) and the
swscale bicubic / tv->pc range path that the reference's worker runs
(ffmpeg_distributed.py:131-141).  See mjpeg_oracle.c for the per-function FFmpeg
citations and the parity status ("unpinned against FFmpeg": FFmpeg is absent from
/root/reference, this container and the GPU box).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
from .oracle import *  # noqa: F401,F403
