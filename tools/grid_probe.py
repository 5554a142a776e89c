#!/usr/bin/env python3
"""Open a c2 encoder on a variant library with MJG_DEBUG_GRID=1 (the variant prints its k_encode
grid: CUs, workgroups per CU, LDS).  usage: python3 tools/grid_probe.py NAME"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["MJG_DEBUG_GRID"] = "1"
from ffmpeg_distributed_amd import _lib  # noqa: E402
_lib.LIB_PATH = os.path.join(ROOT, "ffmpeg_distributed_amd", f"libmjgpu_v_{sys.argv[1]}.so")
from ffmpeg_distributed_amd.encoder import MjpegEncoder  # noqa: E402
enc = MjpegEncoder(0, 3840, 2160, 3840, 2160, full_range=False, qscale=5, max_batch=8, huffman="default")
enc.close()
