"""MI355X-native drop-in for the data-parallel hot path of Rouji/ffmpeg_distributed:
the per-segment worker (ffmpeg_distributed.py:131-141) for the profile
`[-vf scale=W:H:flags=bicubic] -c:v mjpeg -q:v N -dct int -huffman default -bitexact`.

- encoder.MjpegEncoder: HIP/gfx950 MJPEG encode over libmjgpu.so (include/mjgpu.h)
- dispatcher: the reference's split / queue / worker threads / concat, plus `gpu:N` hosts
- worker: the `gpu:N` worker process (stdin segment -> stdout segment)
"""
__version__ = "0.1.0"
