#!/bin/bash
# Per-kernel VGPR / SGPR / scratch / occupancy / LDS of libmjgpu's kernels for the current sources
# (or SRC=dir holding api.hip & friends).  Extra args: hipcc flags (e.g. -DFOO).
cd "${SRC:-$(dirname "$0")/../ffmpeg_distributed_amd/csrc}"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1 -Xclang -target-feature -Xclang -dot6-insts -Xclang -target-feature -Xclang -dot4-insts -I"$(dirname "$0")/../include" -I/root/repo/include \
  --cuda-device-only -c -o /tmp/regs.o "$@" api.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1); print(); print(cur[:60].ljust(60), end=""); continue
    m = re.search(r"remark: +(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|SGPRs Spill): (\d+)", line)
    if m and cur:
        print(f"  {m.group(1).split()[0]}={m.group(2)}", end="")
print()'
