#!/bin/bash
# Print k_encode VGPR/scratch for the current sources (optionally extra -D flags).
cd "$(dirname "$0")/../ffmpeg_distributed_amd/csrc"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I../../include --cuda-device-only -c -o /tmp/regs.o "$@" api.hip -Rpass-analysis=kernel-resource-usage 2>&1 | grep -A7 "${KERNEL:-k_encode}" | grep -E "error|VGPRs:|SGPRs:|Scratch|Occupancy" | sed 's/.*remark: *//' | tr '\n' ' '; echo
