#!/bin/bash
# Build the standalone PMC experiment binaries (run on the CPU container before a gpurun call;
# the binaries are not tracked).  Used by tools/gpu/exp_zsr.sh and tools/gpu/exp_zsw.sh.
set -e
cd "$(dirname "$0")"
for x in zs_real zs_writes; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-result -I../../csrc/include -o "$x" "$x.hip"
done
