#!/bin/bash
# Round 4, take 10: latency after the host-side fixes (select memo by tier-state version, grid-cap
# fast path), plus a cProfile of rank 0's 4 KiB loop.
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
step latency_layers 240 python bench/latency_layers.py --procs 2 --iters 3000
step small_latency 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,1048576
step small_latency_prof 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096 \
  --profile gpurun_out/$OUT/prof
grep -h '^{' gpurun_out/$OUT/latency_layers.log gpurun_out/$OUT/small_latency.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
