#!/bin/bash
# Round 4, take 11: latency with the ctypes-free launcher + capture state passed down, then the IPC,
# graph and debug-build GPU tests (every staged allreduce now launches through _mp4x_launch).
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
  step latency_layers 240 python bench/latency_layers.py --procs 2 --iters 3000
  step small_latency 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,1048576
  step small_latency_prof 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096 --profile gpurun_out/$OUT/prof
) || exit $?
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step gpu_tests 700 $PYT --timeout 300 -m gpu tests/test_ipc_gpu.py tests/test_ipc_zc_gpu.py tests/test_ipc_opmatrix_gpu.py \
  tests/test_graph_gpu.py tests/test_debug_build_gpu.py tests/test_ipc_stress_gpu.py
grep -h '^{' gpurun_out/$OUT/latency_layers.log gpurun_out/$OUT/small_latency.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
