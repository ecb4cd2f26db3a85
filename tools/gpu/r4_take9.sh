#!/bin/bash
# Round 4, take 9: latency after the barrier fast path (spin bound read only by a waiting lane,
# peer Signal pointers from SGPRs): the same latency benches as take 8, then the IPC / straggler
# GPU tests that exercise the barrier.
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
  step latency_layers 240 python bench/latency_layers.py --procs 2 --iters 3000
  step small_latency 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,1048576
) || exit $?
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step ipc_tests 700 $PYT --timeout 400 tests/test_ipc_zc_gpu.py tests/test_ipc_straggler_gpu.py tests/test_ipc_opmatrix_gpu.py
grep -h '^{' gpurun_out/$OUT/*.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
