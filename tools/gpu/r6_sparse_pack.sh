#!/bin/bash
# Round 6: sparse exchanges with native record pack/unpack straight into the staging buffer.
# Exactness (sparse IPC + hash + copy-plan GPU tests), the config-4 phase breakdown at 2 ranks on
# one GPU, and one rocprofv3 kernel trace of it.
#   OUT=<dir> bash tools/gpu/r6_sparse_pack.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
step tests 420 $PYT tests/test_sparse_ipc_gpu.py tests/test_sparse_hash_gpu.py tests/test_ipc_plan_gpu.py
step phases 180 python bench/sparse_phases.py --procs 2 --iters 20
step trace 240 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/$OUT/trace" -o run -- \
  python3 bench/sparse_phases.py --procs 2 --iters 20
grep -h '^{' gpurun_out/$OUT/phases.log > gpurun_out/$OUT/phases.jsonl || true
exit $STATUS
