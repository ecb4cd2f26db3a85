#!/bin/bash
# Round 6: the cross-GPU test module in dry-run mode (every rank on cuda:0, gloo for RCCL), the
# stream-order soak with its outcomes recorded, and the latency layers after the guard.
#   OUT=<dir> [NO_DRYRUN=1] [NO_LATENCY=1] bash tools/gpu/r6_check.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu"
MP4X_TEST_RECORD="$PWD/gpurun_out/$OUT/stream_order.jsonl" step stream_order 600 $PYT tests/test_stream_order_gpu.py
if [ -z "$NO_LATENCY" ]; then
  (
    export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
    step latency_layers 240 python bench/latency_layers.py --procs 2 --iters 3000
    step small_latency 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,1048576
    step all_ops 240 python bench/small_latency.py --procs 2 --iters 2000 --all-ops --sizes 4096,800000
  ) || exit $?
  grep -h '^{' gpurun_out/$OUT/latency_layers.log gpurun_out/$OUT/small_latency.log gpurun_out/$OUT/all_ops.log \
    > gpurun_out/$OUT/latency.jsonl || true
fi
if [ -z "$NO_DRYRUN" ]; then
  MP4X_TEST_MULTI_DRYRUN=1 step multigpu_dryrun ${DRY_LIMIT:-1500} $PYT --durations=40 tests/test_multigpu_gpu.py ${K:+-k "$K"}
  grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" "gpurun_out/$OUT/multigpu_dryrun.log" \
    > "gpurun_out/$OUT/multigpu_dryrun.txt" || true
fi
exit $STATUS
