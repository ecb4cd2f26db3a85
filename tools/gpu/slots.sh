#!/bin/bash
# The IPC kernel families after a change to the barrier / one-shot protocol: every IPC test module
# that drives the kernels (self-test, soak with rank skew, straggler, graphs, operator matrix, fast
# path, zero-copy), then the latency layers at 2 ranks with and without the slots, and the staged
# two-shot's sizes (1-4 MiB) with slots of 4 MiB (slotted) and 256 KiB (its end barrier kept).
#   OUT=<dir> [NO_TESTS=1] bash tools/gpu/slots.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
[ -n "$NO_TESTS" ] || step ipc_tests 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_ipc_stress_gpu.py tests/test_ipc_gpu.py tests/test_ipc_zc_gpu.py tests/test_fast_path_gpu.py \
  tests/test_graph_gpu.py tests/test_ipc_straggler_gpu.py tests/test_ipc_opmatrix_gpu.py tests/test_ipc_plan_gpu.py
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
  step layers_slots 240 python bench/latency_layers.py --procs 2 --iters 3000
  step layers_noslots 240 env MP4X_IPC_SLOTS=0 python bench/latency_layers.py --procs 2 --iters 3000
  step small_slots 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,262144
  step small_noslots 240 env MP4X_IPC_SLOTS=0 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,262144
  step small_slots_p4 240 python bench/small_latency.py --procs 4 --iters 2000 --sizes 4096,65536
  step small_noslots_p4 240 env MP4X_IPC_SLOTS=0 python bench/small_latency.py --procs 4 --iters 2000 --sizes 4096,65536
  S2=1048576,2097152,4194304
  step two_slots 240 python bench/small_latency.py --procs 2 --iters 1000 --sizes $S2
  step two_noslots 240 env MP4X_IPC_SLOT_BYTES=262144 python bench/small_latency.py --procs 2 --iters 1000 --sizes $S2
  step two_slots_p4 240 python bench/small_latency.py --procs 4 --iters 1000 --sizes $S2
  step two_noslots_p4 240 env MP4X_IPC_SLOT_BYTES=262144 python bench/small_latency.py --procs 4 --iters 1000 --sizes $S2
) || exit $?
for f in layers_slots layers_noslots small_slots small_noslots small_slots_p4 small_noslots_p4 \
         two_slots two_noslots two_slots_p4 two_noslots_p4; do
  grep -h '^{' gpurun_out/$OUT/$f.log | sed "s/^{/{\"variant\": \"$f\", /" >> gpurun_out/$OUT/latency.jsonl || true
done
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/$OUT/ipc_tests.log > gpurun_out/$OUT/ipc_tests_results.txt || true
exit $STATUS
