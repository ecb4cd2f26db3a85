#!/bin/bash
# Round 4, take 6: the rest of the GPU suite under the chunk-pool memAlloc (the straggler, operator
# matrix, memFree-policy, memAlloc and lifetime modules passed on their own in takes 3-5), then
# BASELINE configs 5 and 3 at 8 ranks on one GPU with no grid knob, a 2-rank bench rehearsal with
# the baseline configs, the N=1 bench and the smoke.
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step suite 700 $PYT -m gpu --timeout 120 --durations=25 tests \
  --deselect tests/test_ipc_straggler_gpu.py --deselect tests/test_ipc_opmatrix_gpu.py \
  --deselect tests/test_vmm_policy_gpu.py --deselect tests/test_vmm_gpu.py --deselect tests/test_ipc_lifetime_gpu.py
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=2 MP4X_WATCHDOG=0 MP4X_IPC_SPIN_S=60
  step cfg5_np8 300 $R --nproc-per-node 8 --master-port 29641 bench/collectives.py --config fp8_8gb --codecs fp8 \
    --check --iters 3 --warmup 1
) || exit $?
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=2 MP4X_WATCHDOG=0 MP4X_IPC_SPIN_S=60
  step cfg3_np8 240 $R --nproc-per-node 8 --master-port 29642 bench/collectives.py --config zero_bf16 --check \
    --iters 5 --warmup 2
) || exit $?
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=60 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
  step bench_np2_rehearsal 300 $R --nproc-per-node 2 --master-port 29643 bench.py --gpus 2 --steps 10 --warmup 3 \
    --no-rccl-baseline --sweep-sizes 65536,4194304 --no-rooted-sweep
) || exit $?
step bench_n1 240 python bench.py --steps 20 --warmup 5
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
grep -h '^{' gpurun_out/$OUT/*.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
