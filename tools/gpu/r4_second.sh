#!/bin/bash
# Round 4, second call: BASELINE config 5 (8 GB fp8-compressed allreduce) at 8 ranks on one GPU
# with NO grid knob (co-residency caps derived from occupancy), config 3 at 8 ranks, the operator
# matrix timing + kernel trace, and the round-end N=1 bench + smoke.
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=2 MP4X_WATCHDOG=0 MP4X_IPC_SPIN_S=60
  step cfg5_np8 420 $R --nproc-per-node 8 --master-port 29641 bench/collectives.py --config fp8_8gb --codecs fp8 \
    --check --iters 3 --warmup 1
) || exit $?
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=2 MP4X_WATCHDOG=0 MP4X_IPC_SPIN_S=60
  step cfg3_np8 300 $R --nproc-per-node 8 --master-port 29642 bench/collectives.py --config zero_bf16 --check \
    --iters 5 --warmup 2
) || exit $?
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=60 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
  step bench_np2_rehearsal 480 $R --nproc-per-node 2 --master-port 29643 bench.py --gpus 2 --steps 10 --warmup 3 \
    --no-rccl-baseline --sweep-sizes 65536,4194304 --no-rooted-sweep
) || exit $?
bash tools/gpu/r4_opprof.sh
rc=$?; [ $rc -gt 2 ] && exit $rc
step bench_n1 300 python bench.py --steps 20 --warmup 5
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
grep -h '^{' gpurun_out/$OUT/*.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
