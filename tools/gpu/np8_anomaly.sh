#!/bin/bash
# the staged IPC two-shot allreduce of 80 MB took ~70 ms with 8 ranks on one
# GPU (0.39 ms with 4).  Kernel traces of rank 0 at 80 MB and 8 MB (8 ranks), then timing-only
# runs that vary one thing at a time: 4 ranks; 8 ranks with ONE hardware queue per process
# (GPU_MAX_HW_QUEUES=1: 8 queues in total instead of 32 — tests the queue-oversubscription
# explanation); 8 ranks at the 64 MiB buffer (the small instance instead of the 256 MiB one).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/np8
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=5
run() {  # run <name> <np> <bytes> <rank0 profiler args...>
  local name=$1; local np=$2; local b=$3; shift 3
  PROF0="$*" timeout -k 10 -s KILL 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port 29619 --no-python bash tools/gpu/rank_prof.sh \
    --gpus $np --steps ${STEPS:-10} --warmup 3 --no-autotune --algo ipc2 --alloc plain --no-rccl-baseline \
    --no-tier-sweep --bytes $b > gpurun_out/np8/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{"metric"' gpurun_out/np8/$name.log | python3 -c \
    'import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({k: r[k] for k in ("n_gpus","ms_per_step","p50_ms","p99_ms","verified")} | {"calls": r["config"]["calls"]}))'
  return $rc
}
run trace_np8_80MB 8 80000000 --kernel-trace --stats -f csv -d gpurun_out/np8/trace_np8_80MB -o rank0 && \
run trace_np8_8MB 8 8000000 --kernel-trace --stats -f csv -d gpurun_out/np8/trace_np8_8MB -o rank0 && \
run np4_80MB 4 80000000 && \
GPU_MAX_HW_QUEUES=1 run np8_80MB_1queue 8 80000000 && \
MP4X_IPC_TWOSHOT_MAX=134217728 MP4X_IPC_BYTES=134217728 run np8_80MB_smallinst 8 80000000
