#!/bin/bash
# Zero-copy two-shot allreduce (registered buffer, MP4X_DEVICE_ALGO=ipc2z), 2 ranks sharing ONE
# GPU, 1 GB f32: (1) rocprofv3 kernel trace + stats of every rank, (2)/(3) PMC passes on rank 0
# only (FETCH_SIZE, then WRITE_SIZE: device-wide counters, so they include rank 1's traffic of the
# same step).  Staged two-shot (ALGO=ipc2) for comparison with STAGED=1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/zcprof
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_DEVICE_ALGO=${ALGO:-ipc2z} MP4X_IPC_SPIN_S=5
B=${BYTES:-1000000000}
run() {  # run <name> <timeout> <rank0 profiler args...>
  local name=$1; local t=$2; shift 2
  PROF0="$*" timeout -k 10 -s KILL $t python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29615 --no-python bash tools/gpu/rank_prof.sh \
    --gpus 2 --steps ${STEPS:-10} --warmup 3 --no-autotune $EXTRA --bytes $B > gpurun_out/zcprof/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{"metric"' gpurun_out/zcprof/$name.log | cut -c1-400
  return $rc
}
run trace_$ALGO$TAG 300 --kernel-trace --stats -f csv -d gpurun_out/zcprof/trace_$ALGO$TAG -o rank_%pid% && \
STEPS=3 run pmc_fetch_$ALGO$TAG 120 --pmc FETCH_SIZE -f csv -d gpurun_out/zcprof/pmc_fetch_$ALGO$TAG -o rank_%pid% && \
STEPS=3 run pmc_write_$ALGO$TAG 120 --pmc WRITE_SIZE -f csv -d gpurun_out/zcprof/pmc_write_$ALGO$TAG -o rank_%pid%
