#!/bin/bash
# Fused fp8 IPC two-shot, wide (16 B per lane) vs the r1 narrow form (MP4X_FP8_NARROW=1):
# bit-exactness tests, shared-GPU timing (2 procs, 256 MiB f32 payload) and a PMC pass on rank 0
# of a 2-rank bench.py --codec fp8 run (vector-memory read instructions, TCP->TCC read requests).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/fp8prof
export TMPDIR=/tmp
for v in 0 1; do
  MP4X_FP8_NARROW=$v timeout -k 10 200 python -u -m pytest tests/test_ipc_fp8_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/fp8prof/tests_narrow$v.log 2>&1 || { echo "tests narrow=$v failed"; exit 1; }
  tail -1 gpurun_out/fp8prof/tests_narrow$v.log
  MP4X_FP8_NARROW=$v timeout -k 10 200 python bench/ipc_shared_gpu.py --procs 2 --iters 20 --sizes 268435456 \
    --buf-mib 300 --algos 1,2 > gpurun_out/fp8prof/bench_narrow$v.log 2>&1 || { echo "bench narrow=$v failed"; exit 1; }
  grep '^{' gpurun_out/fp8prof/bench_narrow$v.log | sed "s/^/narrow=$v /"
  MP4X_FP8_NARROW=$v PROF0="--pmc SQ_INSTS_VMEM_RD TCP_TCC_READ_REQ_sum -f csv -d gpurun_out/fp8prof/pmc_narrow$v -o rank_%pid%" \
    MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 timeout -k 10 -s KILL 150 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29619 --no-python bash tools/gpu/rank_prof.sh \
    --gpus 2 --steps 3 --warmup 2 --no-autotune --no-register --codec fp8 --bytes 268435456 \
    > gpurun_out/fp8prof/pmc_narrow$v.log 2>&1 || { echo "pmc narrow=$v failed"; exit 1; }
  echo "pmc narrow=$v done"
done
