#!/bin/bash
# BASELINE configs 3 (4 GB bf16 RS + AG, memAlloc, zero-copy) and 5 (8 GB f32 fp8-compressed
# allreduce, fused IPC fp8 two-shot) with 8 ranks sharing one GPU (gloo stands in for RCCL).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/cfg8
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=2
run() { local name=$1; shift
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29651 bench/collectives.py "$@" > gpurun_out/cfg8/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/cfg8/$name.log | tee gpurun_out/cfg8/$name.jsonl | cut -c1-400; return $rc; }
run config3_np8 --config zero_bf16 --check --iters 3 --warmup 1 && \
run config5_np8 --config fp8_8gb --codecs fp8 --check --iters 3 --warmup 1
