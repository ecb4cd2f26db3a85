#!/bin/bash
# Rehearse the multi-rank bench path with 2 ranks sharing the single GPU (RCCL permitting).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export MP4X_DEVICE_INDEX=0 NCCL_DEBUG=WARN
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --bytes 100000000 > gpurun_out/dup.log 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/dup.log | tail -25
