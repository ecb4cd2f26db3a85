#!/bin/bash
# N=2 rehearsal of the multi-rank bench flow on ONE GPU: both ranks on cuda:0, gloo instead of
# RCCL for the "rccl" schedule (RCCL refuses two ranks per GPU), IPC kernels for real.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_AUTOTUNE_CANDIDATES=${CANDS:-rccl,ipc2,ipc2p,a2a}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus ${NP:-2} --steps 5 --warmup 2 --bytes ${BYTES:-268435456} > gpurun_out/rehearsal.log 2>&1
rc=$?; echo rc=$rc; grep -v "amdgpu.ids\|Warning\|hostname" gpurun_out/rehearsal.log | tail -15
exit $rc
