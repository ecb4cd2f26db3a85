#!/bin/bash
# rocprofv3 kernel stats of the IPC two-shot allreduce: 2 ranks sharing ONE GPU (gloo for the
# host-side collectives), 64 MiB f32, algorithm pinned to ipc2.  Each rank runs under its own
# rocprofv3 (torchrun never touches the GPU itself).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ipcprof
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_DEVICE_ALGO=${ALGO:-ipc2}
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29613 --no-python rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/ipcprof -o rank_%pid% \
  -- python3 bench.py --gpus 2 --steps 20 --warmup 3 --no-autotune --bytes ${BYTES:-67108864} > gpurun_out/ipcprof.log 2>&1
rc=$?; echo rc=$rc; grep metric gpurun_out/ipcprof.log; ls -R gpurun_out/ipcprof | head -20
exit $rc
