#!/bin/bash
# IPC tests (incl. pipelined large messages) + shared-GPU protocol bench of the large path.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ipc_gpu.py -x -q -m gpu > gpurun_out/ipc.log 2>&1; rc=$?; echo rc=$rc; grep -v amdgpu.ids gpurun_out/ipc.log | tail -8
[ $rc -eq 0 ] || exit $rc
for ov in 1 0; do
  MP4X_IPC_OVERLAP=$ov timeout -k 10 300 python bench/ipc_shared_gpu.py --procs 2 --iters 10 --sizes 268435456 --buf-mib 64 --algos 1 > gpurun_out/ipc_large_ov$ov.log 2>&1; rc=$?
  echo overlap=$ov rc=$rc; grep -v amdgpu.ids gpurun_out/ipc_large_ov$ov.log | tail -3
  [ $rc -eq 0 ] || exit $rc
done
