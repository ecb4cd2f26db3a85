#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_ipc_gpu.py tests/test_ipc_stress_gpu.py -m gpu -x -q > gpurun_out/ipcstress.log 2>&1; rc=$?
echo rc=$rc; grep -v amdgpu.ids gpurun_out/ipcstress.log | tail -25
exit $rc
