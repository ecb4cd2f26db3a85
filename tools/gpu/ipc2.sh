#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ipc_gpu.py -x -q -m gpu > gpurun_out/ipc.log 2>&1; rc=$?; echo rc=$rc; grep -v amdgpu.ids gpurun_out/ipc.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench/ipc_shared_gpu.py --procs 2 > gpurun_out/ipc_lat2.log 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/ipc_lat2.log
