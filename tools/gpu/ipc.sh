#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests/test_ipc_gpu.py -x -q -m gpu > gpurun_out/ipc.log 2>&1; rc=$?; echo rc=$rc; grep -v amdgpu.ids gpurun_out/ipc.log | tail -40
