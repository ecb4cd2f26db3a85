#!/bin/bash
# Kernel numerics (incl. K8 FIRST) + loopback device engine (RHD, map family) with real kernels.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py tests/test_loopback_gpu.py tests/test_thread_gpu.py -m gpu -x -q > gpurun_out/pytest_maps.log 2>&1; rc=$?
echo pytest rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_maps.log | tail -25
exit $rc
