#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_loopback_gpu.py -m gpu -x -q -k "zs or loopback" > gpurun_out/pytest_zs.log 2>&1; rc=$?
echo pytest rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_zs.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_kernels.py > gpurun_out/kbench6.log 2>&1; rc=$?; echo kbench rc=$rc; grep -A2 k6b gpurun_out/kbench6.log
exit $rc
