#!/bin/bash
# K4b partition-pack numerics + sparse loopback paths, then kernel bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_loopback_gpu.py -m gpu -x -q > gpurun_out/pytest_pack.log 2>&1; rc=$?
echo pytest rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_pack.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/kbench4.log 2>&1; rc=$?; echo rc=$rc; grep -v amdgpu.ids gpurun_out/kbench4.log | tail -40
exit $rc
