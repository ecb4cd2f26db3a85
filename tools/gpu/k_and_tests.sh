#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/kbench3.log 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/kbench3.log | tail -12
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/bench_n1.log
