#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_kernels.py --variants > gpurun_out/kvariants2.log 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/kvariants2.log
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/kbench2.log 2>&1; echo rc=$?; grep -v amdgpu.ids gpurun_out/kbench2.log
