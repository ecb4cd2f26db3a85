#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_kernels.py --variants > gpurun_out/kvariants.log 2>&1; echo rc=$?; cat gpurun_out/kvariants.log | grep -v amdgpu.ids
