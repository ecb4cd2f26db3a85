#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -40
