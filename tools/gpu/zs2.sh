#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_loopback_gpu.py -m gpu -x -q -k "zs or loopback" > gpurun_out/pytest_zs.log 2>&1; rc=$?
echo pytest rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_zs.log | tail -5
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/zsprof2" -o zs --output-format csv -- python3 "$R/tools/zs_prof.py" > "$R/gpurun_out/zsprof2.log" 2>&1; rc=$?
echo rc=$rc
exit $rc
