#!/bin/bash
# Round checkpoint: full GPU test suite, smoke(), N=1 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1; rc=$?
echo smoke rc=$rc; grep -v amdgpu.ids gpurun_out/smoke.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?; echo bench rc=$rc; grep metric gpurun_out/bench_default.log
exit $rc
