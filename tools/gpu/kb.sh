#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "fp8 or quant" > gpurun_out/pytest_kb.log 2>&1; rc=$?
echo pytest rc=$rc; tail -2 gpurun_out/pytest_kb.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_kernels.py > gpurun_out/kbench7.log 2>&1; rc=$?; echo kbench rc=$rc
grep -v amdgpu.ids gpurun_out/kbench7.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
for k,v in d.items(): print(f'{k:45s} {v[\"ms\"]:.4f} ms {v[\"GBps\"]:.0f} GB/s')"
exit $rc
