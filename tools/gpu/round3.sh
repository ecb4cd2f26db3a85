#!/bin/bash
# Full GPU tests, kernel bench, N=1 bench, rocprofv3 kernel stats of the loopback schedules.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest rc=$rc; grep -v amdgpu.ids gpurun_out/pytest_gpu.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_kernels.py > gpurun_out/kbench5.log 2>&1; rc=$?; echo kbench rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_n1.log 2>&1; rc=$?; echo bench rc=$rc; grep metric gpurun_out/bench_n1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/loopback_paths.py > gpurun_out/loopback_paths.jsonl 2>&1; rc=$?; echo lb rc=$rc; grep -v amdgpu.ids gpurun_out/loopback_paths.jsonl
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
LB_ITERS=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/lbprof" -o lb --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench/loopback_paths.py" > "$GRAFT_REPO_ROOT/gpurun_out/lbprof.log" 2>&1; rc=$?
echo rocprof rc=$rc; find "$GRAFT_REPO_ROOT/gpurun_out/lbprof" -name "*kernel_stats.csv" | head -3
exit $rc
