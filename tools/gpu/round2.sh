#!/bin/bash
# GPU tests + IPC protocol latency + rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
step() {
  local name=$1; local t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step ipc_lat 600 python bench/ipc_shared_gpu.py --procs 4
step prof_kernels 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kernels -o kb --output-format csv -- python tools/bench_kernels.py --quick --iters 10
step prof_bench 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/bench -o bench --output-format csv -- python bench.py --steps 10 --warmup 3
find gpurun_out/prof -name "*stats*" | head
