#!/bin/bash
# One gpurun call: GPU tests, smoke, 1-GPU bench, kernel micro-bench.  Each GPU step has
# its own time limit; a crash/timeout/abort (anything but a plain test failure) stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1; local t=$2; shift 2
  echo "== $name" ; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python bench.py --steps 10 --warmup 3
step kbench 300 python tools/bench_kernels.py
