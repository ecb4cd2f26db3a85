#!/bin/bash
# Round checkpoint + N=1 bench kernel profile (rocprofv3 --kernel-trace --stats).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
bash tools/gpu/full.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- \
  python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_bench.log 2>&1; rc=$?
echo prof rc=$rc; find gpurun_out/prof_bench -name '*kernel_stats.csv' | head -3
exit $rc
