#!/bin/bash
# Config-4 Map API on the box: bench/map_api.py (8 virtual ranks, 200k keys x float[64]) and its
# rocprofv3 kernel stats.  Each GPU step has its own limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench/map_api.py > gpurun_out/map_api.log 2>&1 || exit $?
tail -2 gpurun_out/map_api.log
MAP_SWITCH_S=0.0002 timeout -k 10 300 python bench/map_api.py > gpurun_out/map_api_switch.log 2>&1 || exit $?
tail -1 gpurun_out/map_api_switch.log
MAP_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/mapprof -o mapprof -- \
  python3 bench/map_api.py > gpurun_out/map_prof.log 2>&1 || exit $?
find gpurun_out/mapprof -name "*kernel_stats.csv" | head -3
