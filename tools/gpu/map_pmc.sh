#!/bin/bash
# PMC (FETCH_SIZE, WRITE_SIZE; one counter group per run) of the config-4 Map API kernels
# (K4b pack, K3 row take, K5 reduce-by-key) on the 8-virtual-rank bench, 2 iterations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  MAP_ITERS=1 timeout -s KILL 240 rocprofv3 --pmc $c -f csv -d gpurun_out/mappmc_$c -o pmc -- \
    python3 bench/map_api.py > gpurun_out/map_pmc_$c.log 2>&1 || exit $?
done
find gpurun_out/mappmc_* -name "*counter_collection.csv" | head
