#!/bin/bash
# In-situ A/B of the K1 grid cap for the N=1 bench (the out-of-place 1 GB copy = K1 with one
# input): default one-tile-per-block grid vs grid-stride caps, interleaved rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/k1ab
for round in 1 2 3; do
  for cap in 0 4096 8192 16384; do
    MP4X_K1_GRID=$cap timeout -k 10 120 python bench.py --steps 50 --warmup 10 > gpurun_out/k1ab/r${round}_cap$cap.json 2> /dev/null || exit 1
    python3 -c "import json,sys; r=json.load(open('gpurun_out/k1ab/r${round}_cap$cap.json')); print($round, $cap, r['ms_per_step'], r['value'], r['p50_ms'])"
  done
done
