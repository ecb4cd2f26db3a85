#!/bin/bash
# Round-3 map records on the GPU box's CPU share:
#  (1) host allreduceMap (Dict[str, float32[16]], 50k keys/rank) columnar path at p = 2 / 4 / 8, and
#      the round-2 per-entry path (MP4X_HOST_MAP_COLUMNAR=0) at p = 8 for contrast;
#  (2) BASELINE config 4 FIRST call (200k new keys per rank, 8 processes): key-dictionary round
#      peer to peer (default) vs through the master (MP4X_KEYS_VIA_MASTER=1, the round-2 path).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/maps
for p in 2 4 8; do
  timeout -k 10 240 python bench/host_map.py --p $p --iters 7 > gpurun_out/maps/host_map_p$p.log 2>&1 || exit 1
  tail -1 gpurun_out/maps/host_map_p$p.log
done
MP4X_HOST_MAP_COLUMNAR=0 timeout -k 10 240 python bench/host_map.py --p 8 --iters 7 > gpurun_out/maps/host_map_p8_entries.log 2>&1 || exit 1
tail -1 gpurun_out/maps/host_map_p8_entries.log
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
timeout -k 10 400 python bench/map_api_procs.py --p 8 --iters 2 --fresh-dict > gpurun_out/maps/cfg4_p8_p2p.log 2>&1 || exit 1
tail -1 gpurun_out/maps/cfg4_p8_p2p.log
MP4X_KEYS_VIA_MASTER=1 timeout -k 10 400 python bench/map_api_procs.py --p 8 --iters 2 --fresh-dict > gpurun_out/maps/cfg4_p8_master.log 2>&1 || exit 1
tail -1 gpurun_out/maps/cfg4_p8_master.log
