#!/bin/bash
# BASELINE config 4 with a FRESH dict per call (same key objects, new dict: the GBDT /
# feature-count pattern), real processes on one GPU, exchanges over the IPC mesh: the native
# walk's position hint on (default) vs off (MP4X_MAP_KEY_HINT=0), 4 and 8 processes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/maps2
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
run() {  # run <name> <p> [env...]
  local name=$1; local p=$2; shift 2
  local q=""; [ "$p" -gt 4 ] && q="GPU_MAX_HW_QUEUES=2"
  env $q "$@" timeout -k 10 300 python bench/map_api_procs.py --p $p --iters 3 --fresh-dict \
    > gpurun_out/maps2/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/maps2/$name.log; return $rc
}
run fresh_p4_hint 4 MP4X_MAP_KEY_HINT=1 && run fresh_p4_nohint 4 MP4X_MAP_KEY_HINT=0 && \
run fresh_p8_hint 8 MP4X_MAP_KEY_HINT=1 && run fresh_p8_nohint 8 MP4X_MAP_KEY_HINT=0
