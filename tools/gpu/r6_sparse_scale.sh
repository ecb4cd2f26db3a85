#!/bin/bash
# Round 6: config 4 after the split-staging exchanges, at more ranks on one GPU: the tensor form
# phase by phase (4 / 8 processes) and allreduceMap with real processes (same dict / fresh dict).
#   OUT=<dir> bash tools/gpu/r6_sparse_scale.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
step phases4 180 python bench/sparse_phases.py --procs 4 --iters 20
step phases8 240 python bench/sparse_phases.py --procs 8 --iters 20
step map4 240 python bench/map_api_procs.py --p 4 --iters 5
step map8 300 python bench/map_api_procs.py --p 8 --iters 5
step map8_fresh 300 python bench/map_api_procs.py --p 8 --iters 5 --fresh-dict
grep -h '^{' gpurun_out/$OUT/*.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
