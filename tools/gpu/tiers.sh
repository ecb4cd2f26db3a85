#!/bin/bash
# The one-shot / two-shot crossover on the staged tier: public-API latency with the schedule forced
# to ipc1 and to ipc2, at NPS ranks sharing the GPU, over SIZES.
#   OUT=<dir> [NPS="2 4"] [SIZES=262144,524288,1048576,2097152,4194304] bash tools/gpu/tiers.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
S=${SIZES:-262144,524288,1048576,2097152,4194304}
for np in ${NPS:-2 4}; do
  for a in ipc1 ipc2; do
    step ${a}_np$np 240 env MP4X_DEVICE_ALGO=$a python bench/small_latency.py --procs $np --iters 1000 --sizes $S || exit $?
    grep -h '^{' gpurun_out/$OUT/${a}_np$np.log | sed "s/^{/{\"forced\": \"$a\", /" >> gpurun_out/$OUT/tiers.jsonl || true
  done
done
exit $STATUS
