#!/bin/bash
# bench.py's multi-rank flow, unchanged (autotune, timed steps, verification, early headline line,
# budgeted extras: tier sweep, rooted sweep, BASELINE configs 3-5), with NP ranks sharing this box's
# one GPU: gloo stands in for RCCL (RCCL refuses two ranks per GPU), the IPC kernels run for real.
# Records each run's wall time (the driver's 8-GPU run must stay well inside its timeout).
# A rank count may repeat (NPS="8 8 8": a soak of the whole flow); runs after the first get a suffix.
#   OUT=<dir> NPS="4 8" [BYTES=1000000000] [EXTRA="--no-configs"] [LIMIT=540] bash tools/gpu/rehearsal.sh
source "$(dirname "$0")/steps.sh"
declare -A seen
for np in ${NPS:-2 4 8}; do
  k=${seen[$np]:-0}; seen[$np]=$((k + 1))
  tag=np$np; [ "$k" -gt 0 ] && tag=np${np}_$k
  q=$(( np > 4 ? 2 : 4 ))                    # hardware queues per process when 8 share the GPU
  t0=$(date +%s)
  step bench_$tag ${LIMIT:-540} env MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=$q \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((29640 + np + 10 * k)) bench.py --gpus $np --steps ${STEPS:-10} --warmup 3 --bytes ${BYTES:-1000000000} \
    --no-rccl-baseline $EXTRA
  echo "$tag wall_s $(( $(date +%s) - t0 ))" | tee -a "gpurun_out/$OUT/walltime.txt"
  grep -h '^{' "gpurun_out/$OUT/bench_$tag.log" > "gpurun_out/$OUT/bench_$tag.jsonl" || true
  grep -h "ruled out\|probe failed\|first-use" "gpurun_out/$OUT/bench_$tag.log" > "gpurun_out/$OUT/ruled_out_$tag.txt" || true
done
exit $STATUS
