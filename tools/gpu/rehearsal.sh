#!/bin/bash
# bench.py's multi-rank flow, unchanged (autotune, timed steps, verification, early headline line,
# budgeted extras: tier sweep, rooted sweep, BASELINE configs 3-5), with NP ranks sharing this box's
# one GPU: gloo stands in for RCCL (RCCL refuses two ranks per GPU), the IPC kernels run for real.
# Records each run's wall time (the driver's 8-GPU run must stay well inside its timeout).
#   OUT=<dir> NPS="4 8" [BYTES=1000000000] [EXTRA="--no-configs"] [LIMIT=540] bash tools/gpu/rehearsal.sh
source "$(dirname "$0")/steps.sh"
for np in ${NPS:-2 4 8}; do
  q=$(( np > 4 ? 2 : 4 ))                    # hardware queues per process when 8 share the GPU
  t0=$(date +%s)
  step bench_np$np ${LIMIT:-540} env MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=$q \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((29640 + np)) bench.py --gpus $np --steps ${STEPS:-10} --warmup 3 --bytes ${BYTES:-1000000000} \
    --no-rccl-baseline $EXTRA
  echo "np$np wall_s $(( $(date +%s) - t0 ))" | tee -a "gpurun_out/$OUT/walltime.txt"
  grep -h '^{' "gpurun_out/$OUT/bench_np$np.log" > "gpurun_out/$OUT/bench_np$np.jsonl" || true
  grep -h "ruled out\|probe failed\|first-use" "gpurun_out/$OUT/bench_np$np.log" > "gpurun_out/$OUT/ruled_out_np$np.txt" || true
done
exit $STATUS
