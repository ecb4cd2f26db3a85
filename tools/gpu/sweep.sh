#!/bin/bash
# The reference's published table shape (bench/collectives.py --sweep ref): every collective of
# the table over double[] of 1e5 .. MAX elements, exact-checked, NPS ranks sharing this box's GPU
# (gloo stands in for RCCL, the IPC kernels run for real).  One JSON line per (op, size).
#   OUT=<dir> [NPS="2 4"] [MAX=1e8] [LIMIT=400] bash tools/gpu/sweep.sh
source "$(dirname "$0")/steps.sh"
for np in ${NPS:-2 4}; do
  q=$(( np > 4 ? 2 : 4 ))
  step sweep_np$np ${LIMIT:-400} env MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=$q \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((29700 + np)) bench/collectives.py --sweep ref --check --max-elems ${MAX:-1e8} || exit $?
  grep -h '^{' "gpurun_out/$OUT/sweep_np$np.log" > "gpurun_out/$OUT/sweep_np$np.jsonl" || true
done
exit $STATUS
