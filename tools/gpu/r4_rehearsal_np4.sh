#!/bin/bash
# Round 4: the multi-rank bench.py flow at 4 ranks on one GPU (gloo for RCCL; the IPC kernels for
# real), with the BASELINE configs under the bench's 60 s spin scope. (The N=8 case is the
# driver's round-end run; it is not started here.)
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
step bench_np4 420 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4 \
  --master-port 29671 bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline --sweep-sizes 65536,4194304
grep -h '^{' gpurun_out/$OUT/bench_np4.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
