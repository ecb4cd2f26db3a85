#!/bin/bash
# Round 4: is the rooted-sweep probe failure of the 4-rank bench rehearsal reproducible, and does
# it depend on the watchdog thread?  (bench.py only logs the verdicts on rank 0)
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4"
step np4_default 300 $R --master-port 29681 bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline \
  --sweep-sizes 65536,4194304 --no-configs
MP4X_WATCHDOG=0 step np4_nowd 300 $R --master-port 29682 bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline \
  --sweep-sizes 65536,4194304 --no-configs
step np4_nosweep 300 $R --master-port 29683 bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline \
  --sweep-sizes 65536 --no-configs
grep -h "ruled out" gpurun_out/$OUT/*.log > gpurun_out/$OUT/ruled_out.txt || true
exit $STATUS
