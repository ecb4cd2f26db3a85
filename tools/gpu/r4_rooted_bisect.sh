#!/bin/bash
# Round 4: bisect the rooted-sweep probe failure of the 4-rank rehearsal (reproducible after the
# 4 MiB tier sweep): peer-mapping close policy, push form, and the zero-copy candidates.
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4"
B="bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline --sweep-sizes 65536,4194304 --no-configs"
MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w MP4X_IPC_CLOSE_PEERS=0 step closepeers0 300 $R --master-port 29691 $B
MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z step nopush 300 $R --master-port 29692 $B
MP4X_AUTOTUNE_CANDIDATES=ipc2 step staged_only 300 $R --master-port 29693 $B
for f in closepeers0 nopush staged_only; do echo "== $f"; grep "ruled out" gpurun_out/$OUT/$f.log; done > gpurun_out/$OUT/ruled_out.txt
exit $STATUS
