#!/bin/bash
# The shared-GPU rehearsals' per-size sweep runs at ~24 ms (one-shot) / ~35 ms (two-shot) per
# call from 256 KiB up with 4 and 8 ranks, while the 256 MiB headline of the same processes
# takes 0.65 / 1.39 ms.  Vary one thing at a time (4 ranks, 16 MiB headline, no rooted sweep):
#   base      default sweep order, rank 0 kernel trace
#   rev       sweep sizes in reverse order (is it the size or the point in time?)
#   q1        GPU_MAX_HW_QUEUES=1
#   nowd      MP4X_WATCHDOG=0
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sweep
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
run() {  # run <name> <np> <extra bench args> ; PROF0 from env
  local name=$1; local np=$2; shift 2
  timeout -k 10 -s KILL 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np \
    --master-addr 127.0.0.1 --master-port 29631 --no-python bash tools/gpu/rank_prof.sh \
    --gpus $np --steps 5 --warmup 2 --bytes 16777216 --no-rccl-baseline --no-rooted-sweep "$@" \
    > gpurun_out/sweep/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  grep '^{"metric"' gpurun_out/sweep/$name.log | python3 -c \
    'import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({"p50": r["p50_ms"], "sweep": r["config"]["tier_sweep_ms"]}))'
  return $rc
}
PROF0="--kernel-trace --stats -f csv -d gpurun_out/sweep/trace_base -o rank0" run base 4 && \
run rev 4 --sweep-sizes 67108864,16777216,4194304,1048576,262144,65536,4096 && \
GPU_MAX_HW_QUEUES=1 run q1 4 && \
MP4X_WATCHDOG=0 run nowd 4
