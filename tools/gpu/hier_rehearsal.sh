#!/bin/bash
# The bench flow as a 2-node job: 8 ranks on one GPU simulated as 2 nodes x 4 ranks
# (MP4X_SIM_NODE_SIZE=4): no global IPC mesh, the node-aware allreduce (IPC sub-mesh per "node",
# gloo standing in for RCCL across) against the flat transport allreduce; verified result.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/hier
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=2 MP4X_SIM_NODE_SIZE=4
MP4X_AUTOTUNE_CANDIDATES=hier,rccl timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29671 bench.py --gpus 8 --steps 5 --warmup 2 --bytes 268435456 \
  --no-rccl-baseline --no-tier-sweep --no-rooted-sweep --autotune-iters 2 > gpurun_out/hier/np8_2nodes.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/hier/np8_2nodes.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({k: r[k] for k in ("n_gpus","ms_per_step","p50_ms","verified","max_abs_err")} | {"algo": r["config"]["algo"], "autotune_ms": r["config"]["autotune_ms"], "calls": r["config"]["calls"]}))'
exit $rc
