#!/bin/bash
# The multi-rank bench flow with NP ranks sharing the GPU (gloo stands in for RCCL, real IPC
# kernels): verification, autotune, per-size sweep.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/rehearse
for np in ${NPS:-4 8}; do
  MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=$(( np > 4 ? 2 : 4 )) timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $np --master-addr 127.0.0.1 --master-port 2964$np bench.py --gpus $np --steps 5 --warmup 2 \
    --bytes ${BYTES:-268435456} --no-rccl-baseline $EXTRA > gpurun_out/rehearse/np$np.log 2>&1 || exit 1
  grep '^{' gpurun_out/rehearse/np$np.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({k: r[k] for k in ("n_gpus","ms_per_step","p50_ms","verified","max_abs_err")} | {"algo": r["config"]["algo"], "autotune_ms": r["config"]["autotune_ms"]}))'
done
