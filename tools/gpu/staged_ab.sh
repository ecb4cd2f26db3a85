#!/bin/bash
# VERDICT r2 Next #2: A/B of the STAGED two-shot's data buffers — fine-grained uncached (default)
# vs coarse-grained (MP4X_IPC_DATA_MEM=coarse, kept coherent by the kernels' system-scope
# release/acquire) — 1 GB f32 allreduce, 2 ranks on one GPU, unregistered buffer (--alloc plain)
# so every call stages through the 256 MiB instance in pieces.  Each run ends with bench.py's
# exact-pattern verification; the IPC self-test at mesh creation runs on the chosen memory too.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/staged_ab
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=5
run() {  # run <name> <np>
  local name=$1; local np=$2
  timeout -k 10 -s KILL 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port 29621 bench.py --gpus $np --steps 10 --warmup 3 --no-autotune --algo ipc2 --alloc plain \
    --no-rccl-baseline --no-tier-sweep --bytes ${BYTES:-1000000000} > gpurun_out/staged_ab/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{"metric"' gpurun_out/staged_ab/$name.log | python3 -c \
    'import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({k: r[k] for k in ("n_gpus","ms_per_step","p50_ms","p99_ms","verified","max_abs_err")} | {"calls": r["config"]["calls"], "selftest_ok": (r["config"]["ipc_selftest"] or {}).get("ok")}))'
  return $rc
}
run uncached_np2 2 && MP4X_IPC_DATA_MEM=coarse run coarse_np2 2 && \
run uncached_np4 4 && MP4X_IPC_DATA_MEM=coarse run coarse_np4 4
