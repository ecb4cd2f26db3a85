#!/bin/bash
# The reference's table rows our round-2 sweeps did not cover, all ranks sharing ONE GPU (gloo
# stands in for RCCL, the IPC kernels run for real; protocol + correctness evidence, not xGMI):
#   * 6 ranks (the reference's 6-slave table, /root/reference/README.md:328-339), 1e5..1e8 doubles;
#   * the 1e9-double (8 GB per rank) rows at 2 / 4 / 6 / 8 ranks, on memAlloc arrays (zero-copy
#     kernels at any size), every op exact-checked.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sweep6
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=20
tr() {  # tr <name> <np> <timeout> <args...>
  local name=$1; local np=$2; local t=$3; shift 3
  local q=""; [ "$np" -gt 4 ] && q="GPU_MAX_HW_QUEUES=2"
  env $q timeout -k 10 $t python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port 29619 bench/collectives.py "$@" > gpurun_out/sweep6/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/sweep6/$name.log > gpurun_out/sweep6/$name.jsonl
  echo "exact rows: $(grep -c '"exact": true' gpurun_out/sweep6/$name.jsonl)"
  grep '"exact": false' gpurun_out/sweep6/$name.jsonl | cut -c1-300
  return $rc
}
if [ "${1:-a}" = "a" ]; then
  tr sweep_ref_np6 6 420 --sweep ref --check --iters 3 --warmup 1 --max-elems 1e8 && \
  tr sweep_1e9_np2 2 300 --sweep ref --check --iters 3 --warmup 1 --sizes 1e9 --sweep-alloc memalloc
else
  tr sweep_1e9_np4 4 300 --sweep ref --check --iters 3 --warmup 1 --sizes 1e9 --sweep-alloc memalloc && \
  tr sweep_1e9_np6 6 360 --sweep ref --check --iters 2 --warmup 1 --sizes 1e9 --sweep-alloc memalloc && \
  tr sweep_1e9_np8 8 420 --sweep ref --check --iters 2 --warmup 1 --sizes 1e9 --sweep-alloc memalloc
fi
