#!/bin/bash
# The reference's table (7 collectives x 1e5..1e8 doubles, exact-value check per row) and the
# BASELINE configs 3 (4 GB bf16 RS+AG) and 5 (8 GB fp8 allreduce) at full size, with 2/4/8 ranks
# sharing ONE GPU: gloo stands in for RCCL, the IPC kernels run for real.  Protocol and
# correctness evidence; the times are ranks time-slicing one GPU, not xGMI bandwidth.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sweep
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
tr() {  # tr <name> <np> <timeout> <args...>
  local name=$1; local np=$2; local t=$3; shift 3
  timeout -k 10 $t python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port 29617 bench/collectives.py "$@" > gpurun_out/sweep/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/sweep/$name.log > gpurun_out/sweep/$name.jsonl
  grep -c '"exact": true' gpurun_out/sweep/$name.jsonl; grep '"exact": false' gpurun_out/sweep/$name.jsonl | cut -c1-300
  return $rc
}
tr sweep_ref_np2 2 400 --sweep ref --check --iters 5 --warmup 2 --max-elems ${MAXE:-1e8} && \
tr sweep_ref_np4 4 500 --sweep ref --check --iters 5 --warmup 2 --max-elems ${MAXE:-1e8} && \
tr sweep_ref_np8 8 500 --sweep ref --check --iters 3 --warmup 1 --max-elems ${MAXE8:-1e7} && \
tr config3_zero_bf16_np4 4 400 --config zero_bf16 --check --iters 3 --warmup 1 && \
tr config5_fp8_8gb_np4 4 400 --config fp8_8gb --codecs fp8 --check --iters 3 --warmup 1
