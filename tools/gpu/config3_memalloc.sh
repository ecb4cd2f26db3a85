#!/bin/bash
# VERDICT r2 Next #2: BASELINE config 3 (reduce-scatter + all-gather of a 4 GB bf16 tensor) on a
# memAlloc tensor (zero-copy RS / AG kernels at any size), 4 ranks on ONE GPU (gloo for RCCL):
# exact check + rank-0 kernel trace (no __amd_rocclr_copyBuffer inside the step) + the staged
# torch.empty form for contrast.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/cfg3
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=5
cat > /tmp/rank_coll3.sh <<'EOS'
#!/bin/bash
if [ "$LOCAL_RANK" = "0" ] && [ -n "$PROF0" ]; then exec rocprofv3 $PROF0 -- python3 bench/collectives.py "$@"; fi
exec python3 bench/collectives.py "$@"
EOS
run() {  # run <name> <alloc> <rank0 profiler args...>
  local name=$1; local alloc=$2; shift 2
  PROF0="$*" timeout -k 10 -s KILL 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-4} \
    --master-addr 127.0.0.1 --master-port 29625 --no-python bash /tmp/rank_coll3.sh \
    --config zero_bf16 --check --iters ${ITERS:-5} --warmup 2 --alloc $alloc > gpurun_out/cfg3/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/cfg3/$name.log | cut -c1-400
  return $rc
}
run memalloc_traced memalloc --kernel-trace --stats -f csv -d gpurun_out/cfg3/trace -o rank0 && \
run memalloc memalloc && \
ITERS=2 run staged plain
