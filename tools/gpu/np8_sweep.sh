#!/bin/bash
# VERDICT r2 weak #5, second half: the anomaly does not reproduce in bench.py (8 ranks, 80 MB,
# staged two-shot: 0.70 ms, profiles/r3/np8_anomaly.txt); here the SWEEP harness itself at 1e7
# doubles, 8 ranks on one GPU: allreduce alone, then the full op sequence (rank 0 traced), to
# see which preceding op's leftovers the allreduce rows absorbed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/np8s
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=5
cat > /tmp/rank_coll.sh <<'EOS'
#!/bin/bash
if [ "$LOCAL_RANK" = "0" ] && [ -n "$PROF0" ]; then exec rocprofv3 $PROF0 -- python3 bench/collectives.py "$@"; fi
exec python3 bench/collectives.py "$@"
EOS
run() {  # run <name> <ops> <rank0 profiler args...>
  local name=$1; local ops=$2; shift 2
  PROF0="$*" timeout -k 10 -s KILL 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29623 --no-python bash /tmp/rank_coll.sh \
    --sweep ref --check --iters 3 --warmup 1 --sizes 1e7 --ops $ops > gpurun_out/np8s/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/np8s/$name.log | cut -c1-260
  return $rc
}
run allreduce_only allreduce && \
run full_seq gather,scatter,allgather,reduce_scatter,broadcast,reduce,allreduce && \
run full_seq_traced gather,scatter,allgather,reduce_scatter,broadcast,reduce,allreduce \
  --kernel-trace --stats -f csv -d gpurun_out/np8s/trace -o rank0
