#!/bin/bash
# PMC byte accounting of the round-3 zero-copy paths (separate --pmc passes, FETCH_SIZE then
# WRITE_SIZE, on rank 0 only; the counters are device-wide, so with every rank on one GPU a
# dispatch window holds the traffic of all ranks' copies of the same barrier-synchronised kernel):
#  * BASELINE config 3 on memAlloc (4 ranks): k_ipc_reduce_range + k_ipc_gather per step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=5
cat > /tmp/rank_coll_pmc.sh <<'EOS'
#!/bin/bash
if [ "$LOCAL_RANK" = "0" ] && [ -n "$PROF0" ]; then exec rocprofv3 $PROF0 -- python3 bench/collectives.py "$@"; fi
exec python3 bench/collectives.py "$@"
EOS
for c in FETCH_SIZE WRITE_SIZE; do
  PROF0="--pmc $c -f csv -d gpurun_out/pmc3/$c -o rank0" timeout -k 10 -s KILL 240 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29629 --no-python bash /tmp/rank_coll_pmc.sh \
    --config zero_bf16 --iters 2 --warmup 1 --alloc memalloc > gpurun_out/pmc3/run_$c.log 2>&1 || exit 1
  echo "$c rc=0"
done
