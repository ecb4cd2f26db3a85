#!/bin/bash
# BASELINE config 5 (8 GB f32 allreduce, fused fp8 two-shot) at full size, 4 ranks on ONE GPU:
# the whole quantised tensor (~2 GB) staged in a VMM-built IPC buffer -> ONE quantise + ONE fused
# kernel per call (round 2: 256 MiB pieces).  Error-bounded check vs the fp64 sum; rank-0 trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/cfg5
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_IPC_SPIN_S=5
cat > /tmp/rank_coll5.sh <<'EOS'
#!/bin/bash
if [ "$LOCAL_RANK" = "0" ] && [ -n "$PROF0" ]; then exec rocprofv3 $PROF0 -- python3 bench/collectives.py "$@"; fi
exec python3 bench/collectives.py "$@"
EOS
run() {  # run <name> <rank0 profiler args...>
  local name=$1; shift 1
  PROF0="$*" timeout -k 10 -s KILL 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29627 --no-python bash /tmp/rank_coll5.sh \
    --config fp8_8gb --codecs fp8 --check --iters 3 --warmup 1 > gpurun_out/cfg5/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; grep '^{' gpurun_out/cfg5/$name.log | cut -c1-400
  return $rc
}
run onepiece_traced --kernel-trace --stats -f csv -d gpurun_out/cfg5/trace -o rank0 && \
MP4X_FP8_ONE_PIECE=0 run pieces
