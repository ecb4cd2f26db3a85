#!/bin/bash
# The operator matrix on the IPC kernels, 2 ranks sharing the GPU: per-call latency of every pair
# (hot compile-time-op kernels vs the runtime-op kernels), then a rank-0 kernel trace of
# Long.BITS_OR and Double.MAX (one kernel per call, no a2a detour).
source "$(dirname "$0")/steps.sh"
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 TMPDIR=/tmp
step opmatrix_np2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29631 bench/opmatrix.py
grep '^{' gpurun_out/$OUT/opmatrix_np2.log > gpurun_out/$OUT/opmatrix_np2.jsonl || true
cat > /tmp/rank_opm.sh <<'EOS'
#!/bin/bash
if [ "$LOCAL_RANK" = "0" ]; then exec rocprofv3 --kernel-trace --stats -f csv -d $OUTDIR/trace -o rank0 -- python3 bench/opmatrix.py "$@"; fi
exec python3 bench/opmatrix.py "$@"
EOS
chmod +x /tmp/rank_opm.sh
OUTDIR=$PWD/gpurun_out/$OUT step opmatrix_trace 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29632 --no-python bash /tmp/rank_opm.sh --pairs Long.BITS_OR,Double.MAX \
  --sizes 1048576 --iters 10 --warmup 2
exit $STATUS
