#!/bin/bash
# Round 4, take 8: host latency after the round-4 call-boundary checks (pinned error words read at
# every device collective), and a kernel-trace profile of a 2-rank bench rehearsal.
source "$(dirname "$0")/steps.sh"
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 TMPDIR=/tmp
step latency_layers 240 python bench/latency_layers.py --procs 2 --iters 3000
step small_latency 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,1048576
cat > /tmp/rank_bench.sh <<'EOS'
#!/bin/bash
if [ "$LOCAL_RANK" = "0" ]; then exec rocprofv3 --kernel-trace --stats -f csv -d $OUTDIR/trace -o rank0 -- python3 bench.py "$@"; fi
exec python3 bench.py "$@"
EOS
chmod +x /tmp/rank_bench.sh
OUTDIR=$PWD/gpurun_out/$OUT MP4X_IPC_SPIN_S=60 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w step bench_np2_trace 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29651 \
  --no-python bash /tmp/rank_bench.sh --gpus 2 --steps 10 --warmup 3 --no-rccl-baseline --sweep-sizes 65536 \
  --no-rooted-sweep
grep -h '^{' gpurun_out/$OUT/*.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
