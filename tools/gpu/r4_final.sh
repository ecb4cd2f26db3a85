#!/bin/bash
# Round 4, final check of the committed tree: host latency, the whole GPU suite (the driver's round-end tier),
# the N=1 bench, 2- and 4-rank bench rehearsals with the baseline configs (under the bench's own
# 60 s spin scope), and the smoke.
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
  step latency_layers 180 python bench/latency_layers.py --procs 2 --iters 3000
  step small_latency 180 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,1048576
) || exit $?
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step suite_full 800 $PYT -m gpu --timeout 400 --durations=30 tests
step bench_n1 240 python bench.py --steps 20 --warmup 5
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
  step bench_np2_rehearsal 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29661 bench.py --gpus 2 --steps 10 --warmup 3 --no-rccl-baseline --sweep-sizes 65536,4194304 \
    --no-rooted-sweep
  step bench_np4_rehearsal 360 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29662 bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline --sweep-sizes 65536,4194304
) || exit $?
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
grep -h '^{' gpurun_out/$OUT/latency_layers.log gpurun_out/$OUT/small_latency.log gpurun_out/$OUT/bench_n1.log \
  gpurun_out/$OUT/bench_np2_rehearsal.log gpurun_out/$OUT/bench_np4_rehearsal.log > gpurun_out/$OUT/all.jsonl || true
exit $STATUS
