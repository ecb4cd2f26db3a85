#!/bin/bash
# The round-end check of the committed tree, as the driver runs it plus the multi-rank rehearsals:
# the whole GPU suite, smoke(), the N=1 bench, bench.py --gpus 2/4/8 rehearsals on the one GPU,
# the latency layers.
#   OUT=<dir> bash tools/gpu/round.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
step suite 1000 python -u -m pytest -v --timeout 170 --timeout-method thread -p no:cacheprovider -m gpu \
  --durations=25 tests
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench_n1 240 python bench.py --steps 20 --warmup 5
for np in 2 4 8; do
  q=$(( np > 4 ? 2 : 4 ))
  t0=$(date +%s)
  step bench_np$np 540 env MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=$q \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((29650 + np)) bench.py --gpus $np --steps 10 --warmup 3 --no-rccl-baseline
  echo "np$np wall_s $(( $(date +%s) - t0 ))" | tee -a "gpurun_out/$OUT/walltime.txt"
done
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
  step latency_layers 240 python bench/latency_layers.py --procs 2 --iters 3000
) || exit $?
grep -E "PASSED|FAILED|ERROR|passed|failed" "gpurun_out/$OUT/suite.log" > "gpurun_out/$OUT/suite_results.txt" || true
grep -h '^{' gpurun_out/$OUT/bench_*.log gpurun_out/$OUT/latency_layers.log > "gpurun_out/$OUT/all.jsonl" || true
exit $STATUS
