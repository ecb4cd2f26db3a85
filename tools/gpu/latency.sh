export OUT=${OUT:-latency}
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
step fast_tests 600 $PYT tests/test_fast_path_gpu.py tests/test_ipc_straggler_gpu.py tests/test_graph_gpu.py tests/test_ipc_gpu.py
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
  step latency_layers 240 python bench/latency_layers.py --procs 2 --iters 3000
  step small_latency 240 python bench/small_latency.py --procs 2 --iters 2000 --sizes 4096,65536,1048576
  step all_ops 240 python bench/small_latency.py --procs 2 --iters 2000 --all-ops --sizes 4096,800000
) || exit $?
step coherence 120 python bench/coherence_probe.py --rounds 200
step coherence_64k 120 python bench/coherence_probe.py --rounds 50 --region-vecs 4096
grep -h '^{' gpurun_out/$OUT/latency_layers.log gpurun_out/$OUT/small_latency.log gpurun_out/$OUT/all_ops.log \
  > gpurun_out/$OUT/latency.jsonl || true
grep -h '^{' gpurun_out/$OUT/coherence.log gpurun_out/$OUT/coherence_64k.log > gpurun_out/$OUT/coherence.jsonl || true
exit $STATUS
