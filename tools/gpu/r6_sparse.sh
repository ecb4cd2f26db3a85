#!/bin/bash
# Round 6: K5h (hash reduce-by-key) exactness tests, the sort-vs-hash A/B on config 4's shape, and
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes for each path (one counter group a run).
#   OUT=<dir> bash tools/gpu/r6_sparse.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
step sparse_tests 300 $PYT tests/test_sparse_hash_gpu.py
step rbk_ab 240 python bench/sparse_rbk.py --ps 2,8 --iters 50
for path in sort hash; do
  step trace_$path 180 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/$OUT/trace_$path" -o run -- \
    python3 bench/sparse_rbk.py --ps 8 --iters 20 --paths $path
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc_${path}_$c 120 rocprofv3 --pmc $c --output-format csv -d "gpurun_out/$OUT/pmc_${path}_$c" -o run -- \
      python3 bench/sparse_rbk.py --ps 8 --iters 20 --paths $path
  done
done
grep -h '^{' gpurun_out/$OUT/rbk_ab.log > gpurun_out/$OUT/rbk_ab.jsonl || true
exit $STATUS
