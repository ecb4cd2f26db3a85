#!/bin/bash
# Round 6: FETCH_SIZE / WRITE_SIZE of K5d (dense reduce-by-key, dictionary ids) and of the K4b
# halves (pack A/B), one counter per pass.
#   OUT=<dir> bash tools/gpu/r6_pmc_sparse.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  step k5d_$c 120 rocprofv3 --pmc $c --output-format csv -d "gpurun_out/$OUT/k5d_$c" -o run -- \
    python3 bench/sparse_rbk.py --ps 8 --dense-ids --paths dense --iters 20
  step pack_$c 120 rocprofv3 --pmc $c --output-format csv -d "gpurun_out/$OUT/pack_$c" -o run -- \
    python3 bench/pack_ab.py --ns 200000 --ps 8 --iters 20
done
exit $STATUS
