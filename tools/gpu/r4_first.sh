#!/bin/bash
# Round 4, first contact of the new IPC kernels: the operator matrix, the straggler families,
# then the whole GPU suite.
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -x -v --timeout-method thread -p no:cacheprovider"
step opmatrix 420 $PYT --timeout 300 tests/test_ipc_opmatrix_gpu.py
step straggler 600 $PYT --timeout 500 tests/test_ipc_straggler_gpu.py
step suite 900 python -u -m pytest -v --durations=25 --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu tests \
  --deselect tests/test_ipc_opmatrix_gpu.py --deselect tests/test_ipc_straggler_gpu.py
B=tools/repro/ipc_lifetime_repro
for v in close_before_free close_after_free never_close; do step repro_ipc_$v 60 $B ipc $v 8388608; done
for v in importer_first exporter_first keep_fds exporter_keeps importer_keeps concurrent; do
  step repro_vmm_$v 60 $B vmm $v 8388608
done
cat gpurun_out/$OUT/repro_*.log | grep '^{' > gpurun_out/$OUT/repro.jsonl || true
exit $STATUS
