#!/bin/bash
# Round 4 first contact, take 2: the lifetime reproducers as two independent processes, then the
# operator matrix / straggler / whole suite with the round-3 memAlloc pool (MP4X_VMM_RELEASE=0:
# the ordered VMM release still made the next allocation's peer views read wrong in take 1).
source "$(dirname "$0")/steps.sh"
bash tools/gpu/r4_repro.sh
rc=$?; [ $rc -gt 2 ] && exit $rc
export MP4X_VMM_RELEASE=0
PYT="python -u -m pytest -x -v --timeout-method thread -p no:cacheprovider"
step opmatrix 420 $PYT --timeout 300 tests/test_ipc_opmatrix_gpu.py
step straggler 600 $PYT --timeout 500 tests/test_ipc_straggler_gpu.py
step suite 900 python -u -m pytest -v --durations=25 --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests --deselect tests/test_ipc_opmatrix_gpu.py --deselect tests/test_ipc_straggler_gpu.py
exit $STATUS
