#!/bin/bash
# Round 4, first contact of the new IPC kernels: the operator matrix, the straggler families,
# then the whole GPU suite.
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -x -v --timeout-method thread -p no:cacheprovider"
step opmatrix 420 $PYT --timeout 300 tests/test_ipc_opmatrix_gpu.py
step straggler 600 $PYT --timeout 500 tests/test_ipc_straggler_gpu.py
step suite 900 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests \
  --deselect tests/test_ipc_opmatrix_gpu.py --deselect tests/test_ipc_straggler_gpu.py
exit $STATUS
