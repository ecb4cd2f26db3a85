#!/bin/bash
# Round 4: the straggler test with both meshes (2 and 4 ranks) at the same time.
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step straggler 500 $PYT --timeout 400 --durations=5 tests/test_ipc_straggler_gpu.py
exit $STATUS
