#!/bin/bash
# Round 6: the dry-run findings re-checked, the IPC-mode test (legacy mode forced), the node-aware
# tests after the opt-in change.
#   OUT=<dir> bash tools/gpu/r6_misc.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu"
MP4X_TEST_RECORD="$PWD/gpurun_out/$OUT/ipc_mode.jsonl" step ipc_mode 300 $PYT tests/test_ipc_mode_gpu.py
step hier 300 $PYT tests/test_hier_gpu.py
MP4X_TEST_MULTI_DRYRUN=1 step dryrun_fixes 700 $PYT tests/test_multigpu_gpu.py -k "autotuners or thread_comm or hier"
exit $STATUS
