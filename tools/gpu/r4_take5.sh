#!/bin/bash
# Round 4, take 5: the chunk-pool memAlloc (new default) — the policy study, the memAlloc and
# lifetime tests, then the whole GPU suite.
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step vmm_policy 420 $PYT --timeout 220 tests/test_vmm_policy_gpu.py
step vmm_tests 420 $PYT --timeout 200 tests/test_vmm_gpu.py tests/test_ipc_lifetime_gpu.py
step suite 900 $PYT -m gpu --timeout 120 --durations=25 tests \
  --deselect tests/test_vmm_policy_gpu.py --deselect tests/test_vmm_gpu.py --deselect tests/test_ipc_lifetime_gpu.py
exit $STATUS
