#!/bin/bash
# Round 4: memAlloc's registered stand-in when only its self-test fails, plus the memAlloc /
# lifetime / policy modules on the current tree.
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step vmm 600 $PYT --timeout 300 tests/test_vmm_gpu.py tests/test_ipc_lifetime_gpu.py tests/test_vmm_policy_gpu.py \
  tests/test_ipc_zc_gpu.py
exit $STATUS
