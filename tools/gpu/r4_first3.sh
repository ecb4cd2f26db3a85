#!/bin/bash
# Round 4 first contact, take 3: the memFree policies side by side (tests/test_vmm_policy_gpu.py),
# the plain-HIP lifetime reproducers, then the operator matrix / straggler / lifetime / whole
# suite under the default policy — or under "pool" when the default one was not exact.
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step vmm_policy 420 $PYT --timeout 200 tests/test_vmm_policy_gpu.py
if grep -q "test_memfree_policy_then_new_allocation_is_exact\[fresh_va\] FAILED" gpurun_out/$OUT/vmm_policy.log; then
  echo "fresh_va not exact: the rest runs with MP4X_VMM_POLICY=pool" | tee -a gpurun_out/$OUT/progress.log
  export MP4X_VMM_POLICY=pool
fi
bash tools/gpu/r4_repro.sh
rc=$?; [ $rc -gt 2 ] && exit $rc
step opmatrix 420 $PYT -x --timeout 300 tests/test_ipc_opmatrix_gpu.py
step straggler 600 $PYT -x --timeout 500 tests/test_ipc_straggler_gpu.py
step lifetime 600 $PYT --timeout 320 tests/test_ipc_lifetime_gpu.py
step suite 900 $PYT -m gpu --timeout 120 --durations=25 tests \
  --deselect tests/test_ipc_opmatrix_gpu.py --deselect tests/test_ipc_straggler_gpu.py \
  --deselect tests/test_ipc_lifetime_gpu.py --deselect tests/test_vmm_policy_gpu.py
exit $STATUS
