#!/bin/bash
# Round 4, take 4: the memFree lifetime study — every MP4X_VMM_POLICY for exactness and device
# memory growth (tests/test_vmm_policy_gpu.py), the plain-HIP reproducer on the runtime mp4x runs
# on, the memAlloc tests, the operator-matrix timing + kernel trace; last, the /opt/rocm build
# of the reproducer with the fd passed by value (unknown convention: a crash there ends the call).
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step vmm_policy 420 $PYT --timeout 220 tests/test_vmm_policy_gpu.py
bash tools/gpu/r4_repro.sh
rc=$?; [ $rc -gt 2 ] && exit $rc
step vmm_tests 420 $PYT --timeout 200 tests/test_vmm_gpu.py tests/test_ipc_lifetime_gpu.py
bash tools/gpu/r4_opprof.sh
rc=$?; [ $rc -gt 2 ] && exit $rc
REPRO_BIN=tools/repro/ipc_lifetime_repro_sys REPRO_FD_BY_VALUE=1 step repro_sys_byvalue_ordered 60 \
  tools/repro/run_pair.sh vmm ordered
grep -h '^{' gpurun_out/$OUT/repro_sys*.log >> gpurun_out/$OUT/repro.jsonl || true
exit $STATUS
