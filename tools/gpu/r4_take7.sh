#!/bin/bash
# Round 4, take 7: the zero-copy registered two-shot tests with HIP's error log on (which API call
# left "invalid argument" for PyTorch's next launch in take 6), then the whole GPU suite on the
# current tree (HIP error hygiene: failed mp4x HIP calls no longer stay the thread's last error).
source "$(dirname "$0")/steps.sh"
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
AMD_LOG_LEVEL=1 MP4X_TEST_LOG=1 step zc_diag 400 $PYT --timeout 200 tests/test_ipc_zc_gpu.py -k registered_two_shot_exact
step suite_full 780 $PYT -m gpu --timeout 400 --durations=30 tests
exit $STATUS
