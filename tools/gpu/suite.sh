#!/bin/bash
# The GPU test suite (the driver's round-end tier), or a subset: one pytest process, every test
# under pytest-timeout, the whole call under its own limit.
#   OUT=<dir> [TESTS="tests/test_ipc_lifetime_gpu.py"] [K="expr"] [LIMIT=900] bash tools/gpu/suite.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
step suite ${LIMIT:-900} python -u -m pytest -v --timeout ${TEST_TIMEOUT:-300} --timeout-method thread \
  -p no:cacheprovider -m gpu ${K:+-k "$K"} --durations=25 ${TESTS:-tests}
grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" "gpurun_out/$OUT/suite.log" > "gpurun_out/$OUT/suite_results.txt" || true
exit $STATUS
