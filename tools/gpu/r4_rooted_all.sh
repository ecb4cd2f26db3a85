#!/bin/bash
# Round 4: rooted-probe failure after the 4 MiB tier sweep — bisect in bench.py, then the
# isolated diagnostic with root = p - 1.
source "$(dirname "$0")/steps.sh"
bash tools/gpu/r4_rooted_bisect.sh
rc=$?; [ $rc -gt 2 ] && exit $rc
bash tools/gpu/r4_rooted_diag2.sh
exit $?
