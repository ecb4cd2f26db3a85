#!/bin/bash
# run_pair.sh <ipc|vmm> <variant> [bytes]: the exporter and the importer of ipc_lifetime_repro as
# two independent processes; both outputs on stdout; rc = worst of both.  REPRO_BIN picks the build
# (default: the one linked against PyTorch's HIP runtime, tools/repro/build.sh).
B="${REPRO_BIN:-$(dirname "$0")/ipc_lifetime_repro}"
name="$1_$2_$$"
"$B" exporter "$1" "$2" "$name" "${3:-8388608}" &
e=$!
"$B" importer "$1" "$2" "$name" "${3:-8388608}"
ri=$?
wait $e
re=$?
r=$ri
[ $re -gt $r ] && r=$re
# the program's own failure codes (3 HIP error, 4 socket, 5 protocol) are an ordinary failed
# check for the step runner; a signal / time limit (>= 124) stays abnormal
[ $r -ge 3 ] && [ $r -le 5 ] && r=1
exit $r
