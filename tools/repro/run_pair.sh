#!/bin/bash
# run_pair.sh <ipc|vmm> <variant> [bytes]: the exporter and the importer of
# ipc_lifetime_repro as two independent processes; both outputs on stdout; rc = worst of both.
B="$(dirname "$0")/ipc_lifetime_repro"
name="$1_$2_$$"
"$B" exporter "$1" "$2" "$name" "${3:-8388608}" &
e=$!
"$B" importer "$1" "$2" "$name" "${3:-8388608}"
ri=$?
wait $e
re=$?
[ $re -gt $ri ] && exit $re
exit $ri
