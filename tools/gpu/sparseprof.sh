#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/spprof" -o sp --output-format csv -- python3 "$R/tools/prof_sparse.py" > "$R/gpurun_out/spprof.log" 2>&1; rc=$?
echo rc=$rc; exit $rc
