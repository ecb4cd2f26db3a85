#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/exp_zsw"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$R/gpurun_out/exp_zsw/w" -o w --output-format csv -- "$R/tools/exp/zs_writes" > "$R/gpurun_out/exp_zsw/w.log" 2>&1; rc=$?
echo rc=$rc; tail -2 "$R/gpurun_out/exp_zsw/w.log"; exit $rc
