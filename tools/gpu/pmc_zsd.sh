#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmc_zsd"
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_zsd/w" -o w --output-format csv -- python3 "$R/tools/prof_zs_density.py" > "$R/gpurun_out/pmc_zsd/w.log" 2>&1; rc=$?
echo rc=$rc; exit $rc
