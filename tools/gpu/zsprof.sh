#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/zsprof" -o zs --output-format csv -- python3 "$R/tools/zs_prof.py" > "$R/gpurun_out/zsprof.log" 2>&1; rc=$?
echo rc=$rc; f=$(find "$R/gpurun_out/zsprof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
