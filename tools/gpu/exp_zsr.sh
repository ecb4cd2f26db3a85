#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/exp_zsr"
for d in 0 0.05; do
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$R/gpurun_out/exp_zsr/w$d" -o w --output-format csv -- "$R/tools/exp/zs_real" $d > "$R/gpurun_out/exp_zsr/w$d.log" 2>&1; rc=$?
echo d=$d rc=$rc; grep done "$R/gpurun_out/exp_zsr/w$d.log"; [ $rc -eq 0 ] || exit $rc
done
