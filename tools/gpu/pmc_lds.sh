#!/bin/bash
# PMC counters of the LDS-staged kernels (kernel-trace/stats + pmc only).
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/pmc_lds"
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc_lds/avail.txt" 2>&1 || true
grep -oE "SQ_[A-Z_]*LDS[A-Z_]*" "$R/gpurun_out/pmc_lds/avail.txt" | sort -u > "$R/gpurun_out/pmc_lds/lds_counters.txt" || true
cat "$R/gpurun_out/pmc_lds/lds_counters.txt"
run() { local name=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --pmc "$@" -d "$R/gpurun_out/pmc_lds/$name" -o $name --output-format csv -- python3 "$R/tools/prof_lds.py" > "$R/gpurun_out/pmc_lds/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then grep -v "^    @" "$R/gpurun_out/pmc_lds/$name.log" | tail -5; exit $rc; fi; }
run fetch FETCH_SIZE
run write WRITE_SIZE
C=""; for c in SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE; do grep -qx "$c" "$R/gpurun_out/pmc_lds/lds_counters.txt" && C="$C $c"; done
echo "lds counters: $C"
[ -n "$C" ] && run lds $C
exit 0
