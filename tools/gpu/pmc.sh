#!/bin/bash
# rocprofv3 PMC counters for the mp4x kernels (kernel-trace/stats only; no sys/runtime trace).
# gfx950 TCC has 4 slots per pass: FETCH_SIZE (3) and WRITE_SIZE (2) need separate passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc "$@" -d gpurun_out/pmc/$name -o $name --output-format csv -- python tools/bench_kernels.py --quick --iters 3 --mb 512 > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then grep -v "^    @" gpurun_out/pmc/$name.log | tail -5; exit $rc; fi; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run l2 TCC_HIT_sum TCC_MISS_sum
run waves SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
ls gpurun_out/pmc/*
