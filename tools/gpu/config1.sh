#!/bin/bash
# BASELINE config 1 (2-thread in-process float[1024] allreduceArray, CPU only) on the box's CPU
# share: the native team through the CPython binding with the GIL hand-off chain (default), the
# chain off, and the r1 ctypes path; then pinned placements (same cpu / two cpus).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/cfg1
O=gpurun_out/cfg1/config1.jsonl; : > $O
lscpu -e=CPU,CORE,SOCKET,NODE > gpurun_out/cfg1/lscpu.txt 2>&1 || true
cat /sys/fs/cgroup/cpuset.cpus.effective >> gpurun_out/cfg1/lscpu.txt 2>/dev/null || true
run() { timeout -k 5 60 "$@" >> $O || exit 1; }
for r in 1 2 3 4 5; do run python bench/thread_cpu.py --iters 5000; done
for r in 1 2 3; do MP4X_TEAM_HANDOFF_US=0 run python bench/thread_cpu.py --iters 5000; done
for r in 1 2 3; do MP4X_TEAM_EXT=0 MP4X_TEAM_HANDOFF_US=0 run python bench/thread_cpu.py --iters 5000; done
C=$(python -c "import os; c=sorted(os.sched_getaffinity(0)); print(c[0], c[1], c[len(c)//2])")
set -- $C
for r in 1 2; do echo "{\"pin\": \"$1\"}" >> $O; run taskset -c $1 python bench/thread_cpu.py --iters 3000; done
for r in 1 2; do echo "{\"pin\": \"$1,$2\"}" >> $O; run taskset -c $1,$2 python bench/thread_cpu.py --iters 5000; done
for r in 1 2; do echo "{\"pin\": \"$1,$3\"}" >> $O; run taskset -c $1,$3 python bench/thread_cpu.py --iters 5000; done
run python bench/thread_cpu.py --iters 5000 --threads 4
cat $O
