#!/bin/bash
# 8-rank bench flow on ONE GPU with the autotune correctness probe (p = 8 pattern, m = 12):
# IPC candidates only (gloo would stand in for RCCL), 64 MiB and 1 MiB payloads.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
: > gpurun_out/probe_np8.jsonl
for b in 1048576 67108864; do
  NP=8 BYTES=$b CANDS=ipc1,ipc2,ipc2p bash tools/gpu/bench_rehearsal.sh > /dev/null || { tail -20 gpurun_out/rehearsal.log; exit 1; }
  grep '^{' gpurun_out/rehearsal.log >> gpurun_out/probe_np8.jsonl
  grep -i "autotune" gpurun_out/rehearsal.log | grep -v "^{" | head -5
done
python3 -c "
import json
for l in open('gpurun_out/probe_np8.jsonl'):
    d = json.loads(l); print(d['n_gpus'], d['config']['payload_bytes'], d['config']['algo'], d['config']['autotune_ms'], d['p50_ms'])"
