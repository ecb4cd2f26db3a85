#!/bin/bash
# Autotune correctness probes on ONE GPU: every IPC candidate must pass the exact-pattern probe
# (finite autotune time) for 2 and 4 ranks, small (one-shot) and large (pieces) messages.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rccl_variant_gpu.py \
  > gpurun_out/probe_tests.log 2>&1 || { tail -20 gpurun_out/probe_tests.log; exit 1; }
tail -1 gpurun_out/probe_tests.log
: > gpurun_out/probe_rehearsal.jsonl
for cfg in "2 1048576 rccl,ipc1,ipc2,a2a" "2 268435456 rccl,ipc2,ipc2p,a2a" "4 4194304 rccl,ipc1,ipc2,a2a,rhd"; do
  set -- $cfg
  NP=$1 BYTES=$2 CANDS=$3 bash tools/gpu/bench_rehearsal.sh > /dev/null || { tail -20 gpurun_out/rehearsal.log; exit 1; }
  grep '^{' gpurun_out/rehearsal.log >> gpurun_out/probe_rehearsal.jsonl
  grep -i "autotune" gpurun_out/rehearsal.log | grep -v "^{" | head -5
done
python3 - <<'PY'
import json
for l in open("gpurun_out/probe_rehearsal.jsonl"):
    d = json.loads(l); print(d["n_gpus"], d["config"]["payload_bytes"], d["config"]["algo"], d["config"]["autotune_ms"])
PY
