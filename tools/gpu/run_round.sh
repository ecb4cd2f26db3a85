#!/bin/bash
# One gpurun call: GPU tests, smoke, 1-GPU bench, and (REHEARSE=1) multi-rank bench rehearsals
# with every rank on the one GPU (gloo for the transport schedules, IPC kernels for real).
# Each GPU step has its own time limit; a crash/timeout/abort (anything but a plain test
# failure) stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1; local t=$2; shift 2
  echo "== $name" ; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc"; grep -v "amdgpu.ids\|hostname of the client\|Gloo\] Rank\|Expected number" "gpurun_out/$name.log" | tail -${TAILN:-6}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rehearse() {  # rehearse <name> <np> [env...]
  local name=$1; local np=$2; shift 2
  step "$name" 400 env MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_AUTOTUNE_CANDIDATES=${CANDS:-rccl,ipc2,ipc2p,ipc2z} "$@" \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus $np --steps 5 --warmup 2 --bytes ${BYTES:-1000000000}
}
if [ -z "$NOTESTS" ]; then
  step pytest_gpu 900 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step bench1 300 python bench.py --steps 10 --warmup 3
fi
if [ -n "$REHEARSE" ]; then
  rehearse rehearsal_np2 2
  rehearse rehearsal_np4 4
  rehearse rehearsal_np2_inject 2 MP4X_IPC_SELFTEST_INJECT=1
fi
