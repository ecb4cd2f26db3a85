#!/bin/bash
# One GPU call that reproduces the driver's round-end checks from a CLEAN tree: build() from
# source (no prebuilt .so), the GPU test suite on those freshly built libraries, smoke(), the N=1
# bench, then the multi-rank bench flow with 2 / 4 / 8 ranks sharing the GPU (gloo for RCCL,
# real IPC kernels; the new verified / rccl_* / tier-sweep fields).  Each step has its own time
# limit; a failing step ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/round
set -o pipefail
step() { local name=$1; local t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/round/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
rm -rf build mp4x/_native/*.so
step build 900 python -c "import __graft_entry__ as g; g.build()" && ls -la mp4x/_native/ >> gpurun_out/round/build.log && \
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread && \
tail -3 gpurun_out/round/pytest_gpu.log && \
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && tail -1 gpurun_out/round/smoke.log && \
step bench_n1 300 python bench.py && grep '^{' gpurun_out/round/bench_n1.log | cut -c1-300 && \
for np in 2 4 8; do
  MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 GPU_MAX_HW_QUEUES=$(( np > 4 ? 2 : 4 )) step rehearsal_np$np 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $np --master-addr 127.0.0.1 --master-port 2963$np bench.py --gpus $np --steps 5 --warmup 2 \
    --bytes 268435456 --no-rccl-baseline || exit 1
  grep '^{' gpurun_out/round/rehearsal_np$np.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({k: r[k] for k in ("n_gpus","ms_per_step","p50_ms","verified","max_abs_err")} | {"algo": r["config"]["algo"], "selftest": (r["config"]["ipc_selftest"] or {}).get("ok"), "autotune_ms": r["config"]["autotune_ms"]}))'
done
