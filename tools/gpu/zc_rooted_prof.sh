#!/bin/bash
# rocprofv3 kernel stats of rank 0 while the 7 collectives of the reference's table run on a
# memAlloc array (1e8 doubles, 4 ranks sharing one GPU): every collective should be ONE
# zero-copy IPC kernel per call (k_ipc_twoshot / k_ipc_reduce_range / k_ipc_gather /
# k_ipc_copy_plan) with no __amd_rocclr_copyBuffer and no staging copies.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/zcprof
export TMPDIR=/tmp MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
cat > /tmp/rank_zc.sh <<'EOS'
#!/bin/bash
if [ "$LOCAL_RANK" = "0" ]; then exec rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/zcprof/trace -o rank0 -- python3 bench/collectives.py "$@"; fi
exec python3 bench/collectives.py "$@"
EOS
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29627 --no-python bash /tmp/rank_zc.sh --sweep ref --check --iters 3 --warmup 1 --sizes 1e8 \
  --sweep-alloc memalloc > gpurun_out/zcprof/run.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/zcprof/run.log | cut -c1-200
find gpurun_out/zcprof/trace -name '*kernel_stats.csv' -exec cp {} gpurun_out/zcprof/rank0_kernel_stats.csv \;
cut -d, -f1-4 gpurun_out/zcprof/rank0_kernel_stats.csv | head -20
exit $rc
