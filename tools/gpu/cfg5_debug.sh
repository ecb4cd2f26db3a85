cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/cfg5
export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29652 bench/collectives.py --config fp8_8gb --codecs fp8 --check --iters 3 --warmup 1 > gpurun_out/cfg5/np4.log 2>&1
echo "np4 rc=$?"; grep '^{' gpurun_out/cfg5/np4.log | cut -c1-300
GPU_MAX_HW_QUEUES=2 MP4X_IPC_SPIN_S=30 MP4X_WATCHDOG=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29653 bench/collectives.py --config fp8_8gb --codecs fp8 --check --iters 3 --warmup 1 > gpurun_out/cfg5/np8.log 2>&1
echo "np8 rc=$?"; grep '^{' gpurun_out/cfg5/np8.log | cut -c1-300; grep -i "timed out\|Mp4jException\|Error" gpurun_out/cfg5/np8.log | grep -v Gloo | head -5 | cut -c1-300
