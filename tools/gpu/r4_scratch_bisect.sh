#!/bin/bash
# Round 4: which half of the scratch lifecycle precedes the rooted-probe failure (4-rank bench
# rehearsal): the scratch free (MP4X_IPC_SCRATCH_FREE=0 pools it) or the peers' close of their
# scratch mappings (MP4X_IPC_SCRATCH_CLOSE=0 keeps them); then the registration / zero-copy /
# lifetime tests on the default path.
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
(
  export MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
  R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 4"
  B="bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline --sweep-sizes 65536,4194304 --no-configs"
  MP4X_IPC_SCRATCH_FREE=0 step scratch_pooled 300 $R --master-port 29701 $B
  MP4X_IPC_SCRATCH_CLOSE=0 step scratch_kept_mapped 300 $R --master-port 29702 $B
) || exit $?
PYT="python -u -m pytest -v --timeout-method thread -p no:cacheprovider"
step default_tests 500 $PYT --timeout 300 tests/test_ipc_zc_gpu.py tests/test_ipc_lifetime_gpu.py tests/test_ipc_gpu.py
for f in scratch_pooled scratch_kept_mapped; do echo "== $f"; grep "ruled out" gpurun_out/$OUT/$f.log; done > gpurun_out/$OUT/ruled_out.txt
exit $STATUS
