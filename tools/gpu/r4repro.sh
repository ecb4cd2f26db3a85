#!/bin/bash
# Round 4's rooted-probe failure, bisected on the round-4 tree: the same 4-rank bench flow once
# per variant.  Set the tree up first (on the CPU host; it travels with the snapshot, so take
# ./r4tree out of .gpurunignore for these calls):
#   git worktree add r4tree 586a5dd && (cd r4tree && git apply ../profiles/r5/rootcause/r4tree_bisect_knobs.patch
#     && python tools/build_native.py)      # + the acquire-wait build as libmp4x_hip_debug.so, see the patch
# Each
# variant = one round-5 change switched on by an environment variable of the patched worktree
# (R5_ORDERED, R5_LAZY_MEMALLOC, R5_PROBE_LARGE; MP4X_NATIVE_DEBUG=1 loads the build with the
# block_barrier acquire wait).  Lines "ruled out" per variant -> ruled_out_<variant>.txt.
# A variant "A+B" switches several on; TREE=. runs the current tree instead.
#   OUT=<dir> [VARIANTS="base R5_ORDERED ..."] [RUNS=1] [TREE=r4tree] bash tools/gpu/r4repro.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
port=29670
for v in ${VARIANTS:-base R5_ORDERED R5_LAZY_MEMALLOC R5_PROBE_LARGE MP4X_NATIVE_DEBUG}; do
  for k in $(seq 1 ${RUNS:-1}); do
    port=$((port + 1))
    extra=""
    [ "$v" != base ] && extra="$(echo $v | sed 's/+/=1 /g')=1"
    tree=${TREE:-r4tree}
    step r4_${v}_$k 300 env $extra MP4X_DEVICE_BACKEND=gloo MP4X_DEVICE_INDEX=0 MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w \
      python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port $port \
      $tree/bench.py --gpus 4 --steps 10 --warmup 3 --no-rccl-baseline --sweep-sizes 65536,4194304 --no-configs
    echo "$v run $k: $(grep -c 'ruled out' gpurun_out/$OUT/r4_${v}_$k.log) ruled out" | tee -a gpurun_out/$OUT/summary.txt
    grep -h "ruled out\|R5_PROBE" gpurun_out/$OUT/r4_${v}_$k.log > gpurun_out/$OUT/ruled_out_${v}_$k.txt || true
  done
done
exit $STATUS
