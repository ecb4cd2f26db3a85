#!/bin/bash
# Round 4: the rooted probes with root = p - 1 (as bench.py) and root = 0, 4 ranks.
source "$(dirname "$0")/steps.sh"
export MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
step rooted_np4_root3 240 python tools/diag/rooted_probe.py 4
DIAG_ROOT=0 step rooted_np4_root0 240 python tools/diag/rooted_probe.py 4
step rooted_np4_root3_tiers 240 python tools/diag/rooted_probe.py 4 tiers
exit $STATUS
