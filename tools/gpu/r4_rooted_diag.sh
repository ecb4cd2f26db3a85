#!/bin/bash
# Round 4: why the rooted autotune probe ruled out broadcast / gather / scatter 'ipc' at 1 MiB in
# the 4-rank rehearsal (tools/diag/rooted_probe.py records every rank's agreement values), with
# bench.py's preceding steps replayed in stages.
source "$(dirname "$0")/steps.sh"
export MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
step rooted_np4_full 300 python tools/diag/rooted_probe.py 4 head+tune1g+tiers
step rooted_np4_tiers 240 python tools/diag/rooted_probe.py 4 tiers
step rooted_np4_head 240 python tools/diag/rooted_probe.py 4 head+tune1g
exit $STATUS
