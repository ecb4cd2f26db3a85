#!/bin/bash
# Round 4: why the rooted autotune probe ruled out broadcast / gather / scatter 'ipc' at 1 MiB in
# the 4-rank rehearsal (tools/diag/rooted_probe.py records every rank's agreement values).
source "$(dirname "$0")/steps.sh"
export MP4X_AUTOTUNE_CANDIDATES=ipc2,ipc2z,ipc2w
step rooted_np4 240 python tools/diag/rooted_probe.py 4
step rooted_np2 240 python tools/diag/rooted_probe.py 2
exit $STATUS
