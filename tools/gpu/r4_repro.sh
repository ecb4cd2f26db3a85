#!/bin/bash
# The two memory-lifetime anomalies as standalone two-process HIP programs (no torch / mp4x):
# every variant of the release ordering, one JSON line per check (tools/repro/ipc_lifetime_repro.hip),
# on the HIP runtime mp4x runs on (PyTorch's).  Last: the /opt/rocm build with the fd passed by
# value (which convention that runtime expects is not known; a crash there ends the call).
source "$(dirname "$0")/steps.sh"
P=tools/repro/run_pair.sh
for v in close_before_free close_after_free never_close; do step repro_ipc_$v 60 $P ipc $v; done
for v in ordered exporter_first fresh_va keep_owner_va keep_import_va; do step repro_vmm_$v 90 $P vmm $v; done
cat gpurun_out/$OUT/repro_*.log | grep '^{' > gpurun_out/$OUT/repro.jsonl || true
exit $STATUS
