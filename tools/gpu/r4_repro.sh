#!/bin/bash
# The two memory-lifetime anomalies as standalone two-process HIP programs (no torch / mp4x):
# every variant of the release ordering, one JSON line per check (tools/repro/ipc_lifetime_repro.hip).
source "$(dirname "$0")/steps.sh"
B=tools/repro/ipc_lifetime_repro
for v in close_before_free close_after_free never_close; do
  step ipc_$v 60 $B ipc $v 8388608
done
for v in importer_first exporter_first keep_fds exporter_keeps importer_keeps concurrent; do
  step vmm_$v 60 $B vmm $v 8388608
done
cat gpurun_out/$OUT/*.log | grep '^{' > gpurun_out/$OUT/all.jsonl
exit $STATUS
