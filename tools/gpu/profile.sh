#!/bin/bash
# rocprofv3 kernel trace + stats of one command (the program itself right after `--`, never a
# launcher), optionally followed by PMC passes, each in a run of its own (counter groups within the
# per-block limits).
#   OUT=<dir> CMD="python3 bench.py --steps 5" [PMC="SQ_WAVES GRBM_GUI_ACTIVE;FETCH_SIZE WRITE_SIZE"] bash tools/gpu/profile.sh
source "$(dirname "$0")/steps.sh"
export TMPDIR=/tmp
step trace ${LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/$OUT/trace" -o run -- $CMD
i=0
IFS=';' read -ra PASSES <<< "${PMC:-}"
for pass in "${PASSES[@]}"; do
  i=$((i + 1))
  step pmc$i 120 rocprofv3 --pmc $pass --output-format csv -d "gpurun_out/$OUT/pmc$i" -o run -- $CMD
done
find "gpurun_out/$OUT" -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | head -50 > "gpurun_out/$OUT/files.txt"
exit $STATUS
