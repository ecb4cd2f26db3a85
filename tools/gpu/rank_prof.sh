#!/bin/bash
# torchrun --no-python target: rank 0 runs bench.py under rocprofv3 with $PROF0, other ranks
# plainly (exec happens here, before anything touches the GPU).
if [ "$LOCAL_RANK" = "0" ] && [ -n "$PROF0" ]; then
  exec rocprofv3 $PROF0 -- python3 bench.py "$@"
fi
exec python3 bench.py "$@"
