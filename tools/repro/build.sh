#!/bin/bash
# Build the lifetime reproducer twice: ipc_lifetime_repro runs on the HIP runtime PyTorch ships
# (torch/lib — the runtime instance every mp4x rank runs on; launcher.cpp loads it, then the
# reproducer library), ipc_lifetime_repro_sys is a plain hipcc executable on /opt/rocm's runtime.
set -e
cd "$(dirname "$0")"
TL=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
hipcc --offload-arch=gfx950 -O2 -fPIC -DREPRO_AS_LIBRARY -c ipc_lifetime_repro.hip -o ipc_lifetime_repro.o
g++ -shared ipc_lifetime_repro.o -o libipc_lifetime_repro.so -L "$TL" -l:libamdhip64.so
g++ -O2 launcher.cpp -o ipc_lifetime_repro -DHIP_RUNTIME_PATH="\"$TL/libamdhip64.so\"" -ldl
hipcc --offload-arch=gfx950 -O2 ipc_lifetime_repro.hip -o ipc_lifetime_repro_sys
rm -f ipc_lifetime_repro.o
