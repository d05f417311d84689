#!/bin/bash
# Build the current sources into build/live/$1/libfognet_hip.so (A/B timing with
# FOGNET_LIB=... python tools/stage_timing.py); the product library is untouched.
set -e
cd "$(dirname "$0")/.."
d=build/live/$1; mkdir -p $d
S=${SRC:-fognetsimpp_amd/csrc}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result $EXTRA -Iinclude -I$S -shared -o $d/libfognet_hip.so \
  $S/capi.hip $S/replay.hip $S/replay_wide.hip $S/replay_v2.hip $S/replay_region.hip $S/decide.hip $S/tracegen.hip $S/user_stats.hip $S/io.cpp 2>/dev/null
echo built $d
