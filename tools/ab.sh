#!/bin/bash
# A/B kernel timing of variant builds: tools/ab.sh name1 name2 ... (GPU box)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    FOGNET_LIB=build/var/$v/libfognet_hip.so FOGNET_STAGES=${STAGES:-replay,all} timeout -k 10 120 python tools/stage_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
