#!/bin/bash
# Replay-kernel time vs replications per launch at C3 shape (occupancy probe).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for R in ${RS:-1024 2048 3072 3584 4096 5120 8192}; do
  FOGNET_STAGES=${STAGES:-replay,all} timeout -k 10 120 python tools/stage_timing.py $R 2>&1 | grep -v amdgpu.ids | sed "s/^/R=$R /" || exit 1
done
