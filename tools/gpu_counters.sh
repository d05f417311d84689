#!/bin/bash
# Loop counters and per-segment cycle split of replay_kernel (profile builds, `make prof`).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/replay_counters.py --mode count --out gpurun_out/replay_counters.json > gpurun_out/counters.log 2>&1 || exit $?
timeout -k 10 120 python3 tools/replay_counters.py --mode time --out gpurun_out/replay_segments.json >> gpurun_out/counters.log 2>&1
