#!/bin/bash
# Wide-kernel iteration: its parity tests, then C5 kernel time (base variant vs current).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-wide or down or c5 or user or qtime or ring or service or stats_only or smoke or full_size}" > gpurun_out/pytest_wide.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_wide.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in ${VARIANTS:-base}; do
  WORKLOAD=c5 FOGNET_LIB=build/var/$v/libfognet_hip.so FOGNET_STAGES=all,all timeout -k 10 120 python tools/stage_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
WORKLOAD=c5 FOGNET_STAGES=all,all timeout -k 10 120 python tools/stage_timing.py 2>&1 | grep -v amdgpu.ids
