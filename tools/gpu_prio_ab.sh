#!/bin/bash
# Issue-priority A/B at C3 (GPU box): replay parity subset on the product
# library, then replay+statistics kernel time of the variant builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "replay or c2 or sweep or tie or ring or fused or full_size" > gpurun_out/pytest_prio.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_prio.log
[ $rc -ne 0 ] && exit $rc
STAGES=${STAGES:-all} timeout -k 10 400 tools/ab.sh "$@" 2>&1 | tee gpurun_out/prio_ab.log
