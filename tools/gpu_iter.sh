#!/bin/bash
# Kernel iteration on the GPU box: the replay parity subset, then a short C3 bench.
# Stops at the first crash/timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-replay or c1 or c2 or node_counts or sweep or tie or ring or fused or ext_lat or energy or full_size}" \
  > gpurun_out/pytest_iter.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps ${BENCH_STEPS:-5} --warmup 1 --no-cpu > gpurun_out/bench_iter.log 2>&1; rc=$?
echo "bench rc=$rc"
python3 -c "import json; d=json.loads(open('gpurun_out/bench_iter.log').read().strip().splitlines()[-1]); print('value %.4g ms/step %.3f kernel %.3f ms frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac']))"
exit $rc
