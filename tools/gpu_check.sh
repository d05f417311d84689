#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first crash/timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "start $(date +%T)"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc $(date +%T)"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc $(date +%T)"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --cpu-reps ${CPU_REPS:-1024} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc $(date +%T)"; tail -3 gpurun_out/bench.log
exit $rc
