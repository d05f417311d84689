#!/bin/bash
# Kernel-trace profile of the default bench (C3, R=4096 x T=100k x N=256).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof/bench_prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -3 gpurun_out/prof/bench_prof.log
find gpurun_out/prof -name '*stats*' | head
exit $rc
