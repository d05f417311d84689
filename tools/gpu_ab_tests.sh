#!/bin/bash
# A/B of variant builds (VARIANTS, default "base new") at C3, then the GPU suite on the product library
# (C4=1: also a short C4 bench line).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGES=replay,all bash tools/ab.sh ${VARIANTS:-base new} > gpurun_out/ab.log 2>&1 || { tail gpurun_out/ab.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
if [ "${C4:-0}" = 1 ]; then
  timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_c4_ab.log 2>&1 || { tail gpurun_out/bench_c4_ab.log; exit 1; }
  grep '^{' gpurun_out/bench_c4_ab.log | tail -n 1 | cut -c1-330
fi
