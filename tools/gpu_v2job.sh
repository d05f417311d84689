#!/bin/bash
# v2 replay iteration: its parity tests, then one C1 bench line (no CPU leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "v2" > gpurun_out/pytest_v2.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_v2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c1 --steps 2 --warmup 1 --no-cpu > gpurun_out/c1.log 2>&1 || exit 1
grep "^{" gpurun_out/c1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c1', d['ms_per_step'], d['value'])"
