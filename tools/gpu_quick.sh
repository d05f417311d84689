#!/bin/bash
# Quick evidence pass: one GPU test file subset, C3 and C4 bench lines (gpurun_out/quick/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/quick; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTS:-compact_ring or ring_capacity or service_past}" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-reps 256 > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log | tail -n 1 | cut -c1-400
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > $O/bench_c4.log 2>&1 || { tail $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log | tail -n 1 | cut -c1-400
