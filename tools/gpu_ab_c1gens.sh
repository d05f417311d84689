#!/bin/bash
# C1 rows kernel: several timer periods per batch (kBatchGens) -- v2 GPU tests on the in-tree
# library, then bench.py --workload c1 per variant build (build/live/<v>).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c1gens; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "v2" --timeout 300 --timeout-method thread > $O/pytest_v2.log 2>&1 || { tail -40 $O/pytest_v2.log; exit 1; }
tail -n 2 $O/pytest_v2.log
for rep in 1 2; do
for v in ${VARS:-base g1 g3 g5 g8}; do
  FOGNET_LIB=build/live/$v/libfognet_hip.so timeout -k 10 300 python tools/bench_var.py --workload c1 --steps 3 --warmup 1 --no-cpu > $O/b_$v.log 2>&1 || { tail $O/b_$v.log; exit 1; }
  echo "$v $(grep '^{' $O/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2))')"
done
done
