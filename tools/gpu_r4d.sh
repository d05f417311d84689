#!/bin/bash
# GPU suite on the in-tree library, C5 lines (both policies, no CPU leg) and the C4 + C1 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4d; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
for pol in EXT_HIER REF_V3; do
  timeout -k 10 300 python bench.py --workload c5 --policy $pol --steps 10 --warmup 2 --no-cpu > $O/c5_$pol.log 2>&1 || { tail $O/c5_$pol.log; exit 1; }
  echo "c5 $pol $(grep '^{' $O/c5_$pol.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["failed_replications"])')"
done
PART=4 bash tools/gpu_final.sh
