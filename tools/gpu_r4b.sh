#!/bin/bash
# GPU suite, then A/B of variant builds (VARIANTS under build/ab/) on C5 (flat REF_V3, EXT_HIER by
# region, EXT_HIER sequential via FOGNET_HIER_REGIONS=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4b; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -n 2 $O/pytest_gpu.log
fi
for rep in 1 2; do
  for v in ${VARIANTS:-wold wnew}; do
    for cfg in "REF_V3 1" "EXT_HIER 1" "EXT_HIER 0"; do
      set -- $cfg
      FOGNET_HIER_REGIONS=$2 FOGNET_LIB=build/ab/$v/libfognet_hip.so timeout -k 10 300 python tools/bench_var.py --workload c5 --policy $1 --steps 5 --warmup 1 --no-cpu > $O/ab_$v.log 2>&1 || { tail $O/ab_$v.log; exit 1; }
      echo "$v $1 regions=$2 $(grep '^{' $O/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["failed_replications"])')"
    done
  done
done
step done
