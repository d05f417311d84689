#!/bin/bash
# A/B of variant builds (VARIANTS) on the C5 workload (both policies), then the wide parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VARIANTS:-base new}; do
    for pol in EXT_HIER REF_V3; do
      FOGNET_LIB=build/ab/$v/libfognet_hip.so timeout -k 10 300 python tools/bench_var.py --workload c5 --policy $pol --steps 5 --warmup 1 --no-cpu > gpurun_out/ab_c5_$v.log 2>&1 || { tail gpurun_out/ab_c5_$v.log; exit 1; }
      echo "$v $pol $(grep '^{' gpurun_out/ab_c5_$v.log | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],2))')"
    done
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1 || { tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
