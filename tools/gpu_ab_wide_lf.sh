#!/bin/bash
# Wide kernel: group view loads issued before the advert's view stores (build/live/lf; lf2 = in-tree: the uncached record too)
# against build/live/base -- wide/C5/hier GPU tests, then C5 flat REF_V3 (R = 1024, 128), the
# saturated EXT_HIER bench and C5 EXT_HIER.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/widelf; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "wide or c5 or hier or down or head_next or saturated or service_times or capacity" --timeout 300 --timeout-method thread > $O/pytest_wide.log 2>&1 || { tail -40 $O/pytest_wide.log; exit 1; }
tail -n 2 $O/pytest_wide.log
for rep in 1 2; do
for v in ${VARS:-base lf lf2}; do
  for R in 1024 128; do
    WORKLOAD=c5 POLICY=REF_V3 FOGNET_STAGES=all FOGNET_LIB=build/live/$v/libfognet_hip.so timeout -k 10 300 python tools/stage_timing.py $R > $O/s_$v.log 2>&1 || { tail $O/s_$v.log; exit 1; }
    echo "R=$R $(cat $O/s_$v.log | grep -v amdgpu.ids)"
  done
  FOGNET_LIB=build/live/$v/libfognet_hip.so timeout -k 10 300 python tools/bench_var.py --workload c5 --c5-recipe saturate --steps 3 --warmup 1 --no-cpu > $O/b_$v.log 2>&1 || { tail $O/b_$v.log; exit 1; }
  echo "$v saturate $(grep '^{' $O/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2))')"
done
done
