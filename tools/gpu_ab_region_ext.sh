#!/bin/bash
# Region kernel: runs on an idle node past its own busy-0 adverts (ext = in-tree) against
# noext (FOGNET_REGION_EXT_RUNS=0) -- hier/C5/region GPU tests, then the C5 EXT_HIER step
# (bench.py --workload c5, R = 1024) and the R = 128 shard (stage_timing), two passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/regext; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "hier or c5 or region or escalat" --timeout 300 --timeout-method thread > $O/pytest_hier.log 2>&1 || { tail -40 $O/pytest_hier.log; exit 1; }
tail -n 2 $O/pytest_hier.log
for rep in 1 2; do
for v in ${VARS:-noext ext}; do
  FOGNET_LIB=build/live/$v/libfognet_hip.so timeout -k 10 300 python tools/bench_var.py --workload c5 --steps 10 --warmup 2 --no-cpu > $O/b_$v.log 2>&1 || { tail $O/b_$v.log; exit 1; }
  echo "$v c5 EXT_HIER R=1024 $(grep '^{' $O/b_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))') ms/step"
  WORKLOAD=c5 POLICY=EXT_HIER FOGNET_STAGES=all FOGNET_LIB=build/live/$v/libfognet_hip.so timeout -k 10 300 python tools/stage_timing.py 128 > $O/s_$v.log 2>&1 || { tail $O/s_$v.log; exit 1; }
  echo "  R=128 $(grep -v amdgpu.ids $O/s_$v.log)"
done
done
