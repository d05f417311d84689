#!/bin/bash
# A/B of variant builds (VARIANTS under build/ab/) on C3 (R = 4096 and 1024), then the GPU suite on
# the in-tree library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abc3; mkdir -p $O
for rep in 1 2; do
  for v in ${VARIANTS:-c3base hz1 hz2}; do
    for R in ${RS:-4096 1024}; do
      FOGNET_LIB=build/ab/$v/libfognet_hip.so timeout -k 10 300 python tools/bench_var.py --R $R --steps 10 --warmup 2 --no-cpu > $O/ab_$v.log 2>&1 || { tail $O/ab_$v.log; exit 1; }
      echo "$v R=$R $(grep '^{' $O/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), round(d["roofline"]["kernel_avg_ms"],3), d["failed_replications"])')"
    done
  done
done
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -n 2 $O/pytest_gpu.log
fi
