#!/bin/bash
# C1 step time for v2 rows-kernel variants: "lib:row" pairs in CASES (lib under build/ab/, row = FOGNET_V2_ROW).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abc1; mkdir -p $O
for c in ${CASES:-v2lb1:16 v2lb1:64}; do
  v=${c%%:*}; row=${c##*:}
  FOGNET_V2_ROW=$row FOGNET_LIB=build/ab/$v/libfognet_hip.so timeout -k 10 300 python3 tools/bench_var.py --workload c1 --steps 2 --warmup 1 --no-cpu > $O/$v-$row.log 2>&1 || { tail $O/$v-$row.log; exit 1; }
  echo "$v row=$row $(grep '^{' $O/$v-$row.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["failed_replications"], d["stats"])')"
done
