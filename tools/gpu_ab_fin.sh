#!/bin/bash
# rocprof kernel statistics of C5 (POLICY, default EXT_HIER) for variant builds (VARIANTS under build/ab/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/abfin_${POLICY:-EXT_HIER}; mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-f0 f1}; do
  FOGNET_LIB=build/ab/$v/libfognet_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o k -- python3 tools/bench_var.py --workload c5 --policy ${POLICY:-EXT_HIER} --steps 3 --warmup 1 --no-cpu > $O/$v.log 2>&1 || { tail $O/$v.log; exit 1; }
  echo "$v $(grep '^{' $O/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
  python3 tools/kstats.py $O/$v --skip 1 | grep -E "region|wide_kernel" | cut -c1-160
done
