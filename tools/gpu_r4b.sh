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
if [ "${PROF:-1}" = 1 ]; then
  step prof_c3
  timeout -k 10 300 python tools/replay_counters.py --mode time --R 1024 --out $O/c3_time_R1024.json > /dev/null 2> $O/prof_time.err || { tail $O/prof_time.err; exit 1; }
  timeout -k 10 300 python tools/replay_counters.py --mode count --R 1024 --out $O/c3_count_R1024.json > /dev/null 2> $O/prof_count.err || { tail $O/prof_count.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c3_time_R1024.json')); print(json.dumps(d['all'])); print(json.dumps(d['per_rep_total_cycles']))"
  python3 -c "import json; d=json.load(open('$O/c3_count_R1024.json')); print(json.dumps(d['all']))"
fi
