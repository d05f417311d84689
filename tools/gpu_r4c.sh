#!/bin/bash
# A/B of region-kernel variants (build/ab/*) on C5 EXT_HIER at R_total 1024 and 128, + the C3 loop counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4c; mkdir -p $O
step() { echo "== $1 $(date +%T)"; }
for rep in 1 2; do
  for v in ${VARIANTS:-wnew rg16}; do
    for RT in 1024 128; do
      FOGNET_LIB=build/ab/$v/libfognet_hip.so timeout -k 10 300 python tools/bench_var.py --workload c5 --policy EXT_HIER --R-total $RT --steps 5 --warmup 1 --no-cpu > $O/ab_$v.log 2>&1 || { tail $O/ab_$v.log; exit 1; }
      echo "$v EXT_HIER R=$RT $(grep '^{' $O/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), d["failed_replications"])')"
    done
  done
done
step prof_count
timeout -k 10 300 python tools/replay_counters.py --mode count --R 1024 --out $O/c3_count_R1024.json > /dev/null 2> $O/prof_count.err || { tail $O/prof_count.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c3_count_R1024.json')); print(json.dumps(d['all']))"
step done
