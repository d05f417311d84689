#!/bin/bash
# Whole-job parity evidence: the bench's CPU-baseline leg over every replication
# of C3 (4096) and C5 (1024, both policies), and 16,384 of C4's first shard
# (statistics records): "parity" in each line compares the oracle with the device.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fullparity; mkdir -p $O
run() {  # name, args
  timeout -k 10 500 python bench.py $2 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  grep '^{' $O/$1.log | tail -n 1 > $O/$1.json
  python3 -c "
import json; d=json.load(open('$O/$1.json')); c=d['cpu_baseline']
print('$1', 'parity', c['parity'], c['parity_sample'][-40:], 'cpu %.3e' % c['value'], 'gpu %.3e' % d['value'])"
}
run c3_all "--steps 3 --warmup 1 --cpu-reps 4096"
run c5_flat_all "--workload c5 --policy REF_V3 --steps 3 --warmup 1 --cpu-reps 1024"
run c5_hier_all "--workload c5 --policy EXT_HIER --steps 3 --warmup 1 --cpu-reps 1024"
run c4_16k "--workload c4 --steps 1 --warmup 1 --cpu-reps 16384"
