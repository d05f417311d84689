#!/bin/bash
# C4 block-size sweep (generated replay): ms per step for each --block.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in ${BLOCKS:-0 131072 262144}; do
  timeout -k 10 200 python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu --block $b > gpurun_out/c4_b$b.log 2>&1 || exit 1
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/c4_b$b.log') if x.startswith('{')][-1]; d=json.loads(l)
print('block $b', round(d['ms_per_step'],1), 'ms/step', '%.3e' % d['value'])"
done
