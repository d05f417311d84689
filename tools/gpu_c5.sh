#!/bin/bash
# Wide-kernel iteration: its parity tests, then C5 (flat REF_V3 and EXT_HIER) bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${PYTEST_K:-wide or down or hier or c5 or generated or stats_only or ring or user}" > gpurun_out/pytest_c5.log 2>&1 || { tail -30 gpurun_out/pytest_c5.log; exit 1; }
tail -n 2 gpurun_out/pytest_c5.log
for pol in REF_V3 EXT_HIER; do
  timeout -k 10 200 python bench.py --workload c5 --policy $pol --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_$pol.log 2>&1 || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/c5_$pol.log') if x.startswith('{')][-1]; d=json.loads(l)
print('c5 $pol', round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['kernel_avg_ms'],2), 'kernel ms', '%.3e' % d['value'])"
done
