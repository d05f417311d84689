#!/bin/bash
# One evidence pass: the whole GPU suite, smoke, the C3 bench line, C5 lines
# (both policies, short) — each step under its own time limit, stopping at the
# first crash or timeout.  Outputs under gpurun_out/round/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/round; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -n 3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
if [ "${SKIP_C3:-0}" != 1 ]; then
step bench_c3
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log | tail -n 1 > $O/bench_c3.json
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['kernel_avg_ms'],2), 'kernel ms', '%.3e' % d['value'], 'parity', d['cpu_baseline'].get('parity'))"
fi
for pol in EXT_HIER REF_V3; do
  step bench_c5_$pol
  timeout -k 10 300 python bench.py --workload c5 --policy $pol --steps 5 --warmup 1 ${C5_ARGS:---no-cpu} > $O/bench_c5_$pol.log 2>&1 || { tail $O/bench_c5_$pol.log; exit 1; }
  grep '^{' $O/bench_c5_$pol.log | tail -n 1 > $O/bench_c5_$pol.json
  python3 -c "import json; d=json.load(open('$O/bench_c5_$pol.json')); print('c5 $pol', round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['kernel_avg_ms'],2), 'kernel ms', '%.3e' % d['value'])"
done
step done
exit $rc
