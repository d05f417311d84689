#!/bin/bash
# Round-4 probe: GPU suite, the C3 line, C3 at R = 1024/2048/4096 (1, 2, 4 waves
# per SIMD: flat time = latency-bound, proportional = issue-bound), and C5 at
# one 8-GPU shard (R_total 128) beside the full 1024-replication step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/probe; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -n 2 $O/pytest_gpu.log
fi
for R in ${RS:-1024 2048 4096}; do
  step c3_R$R
  timeout -k 10 300 python bench.py --R $R --steps 10 --warmup 2 --no-cpu > $O/c3_R$R.log 2>&1 || { tail $O/c3_R$R.log; exit 1; }
  grep '^{' $O/c3_R$R.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["R_per_gpu"], round(d["ms_per_step"],3), round(d["roofline"]["kernel_avg_ms"],3), "%.3e"%d["value_ref_defined"])'
done
for pol in ${C5POL:-REF_V3 EXT_HIER}; do
  for RT in 128 1024; do
    step c5_${pol}_$RT
    timeout -k 10 300 python bench.py --workload c5 --policy $pol --R-total $RT --steps 5 --warmup 1 --no-cpu > $O/c5_${pol}_$RT.log 2>&1 || { tail $O/c5_${pol}_$RT.log; exit 1; }
    grep '^{' $O/c5_${pol}_$RT.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["R_total"], round(d["ms_per_step"],3), d["failed_replications"])'
  done
done
step done
if [ "${HN:-1}" = 1 ]; then
  # round-3 hd_next experiment: the first code shape (A) against the hoisted one (B)
  for v in A B; do
    step hn_$v
    FOGNET_LIB=build/hn/$v/out/libfognet_hip.so timeout -k 10 120 python tools/dbg_hier.py > $O/hn_$v.log 2>&1 || { tail $O/hn_$v.log; exit 1; }
    cat $O/hn_$v.log
  done
fi
