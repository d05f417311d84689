#!/bin/bash
# Round-end evidence, part PART (1: tests, smoke, C3 bench + rocprof kernel trace/stats;
# 2: PMC passes C3, C5 EXT_HIER, C5 REF_V3; 3: C5 lines + rocprof; 4: C4 and C1 lines).
# Outputs under gpurun_out/final/.  Kernel statistics: rocprofv3's --stats (every dispatch) and
# tools/kstats.py over the kernel trace without the warm-up dispatch (the timed steps only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
case "${PART:-1}" in
1)
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -n 2 $O/pytest_gpu.log
  step smoke
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -n 1 $O/smoke.log
  step bench_c3
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
  grep '^{' $O/bench_c3.log | tail -n 1 > $O/bench_c3.json
  step rocprof_c3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/prof_c3.log 2>&1 || { tail $O/prof_c3.log; exit 1; }
  python3 tools/kstats.py $O/prof_c3 --skip 1 --out $O/kstats_c3.csv && head -3 $O/kstats_c3.csv
  ;;
2)
  step pmc_c3
  bash tools/gpu_pmc.sh > $O/pmc_c3.log 2>&1 || { tail $O/pmc_c3.log; exit 1; }
  cp gpurun_out/pmc/pmc_traffic.json $O/
  for pol in EXT_HIER REF_V3; do
    step pmc_c5_$pol
    WORKLOAD=c5 POLICY=$pol bash tools/gpu_pmc.sh > $O/pmc_c5_$pol.log 2>&1 || { tail $O/pmc_c5_$pol.log; exit 1; }
    cp gpurun_out/pmc/pmc_traffic_c5*.json $O/
  done
  ;;
3)
  for pol in EXT_HIER REF_V3; do
    step bench_c5_$pol
    timeout -k 10 300 python bench.py --workload c5 --policy $pol --steps 10 --warmup 2 > $O/bench_c5_$pol.log 2>&1 || { tail $O/bench_c5_$pol.log; exit 1; }
    grep '^{' $O/bench_c5_$pol.log | tail -n 1 > $O/bench_c5_$pol.json
    step rocprof_c5_$pol
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$pol -o c5 -- python3 bench.py --workload c5 --policy $pol --steps 3 --warmup 1 --no-cpu > $O/prof_c5_$pol.log 2>&1 || { tail $O/prof_c5_$pol.log; exit 1; }
    python3 tools/kstats.py $O/prof_c5_$pol --skip 1 --out $O/kstats_c5_$pol.csv && head -3 $O/kstats_c5_$pol.csv
  done
  ;;
4)
  step bench_c4
  timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 > $O/bench_c4.log 2>&1 || { tail $O/bench_c4.log; exit 1; }
  grep '^{' $O/bench_c4.log | tail -n 1 > $O/bench_c4.json
  step bench_c1
  timeout -k 10 400 python bench.py --workload c1 --steps 2 --warmup 1 > $O/bench_c1.log 2>&1 || { tail $O/bench_c1.log; exit 1; }
  grep '^{' $O/bench_c1.log | tail -n 1 > $O/bench_c1.json
  ;;
esac
step done
