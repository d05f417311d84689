#!/bin/bash
# Round-end evidence, part PART (1: tests, smoke, C3 bench line + the kernel trace of that same
# command; 2: PMC passes C3, C5 EXT_HIER, C5 REF_V3; 3: C5 lines (EXT_HIER light, REF_V3,
# EXT_HIER saturating) + their kernel traces; 4: C4 and C1 lines; 5: C4 and C1 kernel traces).  Outputs under
# gpurun_out/final/.  Kernel statistics: tools/kstats.py over the kernel trace without the
# warm-up dispatches (the timed steps only); tools/kprof_sidecar.py turns each into the
# profiles/kernel_profile_<workload>.json that bench.py quotes (kernel_avg_ms_rocprof), refusing
# a profile whose average launch exceeds that run's own ms_per_step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
# kt <name> <kernel> <warmup> <bench args...>: the bench line under rocprofv3 --kernel-trace
kt() {
  local name=$1 kern=$2 w=$3; shift 3
  step kt_$name
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o kt -- python3 bench.py "$@" > $O/kt_$name.log 2>&1 || { tail $O/kt_$name.log; return 1; }
  grep '^{' $O/kt_$name.log | tail -n 1 > $O/kt_$name.json
  python3 tools/kstats.py $O/kt_$name --skip $w --out $O/kstats_$name.csv || return 1
  python3 tools/kprof_sidecar.py $O/kt_$name.json $O/kstats_$name.csv --kernel $kern --out $O/kernel_profile_$name.json \
    --cmd "rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -o kt -- python3 bench.py $*; tools/kstats.py --skip $w"
}
case "${PART:-1}" in
1)
  step pytest
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -n 2 $O/pytest_gpu.log
  step smoke
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -n 1 $O/smoke.log
  step bench_c3
  timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
  grep '^{' $O/bench_c3.log | tail -n 1 > $O/bench_c3.json
  kt c3 replay_kernel 2 || exit 1  # the driver's command: bench.py with its defaults (10 steps, 2 warm-up)
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
  kt c5 replay_region_kernel 2 --workload c5 || exit 1
  kt c5_REF_V3 replay_wide_kernel 2 --workload c5 --policy REF_V3 || exit 1
  kt c5_saturate replay_wide_kernel 1 --workload c5 --c5-recipe saturate --steps 3 --warmup 1 --no-cpu || exit 1
  ;;
4)
  step bench_c4
  timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 > $O/bench_c4.log 2>&1 || { tail $O/bench_c4.log; exit 1; }
  grep '^{' $O/bench_c4.log | tail -n 1 > $O/bench_c4.json
  step bench_c1
  timeout -k 10 400 python bench.py --workload c1 --steps 2 --warmup 1 > $O/bench_c1.log 2>&1 || { tail $O/bench_c1.log; exit 1; }
  grep '^{' $O/bench_c1.log | tail -n 1 > $O/bench_c1.json
  ;;
5)
  kt c4 replay_gen_kernel 1 --workload c4 --steps 3 --warmup 1 --no-cpu || exit 1
  kt c1 replay_v2_rows_kernel 1 --workload c1 --steps 2 --warmup 1 --no-cpu || exit 1
  ;;
esac
step done
