#!/bin/bash
# One GPU call: steps named in STEPS (space-separated), each under its own time limit,
# stopping at the first failure.  Outputs under gpurun_out/$ROUND (default r6).
#   tests:<pytest -k expr>   GPU tests matching the expression
#   suite                    the whole GPU suite
#   bench:<name>:<args>      one bench.py line (args with '+' for spaces) -> <name>.json
#   ab:<variant>:<args>      bench.py on build/live/<variant> (or the tree's library: 'tree'), no CPU leg
#   kt:<name>:<args>         rocprofv3 kernel trace + warm-up-free stats of bench.py (KTLIB=<variant>: a variant build;
#                            KTKERNEL=<kernel>: also the kernel_profile sidecar bench.py quotes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${ROUND:-r6}; mkdir -p $O
export TMPDIR=/tmp
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case "$s" in
    tests:*)
      k="${s#tests:}"; k="${k//+/ }"
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
      tail -n 3 $O/pytest_k.log ;;
    suite)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
      tail -n 2 $O/pytest_gpu.log ;;
    bench:*)
      r="${s#bench:}"; name="${r%%:*}"; a="${r#*:}"; a="${a//+/ }"
      env $BENV timeout -k 10 600 python bench.py $a > $O/bench_$name.log 2>&1 || { tail -20 $O/bench_$name.log; exit 1; }
      grep '^{' $O/bench_$name.log | tail -n 1 > $O/bench_$name.json
      python3 -c "import json; d=json.load(open('$O/bench_$name.json')); print('$name', round(d['ms_per_step'],3), 'ms/step', d['value'], d.get('failed_replications'), d.get('hier_escalation'), d['roofline'].get('kernel_avg_ms'))" ;;
    ab:*)  # ab:<variant under build/live, or "tree">:<bench args>: one bench line of a variant build
      r="${s#ab:}"; v="${r%%:*}"; a="${r#*:}"; a="${a//+/ }"
      lib=build/live/$v/libfognet_hip.so; [ "$v" = tree ] && lib=fognetsimpp_amd/libfognet_hip.so
      FOGNET_LIB=$lib timeout -k 10 600 python tools/bench_var.py $a --no-cpu > $O/ab_$v.log 2>&1 || { tail -20 $O/ab_$v.log; exit 1; }
      echo "ab $v [$a] $(grep '^{' $O/ab_$v.log | tail -n 1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step kernel", d["roofline"].get("kernel_avg_ms", d["roofline"].get("kernel_ms_per_step")), "failed", d["failed_replications"])')" ;;
    prof:*)  # prof:<variant under build/live>:<count|time>:<R>: replay_counters.py on a profile build
      r="${s#prof:}"; v="${r%%:*}"; r="${r#*:}"; m="${r%%:*}"; R="${r#*:}"
      FOGNET_LIB=build/live/$v/libfognet_hip.so timeout -k 10 300 python tools/replay_counters.py --mode $m --R $R --out $O/prof_${v}_${m}_R$R.json > /dev/null 2> $O/prof_$v.err || { tail $O/prof_$v.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/prof_${v}_${m}_R$R.json')); print('$v', json.dumps({k: round(x, 4) for k, x in d['all'].items()}))" ;;
    stage:*)  # stage:<variant or tree>:<R>: replay-only / replay+statistics kernel times (stage_timing.py)
      r="${s#stage:}"; v="${r%%:*}"; R="${r#*:}"
      lib=build/live/$v/libfognet_hip.so; [ "$v" = tree ] && lib=fognetsimpp_amd/libfognet_hip.so
      FOGNET_LIB=$lib FOGNET_STAGES=${STAGES:-all,replay,all,replay} timeout -k 10 300 python tools/stage_timing.py $R 2>&1 | grep -v Warning | sed "s/^/[$v R=$R] /" ;;
    kt:*)  # kt:<name>:<bench args>: rocprofv3 kernel trace + stats of one bench.py run (warm-up dispatches dropped)
      r="${s#kt:}"; name="${r%%:*}"; a="${r#*:}"; a="${a//+/ }"
      if [ -n "$KTLIB" ]; then prog="tools/bench_var.py"; export FOGNET_LIB=build/live/$KTLIB/libfognet_hip.so; else prog=bench.py; fi
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$name -o kt -- python3 $prog $a > $O/kt_$name.log 2>&1 || { tail -20 $O/kt_$name.log; exit 1; }
      unset FOGNET_LIB
      python3 tools/kstats.py $O/kt_$name --skip ${SKIP:-1} --out $O/kstats_$name.csv && python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kstats_$name.csv')))[:6]: print('  ', r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')" || exit 1
      # KTKERNEL=<kernel name>: the bench.py sidecar (kernel_avg_ms_rocprof) of this profiled bench run
      if [ -n "$KTKERNEL" ] && [ -z "$KTLIB" ]; then
        python3 tools/kprof_sidecar.py $O/kt_$name.log $O/kstats_$name.csv --kernel $KTKERNEL --out $O/kernel_profile_$name.json \
          --cmd "rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -o kt -- python3 bench.py $a; tools/kstats.py --skip ${SKIP:-1}" || exit 1
      fi ;;
  esac
done
echo "== done $(date +%T)"
