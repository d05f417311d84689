#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, no tracing domains mixed in)
# over one timed step of the bench workload: C3 (default) or WORKLOAD=c5.
# Plus the FETCH_SIZE calibration: the standalone statistics pass
# (rep_stats_kernel) streams a known byte count (29 B per task of the C3
# outputs + trace) with the element widths the replay's own loads use.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmc; mkdir -p gpurun_out/pmc
if [ "${WORKLOAD:-c3}" = c5 ]; then
  # POLICY=REF_V3: the flat broker (pmc_traffic_c5_REF_V3.json); default EXT_HIER (pmc_traffic_c5.json)
  BARGS="--workload c5 --policy ${POLICY:-EXT_HIER}"; DEC=10240000; CFG=1024,10000,10000
  KERNEL=$([ "${POLICY:-EXT_HIER}" = EXT_HIER ] && echo "replay_region_kernel<1>" || echo replay_wide_kernel)
  OUT=pmc_traffic_c5$([ "${POLICY:-EXT_HIER}" = EXT_HIER ] || echo _${POLICY}).json
else
  BARGS=""; KERNEL=replay_kernel; DEC=409600000; OUT=pmc_traffic.json; CFG=4096,100000,256
fi
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/p$i -o p$i -- \
    python3 bench.py $BARGS --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc/p$i.log 2>&1; rc=$?
  echo "pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $KERNEL $DEC gpurun_out/pmc/$OUT 2048 $CFG ${POLICY:-$([ "${WORKLOAD:-c3}" = c5 ] && echo EXT_HIER || echo REF_V3)} > /dev/null || exit 1
if [ "${WORKLOAD:-c3}" = c3 ]; then
  for grp in "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    FOGNET_STAGES=replay,stats timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/c$i -o c$i -- \
      python3 tools/stage_timing.py > gpurun_out/pmc/c$i.log 2>&1; rc=$?
    echo "calibration pass $i ($grp) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/c$i.log; exit $rc; fi
  done
  python3 tools/pmc_calibrate.py gpurun_out/pmc gpurun_out/pmc/$OUT || exit 1
fi
