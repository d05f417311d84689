#!/bin/bash
# Inputs of the C3 latency-floor model: the one-wave instruction-class latencies
# (build/live/lat_probe, tools/lat_probe.hip) and the replay-only instruction mix at one wave per SIMD
# (R = 1024, FOGNET_STAGES=replay: no statistics pass) from two rocprofv3 PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lat; rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 build/live/lat_probe > $O/lat_probe.json || exit 1
cat $O/lat_probe.json
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  FOGNET_STAGES=replay timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p$i -- \
    python3 tools/stage_timing.py ${R:-1024} > $O/p$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/p$i.log; exit 1; }
done
python3 - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import load
d = load("gpurun_out/lat", "replay_kernel")
per = {k: v / n for k, (v, n) in d.items()}
R = 1024
dec = R * 100000.0
out = {"config": {"R": R, "T": 100000, "N": 256, "stage": "replay only"}, "per_dispatch": per}
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM"):
    out[k + "_per_decision"] = per[k] / dec
wc = per["SQ_WAVE_CYCLES"]
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
    out[k + "_frac"] = per[k] / wc
out["wave_cycles_per_decision"] = 4 * wc / per["SQ_WAVES"] / 100000.0  # SQ_WAVE_CYCLES counts quad-cycles
json.dump(out, open("gpurun_out/lat/replay_mix_R1024.json", "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "per_dispatch"}, indent=1))
PY
