#!/bin/bash
# C1 (v2 model) counters: one PMC pass over one step of `bench.py --workload c1`
# (4096 replications x 19,999 publishes), summarised into gpurun_out/pmc_c1/pmc_c1.json
# (VALU busy, instructions per FES event and per decision).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rm -rf gpurun_out/pmc_c1; mkdir -p gpurun_out/pmc_c1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_c1/p1 -o p1 -- \
  python3 bench.py --workload c1 --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc_c1/p1.log 2>&1 || exit 1
python3 - <<'PY'
import json, os, sys
sys.path.insert(0, "tools")
import pmc_summary
d = pmc_summary.load("gpurun_out/pmc_c1", kernel=os.environ.get("KERNEL", "replay_v2_rows_kernel"))
per = {k: v / n for k, (v, n) in d.items()}
line = [l for l in open("gpurun_out/pmc_c1/p1.log") if l.startswith("{")][-1]
b = json.loads(line)
dec, ev = b["stats"]["decisions"], b["stats"]["events"]
out = {"kernel": os.environ.get("KERNEL", "replay_v2_rows_kernel"), "per_dispatch": per,
       "valu_busy": per["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (per["GRBM_GUI_ACTIVE"] / 8),
       "SQ_INSTS_VALU_per_event": per["SQ_INSTS_VALU"] / ev, "SQ_INSTS_SALU_per_event": per["SQ_INSTS_SALU"] / ev,
       "SQ_INSTS_VALU_per_decision": per["SQ_INSTS_VALU"] / dec,
       "SQ_WAIT_INST_ANY_frac_of_wave_cycles": per["SQ_WAIT_INST_ANY"] / per["SQ_WAVE_CYCLES"],
       "events": ev, "decisions": dec, "dispatches": d["SQ_INSTS_VALU"][1],
       "config": {"R_total": 4096, "workload": "c1"},
       "note": "valu_busy = SQ_ACTIVE_INST_VALU*4/1024 SIMDs/(GRBM_GUI_ACTIVE/8 XCDs)"}
json.dump(out, open("gpurun_out/pmc_c1/pmc_c1.json", "w"), indent=1)
print(json.dumps({k: out[k] for k in ("valu_busy", "SQ_INSTS_VALU_per_event", "SQ_INSTS_SALU_per_event", "SQ_WAIT_INST_ANY_frac_of_wave_cycles")}))
PY
