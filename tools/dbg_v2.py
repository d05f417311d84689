"""Print GPU vs oracle outputs of the v2 replay on the hand-traced cases (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import golden_io  # noqa: E402
import oracle_lib as ol  # noqa: E402

import fognetsimpp_amd as fa  # noqa: E402
from test_parity_gpu import run_v2_gpu  # noqa: E402

ctx = fa.Context(0)
for name, tr, e in golden_io.replay_v2_cases():
    g = run_v2_gpu(ctx, tr, tr["broker_mips"], tr["stop"])
    o = ol.run_v2(tr["arrive"], tr["req"], tr["broker_mips"], tr["mips"], tr["dl"], tr["ul"], tr["first_adv"],
                  tr["stop"])
    print(name)
    for k in ("node", "status", "start", "done"):
        print("  ", k, g[k][0].tolist(), o[k][0].tolist())
    print("   gpu", g["stats"][0])
    print("   orc", o["stats"][0])
