"""Development helper: one small batched solve (ego 0 prints its IPM iterations in a
-DBMPC_DEV_DEBUG build)."""
import os
import sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd")]
from bmpc import plan  # noqa: E402
from bmpc.scenarios import highway_desc, highway_policy_rows, seeded_batch  # noqa: E402
x, z, xref, tgt = seeded_batch(4, seed=0)
pl = plan.BatchPlan(highway_desc(N=20, NB=1), 4)
pl.set_policies(highway_policy_rows(tgt))
r = pl.solve(x, z, xref)
print("status", r["status"], "iters", r["iters"], "J", r["J"], flush=True)
