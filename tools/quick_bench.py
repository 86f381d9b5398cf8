"""Quick GPU timing of one batched solve (development helper).
    python tools/quick_bench.py [B] [N] [NB]     (QB_TRANSFORM=1: a BMPC_PLAN_TRANSFORM plan)"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), REPO, os.path.join(REPO, "belief-planning_amd")]
from common import highway_desc, highway_policy_rows, seeded_batch  # noqa: E402
from bmpc import plan  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
NB = int(sys.argv[3]) if len(sys.argv) > 3 else 1
x, z, xref, tgt = seeded_batch(B, 0)
desc = highway_desc(N, NB)
if os.environ.get("QB_TRANSFORM"):   # the drop-in BranchMPC_CVaR's plan (per-ego S / Fx / bx path)
    from bmpc import abi
    desc.flags |= abi.PLAN_TRANSFORM
pl = plan.BatchPlan(desc, B)
pl.set_policies(highway_policy_rows(tgt))
pl.enable_timing(True)
for step in range(4):
    t0 = time.time()
    r = pl.solve(x, z, xref)
    t1 = time.time()
    tm = pl.timing()
    print(f"step {step}: wall {1e3 * (t1 - t0):.1f} ms  tree {tm['tree_ms']:.2f} ms  ipm {tm['ipm_ms']:.2f} ms  "
          f"status {np.unique(r['status'], return_counts=True)}  iters {r['iters'].mean():.1f}  "
          f"solves/s {B / (t1 - t0):.0f}", flush=True)
    its = r["iters"]
    print("   iters percentiles 50/90/99/max:", np.percentile(its, [50, 90, 99]), its.max(),
          " histogram >=30:", int((its >= 30).sum()), ">=50:", int((its >= 50).sum()), "==100:", int((its >= 100).sum()))
    u0 = r["upred"][:, 0]
    x = x + 0.1 * np.stack([x[:, 2] * np.cos(x[:, 3]), x[:, 2] * np.sin(x[:, 3]), u0[:, 0], u0[:, 1]], 1)
    z = z + 0.1 * np.stack([z[:, 2], 0 * z[:, 0], 0 * z[:, 0], 0 * z[:, 0]], 1)
