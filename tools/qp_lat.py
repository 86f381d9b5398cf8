"""Single-problem latency of bmpc_qp_solve on the belief-MPC QP (tests/golden/belief_m1.npz
step 0), split into the host wrapper and the C call; run under rocprofv3 for the kernel time.
usage: python tools/qp_lat.py [reps]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "belief-planning_amd"), os.path.join(REPO, "tests")]
from bmpc import plan  # noqa: E402
from common import coo, golden  # noqa: E402

g = golden("belief_m1")
P, q, A, l, u = coo(g, "s0_P"), g["s0_q"], coo(g, "s0_A"), g["s0_l"], g["s0_u"]
plan.context(0)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
r = plan.qp_solve(P, q, A, l, u)
lat, prep = [], []
for _ in range(reps):
    t0 = time.perf_counter()
    plan.qp_arrays(P, q, A, l, u)
    t1 = time.perf_counter()
    r = plan.qp_solve(P, q, A, l, u)
    t2 = time.perf_counter()
    prep.append(t1 - t0)
    lat.append(t2 - t1)
print(json.dumps({"latency_ms_median": 1e3 * float(np.median(lat)), "host_arrays_ms_median": 1e3 * float(np.median(prep)),
                  "iters": int(r["iters"][0]), "status": int(r["status"][0]), "info": [int(v) for v in r["info"]]}))
