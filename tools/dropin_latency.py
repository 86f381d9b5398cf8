"""Wall time per closed-loop step of the drop-in modules as the reference's main_branch.py drives
them (BranchMPC_CVaR + Highway_env.step, one ego and one obstacle vehicle), with the solver's own
share: the reference's usage on the GPU path.
    python tools/dropin_latency.py [N] [NB] [steps]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "belief-planning_amd"), REPO]

import Highway_env_branch  # noqa: E402
import Init_MPC  # noqa: E402
import MPC_branch  # noqa: E402
from highway_branch_dyn import PredictiveModel, backup_brake, backup_lc, backup_maintain  # noqa: E402
from utils import Branch_constants  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
NB = int(sys.argv[2]) if len(sys.argv) > 2 else 2
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
n, d, am, rm, dt, N_lane = 4, 2, 6.0, 0.3, 0.1, 4
xRef = np.array([0.5, 1.8, 15, 0])
cons = Branch_constants(s1=2, s2=3, c2=0.5, tran_diag=0.3, alpha=1, R=1.2, am=am, rm=rm, J_c=20, s_c=1,
                        ylb=0., yub=7.2, L=4, W=2.5, col_alpha=5, Kpsi=0.1)
backupcons = [lambda x: backup_maintain(x, cons), lambda x: backup_brake(x, cons), lambda x: backup_lc(x, xRef)]
model = PredictiveModel(n, d, N, backupcons, dt, cons)
mpcParam = Init_MPC.initBranchMPC(n, d, N, NB, xRef, am, rm, N_lane, cons.W)
mpc = MPC_branch.BranchMPC_CVaR(mpcParam, model, ralpha=0.9)
env = Highway_env_branch.Highway_env(NV=2, mpc=mpc, N_lane=N_lane)
solve = mpc.solve
acc = [0.0]


def timed_solve(*a, **k):
    t0 = time.perf_counter()
    r = solve(*a, **k)
    acc[0] += time.perf_counter() - t0
    return r


mpc.solve = timed_solve
for t in range(3):
    env.step(t)
acc[0] = 0.0
t0 = time.perf_counter()
for t in range(3, 3 + steps):
    env.step(t)
wall = (time.perf_counter() - t0) / steps
print(f"drop-in main_branch scene N={N} NB={NB}: {1e3 * wall:.2f} ms per env.step, of which BranchMPC_CVaR.solve "
      f"{1e3 * acc[0] / steps:.2f} ms ({steps} steps after 3 warm-up steps)", flush=True)
