"""ctypes mirror of ``include/bmpc.h`` (the C ABI of libbmpc.so)."""
from __future__ import annotations

import ctypes as C

import numpy as np

MAX_N, MAX_D, MAX_FX, MAX_FU, MAX_M = 8, 4, 8, 8, 4

CTRL_CVAR, CTRL_PROX, CTRL_QP, CTRL_ROBUST = 0, 1, 2, 3
MODEL_HIGHWAY, MODEL_QUADRUPED, MODEL_HIGHWAY_MERGE = 0, 1, 2
PLAN_TRANSFORM = 1      # bmpc_plan_desc.flags: solve's S / Fx / bx on a HIGHWAY CVaR plan
POL_MAINTAIN, POL_BRAKE, POL_LC, POL_MAINTAIN_TRACKV, POL_FORWARD, POL_STOP = range(6)
# the merge ramp's lane-reference (psiref) tracking backups (include/bmpc.h)
POL_MAINTAIN_PSIREF, POL_MAINTAIN_TRACKV_PSIREF, POL_BRAKE_PSIREF = 6, 7, 8
MAX_LANE_REF = 4096

(INFO_T, INFO_U, INFO_BDIM, INFO_NBRANCH, INFO_NV, INFO_NEQ, INFO_NROWS, INFO_NCONES,
 INFO_LP, INFO_BATCH, INFO_WS_DOUBLES, INFO_SOLVER, INFO_COUNT) = range(13)
# solver kernels reported in INFO_SOLVER (include/bmpc.h BMPC_KERNEL_*)
(KERNEL_NONE, KERNEL_IPM_RICH, KERNEL_IPM_LEAN, KERNEL_IPM_BLK4, KERNEL_IPM_BLK8, KERNEL_QP_RICH,
 KERNEL_QP_LEAN, KERNEL_LOOP_RICH, KERNEL_LOOP_LEAN) = range(9)


class Policy(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("p", C.c_double * 4)]


class PlanDesc(C.Structure):
    _fields_ = [
        ("controller", C.c_int32), ("model", C.c_int32),
        ("n", C.c_int32), ("d", C.c_int32),
        ("N", C.c_int32), ("NB", C.c_int32), ("m", C.c_int32),
        ("nFx", C.c_int32), ("nFu", C.c_int32),
        ("maxit", C.c_int32),
        ("dt", C.c_double), ("ralpha", C.c_double),
        ("Q", C.c_double * (MAX_N * MAX_N)),
        ("R", C.c_double * (MAX_D * MAX_D)),
        ("Qf", C.c_double * (MAX_N * MAX_N)),
        ("dR", C.c_double * MAX_D),
        ("Fx", C.c_double * (MAX_FX * MAX_N)),
        ("bx", C.c_double * MAX_FX),
        ("Fu", C.c_double * (MAX_FU * MAX_D)),
        ("bu", C.c_double * MAX_FU),
        ("Qslack", C.c_double * 2),
        ("mc", C.c_double * 8),
        ("feastol", C.c_double), ("abstol", C.c_double), ("reltol", C.c_double),
        ("flags", C.c_int32), ("reserved_flags", C.c_int32),
    ]


ENV_STRIDE, ENV_NSTAT = 16, 8
# scene state / statistics slots (bmpc_env.h)
ENV_X, ENV_Z, ENV_UOBS, ENV_LANE0, ENV_LANE1, ENV_COLL, ENV_OBSPOL, ENV_STEPS = 0, 4, 8, 10, 11, 12, 13, 14
ENVS_J, ENVS_J2, ENVS_INFEAS, ENVS_ITERS, ENVS_SOLVES, ENVS_COLL_STEPS, ENVS_COLLIDED = range(7)


class EnvDesc(C.Structure):
    """bmpc_env_desc: the sim_overtake scene (Highway_env_branch.py:46-72)."""
    _fields_ = [("n_lane", C.c_int32), ("reserved", C.c_int32), ("L", C.c_double), ("W", C.c_double),
                ("Kpsi", C.c_double), ("v0", C.c_double), ("vlen", C.c_double), ("vwid", C.c_double),
                ("target", C.c_double * 4)]


def make_env(n_lane=4, L=4.0, W=2.5, Kpsi=0.1, v0=20.0, target=(0.5, 1.8, 15.0, 0.0), vlen=4.0, vwid=2.4):
    """Scene constants of main_branch.sim_overtake: Branch_constants (main_branch.py:37), the
    construction-time lane-change target xRef (:39), vehicle() size (Highway_env_branch.py:29)."""
    E = EnvDesc()
    E.n_lane, E.L, E.W, E.Kpsi, E.v0, E.vlen, E.vwid = int(n_lane), L, W, Kpsi, v0, vlen, vwid
    _fill(E.target, target)
    return E


def _fill(arr, values):
    v = np.asarray(values, dtype=np.float64).ravel()
    for i, x in enumerate(v):
        arr[i] = float(x)


def make_desc(controller, model, n, d, N, NB, m, dt, Q, R, Fx, bx, Fu, bu, Qslack,
              mc, ralpha=0.9, Qf=None, dR=None, maxit=100,
              feastol=1e-8, abstol=1e-8, reltol=1e-8, flags=0) -> PlanDesc:
    """Pack a plan description (all matrices row-major at their logical size)."""
    Fx = np.asarray(Fx, float).reshape(-1, n)
    Fu = np.asarray(Fu, float).reshape(-1, d)
    if n > MAX_N or d > MAX_D or Fx.shape[0] > MAX_FX or Fu.shape[0] > MAX_FU or m > MAX_M:
        raise ValueError("problem dimensions exceed the C ABI limits")
    D = PlanDesc()
    D.controller, D.model = int(controller), int(model)
    D.n, D.d, D.N, D.NB, D.m = int(n), int(d), int(N), int(NB), int(m)
    D.nFx, D.nFu = int(Fx.shape[0]), int(Fu.shape[0])
    D.maxit = int(maxit)
    D.dt, D.ralpha = float(dt), float(ralpha)
    _fill(D.Q, np.asarray(Q, float).reshape(n, n))
    _fill(D.R, np.asarray(R, float).reshape(d, d))
    _fill(D.Qf, np.asarray(Q if Qf is None else Qf, float).reshape(n, n))
    _fill(D.dR, np.zeros(d) if dR is None else dR)
    _fill(D.Fx, Fx)
    _fill(D.bx, np.asarray(bx, float).ravel())
    _fill(D.Fu, Fu)
    _fill(D.bu, np.asarray(bu, float).ravel())
    _fill(D.Qslack, Qslack)
    _fill(D.mc, mc)
    D.feastol, D.abstol, D.reltol = feastol, abstol, reltol
    D.flags = int(flags)
    return D


def policy_array(rows):
    """rows: iterable (per ego) of iterables of (kind, params) -> ctypes array."""
    rows = [list(r) for r in rows]
    flat = [pp for r in rows for pp in r]
    arr = (Policy * len(flat))()
    for i, (kind, params) in enumerate(flat):
        arr[i].kind = int(kind)
        for j, v in enumerate(params):
            arr[i].p[j] = float(v)
    return arr
