"""Python handle over a libbmpc plan: one batch of egos sharing one controller/model."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from ._lib import check, lib

_CTX = {}


def context(device: int = 0):
    """One bmpc_ctx per HIP device per process."""
    if device not in _CTX:
        h = C.c_void_p()
        check(lib().bmpc_open(device, C.byref(h)), "bmpc_open")
        _CTX[device] = h
    return _CTX[device]


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class BatchPlan:
    """A batch of ``batch`` independent egos, each with its own scenario tree, warm start
    and policy set, solved together by one kernel launch per phase."""

    def __init__(self, desc: abi.PlanDesc, batch: int, device: int = 0):
        self.desc = desc
        self.batch = int(batch)
        self.device = device
        self._ctx = context(device)
        h = C.c_void_p()
        check(lib().bmpc_plan_create(self._ctx, C.byref(desc), self.batch, C.byref(h)), "bmpc_plan_create")
        self._h = h
        info = np.zeros(abi.INFO_COUNT, np.int32)
        check(lib().bmpc_plan_info(h, _p(info)), "bmpc_plan_info")
        self.info = info
        self.T, self.U = int(info[abi.INFO_T]), int(info[abi.INFO_U])
        self.bdim, self.nbranch = int(info[abi.INFO_BDIM]), int(info[abi.INFO_NBRANCH])
        self.nv, self.neq = int(info[abi.INFO_NV]), int(info[abi.INFO_NEQ])
        self.nrows, self.ncones = int(info[abi.INFO_NROWS]), int(info[abi.INFO_NCONES])

    def close(self):
        if getattr(self, "_h", None):
            lib().bmpc_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- state ----------------------------------------------------------------------------
    def set_policies(self, rows, mask=None):
        """rows: per ego, m (kind, params) tuples (``update_backup``)."""
        arr = abi.policy_array(rows)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        check(lib().bmpc_set_policies(self._h, arr, _p(m)), "bmpc_set_policies")

    def get_policies(self):
        """The policies in force, per ego m (kind, params) tuples -- including the device-side
        lane-change re-targets of env_step_device."""
        arr = (abi.Policy * (self.batch * self.desc.m))()
        check(lib().bmpc_get_policies(self._h, arr), "bmpc_get_policies")
        m = self.desc.m
        return [[(int(arr[e * m + i].kind), tuple(arr[e * m + i].p)) for i in range(m)] for e in range(self.batch)]

    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        check(lib().bmpc_reset(self._h, _p(m)), "bmpc_reset")

    # ---- solves ---------------------------------------------------------------------------
    def solve(self, x, z, xref):
        B, n, d = self.batch, self.desc.n, self.desc.d
        x, z, xref = (np.ascontiguousarray(np.asarray(v, np.float64).reshape(B, n)) for v in (x, z, xref))
        out = dict(upred=np.zeros((B, self.U, d)), xpred=np.zeros((B, self.T, n)),
                   branch_w=np.zeros((B, self.nbranch - 1)), J=np.zeros(B),
                   status=np.zeros(B, np.int32), iters=np.zeros(B, np.int32))
        check(lib().bmpc_solve(self._h, _p(x), _p(z), _p(xref), *(_p(out[k]) for k in
                               ("upred", "xpred", "branch_w", "J", "status", "iters"))), "bmpc_solve")
        return out

    def solve_device(self, x_ptr, z_ptr, xref_ptr, upred_ptr=None, xpred_ptr=None, bw_ptr=None,
                     J_ptr=None, status_ptr=None, iters_ptr=None, stream=None):
        """Device-pointer variant (e.g. torch tensors' data_ptr()), asynchronous, enqueued on
        `stream` (a hipStream_t handle; None = the plan's own non-blocking stream, which is
        NOT ordered with the legacy default stream -- pass the caller's stream)."""
        vp = [C.c_void_p(p) if p else None for p in (x_ptr, z_ptr, xref_ptr, upred_ptr, xpred_ptr,
                                                     bw_ptr, J_ptr, status_ptr, iters_ptr, stream)]
        check(lib().bmpc_solve_device(self._h, *vp), "bmpc_solve_device")

    def env_step_device(self, env: abi.EnvDesc, t: int, scene_ptr, upred_ptr, x_ptr, z_ptr, xref_ptr,
                        J_ptr=None, status_ptr=None, iters_ptr=None, stats_ptr=None, stream=None):
        """One closed-loop sim_overtake step of every ego on the device (bmpc_env_step):
        Euler step with the last uPred[0], collision flag, obstacle backup choice, lane /
        lane-change-target bookkeeping and x_ref -> the next solve's x, z, xref.  Async."""
        vp = [C.c_void_p(p) if p else None for p in (scene_ptr, upred_ptr, J_ptr, status_ptr, iters_ptr,
                                                     x_ptr, z_ptr, xref_ptr, stats_ptr, stream)]
        check(lib().bmpc_env_step(self._h, C.byref(env), int(t), *vp), "bmpc_env_step")

    def loop_device(self, env: abi.EnvDesc, t0: int, nsteps: int, scene_ptr, upred_ptr, x_ptr, z_ptr, xref_ptr,
                    J_ptr, status_ptr, iters_ptr, stats_ptr=None, stream=None):
        """nsteps closed-loop steps of every ego (bmpc_loop_device): env_step_device(t) then
        solve_device for t = t0 .. t0+nsteps-1, the same results; one fused launch (k_loop) when
        the batch takes the one-wave IPM.  Async on `stream`."""
        vp = [C.c_void_p(p) if p else None for p in (scene_ptr, upred_ptr, x_ptr, z_ptr, xref_ptr, J_ptr, status_ptr,
                                                     iters_ptr, stats_ptr, stream)]
        check(lib().bmpc_loop_device(self._h, C.byref(env), int(t0), int(nsteps), *vp), "bmpc_loop_device")

    def get_warm_start(self):
        """Checkpoint of the per-ego warm start (uLin, p, Jcons, OldInput)."""
        B, d = self.batch, self.desc.d
        uLin = np.zeros((B, self.U + 1, d))
        p = np.zeros((B, self.bdim, self.desc.m))
        jc = np.zeros(B)
        old = np.zeros((B, d))
        check(lib().bmpc_get_warm_start(self._h, _p(uLin), _p(p), _p(jc), _p(old)), "bmpc_get_warm_start")
        return dict(uLin=uLin, p=p, jcons=jc, old_input=old)

    def set_warm_start(self, uLin, p=None, jcons=None, old_input=None, mask=None):
        """Resume from a checkpoint (the next solve runs updatetree); None keeps a part."""
        B, d = self.batch, self.desc.d
        uLin = np.ascontiguousarray(np.asarray(uLin, np.float64).reshape(B, self.U + 1, d))
        p = None if p is None else np.ascontiguousarray(np.asarray(p, np.float64).reshape(B, self.bdim, self.desc.m))
        jc = None if jcons is None else np.ascontiguousarray(np.asarray(jcons, np.float64).reshape(B))
        old = None if old_input is None else np.ascontiguousarray(np.asarray(old_input, np.float64).reshape(B, d))
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        check(lib().bmpc_set_warm_start(self._h, _p(uLin), _p(p), _p(jc), _p(old), _p(m)), "bmpc_set_warm_start")

    def set_transform(self, S=None, bx=None, s_on=None, mask=None):
        """Per-ego state transformation S [B,n,n] (None = "S is None" for every ego) and
        state bound bx [B,nFx] (None = keep) of the next solves -- the S / bx arguments of
        BranchMPC_CVaR.solve (MPC_branch.py:2043-2057); HIGHWAY_MERGE plans and HIGHWAY CVaR
        plans created with abi.PLAN_TRANSFORM."""
        B, n = self.batch, self.desc.n
        S = None if S is None else np.ascontiguousarray(np.asarray(S, np.float64).reshape(B, n, n))
        bx = None if bx is None else np.ascontiguousarray(np.asarray(bx, np.float64).reshape(B, self.desc.nFx))
        on = None if s_on is None else np.ascontiguousarray(s_on, np.uint8)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        check(lib().bmpc_set_transform(self._h, _p(S), _p(on), _p(bx), _p(m)), "bmpc_set_transform")

    def set_fx(self, Fx, mask=None):
        """Per-ego state-constraint matrix Fx [B,nFx,n] of the next solves -- the Fx argument of
        BranchMPC_CVaR.solve (MPC_branch.py:2055-2056), kept until the next one; transform
        plans only (bmpc_set_fx)."""
        Fx = np.ascontiguousarray(np.asarray(Fx, np.float64).reshape(self.batch, self.desc.nFx, self.desc.n))
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        check(lib().bmpc_set_fx(self._h, _p(Fx), _p(m)), "bmpc_set_fx")

    def branch_dp(self):
        """BranchTree.dp (d p / d x) of every non-leaf branch of the last solve [B,bdim,m,n]."""
        out = np.zeros((self.batch, self.bdim, self.desc.m, self.desc.n))
        check(lib().bmpc_get_branch_dp(self._h, _p(out)), "bmpc_get_branch_dp")
        return out

    def get_robust_warm_start(self):
        """robustMPC's warm start: xLin [B,T,n], uLin [B,U,d], OldInput [B,d]."""
        B, n, d = self.batch, self.desc.n, self.desc.d
        xl, ul, old = np.zeros((B, self.T, n)), np.zeros((B, self.U, d)), np.zeros((B, d))
        check(lib().bmpc_get_robust_warm_start(self._h, _p(xl), _p(ul), _p(old)), "bmpc_get_robust_warm_start")
        return dict(xLin=xl, uLin=ul, old_input=old)

    def set_robust_warm_start(self, xLin, uLin, old_input=None, mask=None):
        """robustMPC resume: the shifted prediction (MPC_branch.py:1429-1431) and OldInput."""
        B, n, d = self.batch, self.desc.n, self.desc.d
        xl = np.ascontiguousarray(np.asarray(xLin, np.float64).reshape(B, self.T, n))
        ul = np.ascontiguousarray(np.asarray(uLin, np.float64).reshape(B, self.U, d))
        old = None if old_input is None else np.ascontiguousarray(np.asarray(old_input, np.float64).reshape(B, d))
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        check(lib().bmpc_set_robust_warm_start(self._h, _p(xl), _p(ul), _p(old), _p(m)),
              "bmpc_set_robust_warm_start")

    def tree(self):
        B, n, d = self.batch, self.desc.n, self.desc.d
        out = dict(xbar=np.zeros((B, self.T, n)), ubar=np.zeros((B, self.U, d)),
                   zbar=np.zeros((B, self.T, n)), w=np.zeros((B, self.nbranch)),
                   p=np.zeros((B, self.bdim, self.desc.m)), sol=np.zeros((B, self.nv)))
        check(lib().bmpc_get_tree(self._h, *(_p(out[k]) for k in ("xbar", "ubar", "zbar", "w", "p", "sol"))),
              "bmpc_get_tree")
        return out

    def set_lane_ref(self, grid, values):
        """The lane reference psiref(X) of the plan's *_PSIREF policies (bmpc_set_lane_ref)."""
        g, v = (np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1)) for a in (grid, values))
        check(lib().bmpc_set_lane_ref(self._h, g.size, _p(g), _p(v)), "bmpc_set_lane_ref")

    def last_kernel(self):
        """The solver kernel the plan's last solve launched (abi.KERNEL_*, BMPC_INFO_SOLVER)."""
        info = np.zeros(abi.INFO_COUNT, np.int32)
        check(lib().bmpc_plan_info(self._h, _p(info)), "bmpc_plan_info")
        return int(info[abi.INFO_SOLVER])

    # ---- timing ---------------------------------------------------------------------------
    PHASES = ("tree", "resid", "scaling", "factor", "coupling", "kkt", "treesolve", "refine", "-",
              "init", "total", "nsolve", "applyW", "applyG", "applyGT", "ntree", "G_lp", "G_cone", "napplyG",
              "ts_pre", "ts_bw", "ts_fw", "ts_post", "riccati", "coup_ts", "coup_dot", "coup_lu", "lu_solve",
              "kkt_back", "ric_load", "ric_a", "ric_b")

    def counters(self, width=24):
        """Per-ego phase cycle counters (non-zero only for a -DBMPC_PROFILE build, whose counter
        block is 32 wide: pass width=32 for it)."""
        out = np.zeros((self.batch, width))
        check(lib().bmpc_get_counters(self._h, _p(out)), "bmpc_get_counters")
        return out

    def enable_timing(self, on=True):
        check(lib().bmpc_enable_timing(self._h, 1 if on else 0), "bmpc_enable_timing")

    def timing(self):
        ms = np.zeros(2)
        cnt = C.c_int32()
        check(lib().bmpc_timing(self._h, _p(ms), C.byref(cnt)), "bmpc_timing")
        return dict(tree_ms=float(ms[0]), ipm_ms=float(ms[1]), count=int(cnt.value))


def model_eval(desc: abi.PlanDesc, pol_rows, x, u, z, device: int = 0, lane_ref=None):
    """Batched PredictiveModel evaluation on the GPU (parity entry); lane_ref = (grid, values)
    of the psiref policies' lane reference (bmpc_model_eval_ref)."""
    x, u, z = (np.ascontiguousarray(np.atleast_2d(np.asarray(v, np.float64))) for v in (x, u, z))
    B, n, d, m, N = x.shape[0], desc.n, desc.d, desc.m, desc.N
    out = dict(A=np.zeros((B, n, n)), B=np.zeros((B, n, d)), C=np.zeros((B, n)), xp=np.zeros((B, n)),
               p=np.zeros((B, m)), dp=np.zeros((B, m, n)), zpred=np.zeros((B, N, m * n)),
               h0=np.zeros(B), dh=np.zeros((B, n)))
    arr = abi.policy_array(pol_rows)
    g, v = (None, None) if lane_ref is None else (np.ascontiguousarray(np.asarray(a, np.float64).reshape(-1))
                                                  for a in lane_ref)
    check(lib().bmpc_model_eval_ref(context(device), C.byref(desc), arr, 0 if g is None else g.size, _p(g), _p(v),
                                    B, _p(x), _p(u), _p(z),
                                    *(_p(out[k]) for k in ("A", "B", "C", "xp", "p", "dp", "zpred", "h0", "dh"))),
          "bmpc_model_eval_ref")
    return out


def hmm_eval(M, m, consts, xb, u, xbackup, device: int = 0):
    """Batched HMM belief-model linearisation on the GPU (HMM_backup_dyn.py:216-276).
    consts = (dt, L, W, ylb, yub, col_alpha, s1, tran_diag)."""
    xb = np.ascontiguousarray(np.atleast_2d(np.asarray(xb, np.float64)))
    B, nb = xb.shape[0], 4 + M * m
    u = np.ascontiguousarray(np.broadcast_to(np.atleast_2d(np.asarray(u, np.float64)), (B, 2)))
    xbk = np.ascontiguousarray(np.broadcast_to(np.asarray(xbackup, np.float64).reshape(-1, M * m, 4), (B, M * m, 4)))
    hc = np.ascontiguousarray(np.asarray(consts, np.float64).reshape(8))
    out = dict(xbp=np.zeros((B, nb)), A=np.zeros((B, nb, nb)), B=np.zeros((B, nb, 2)), C=np.zeros((B, nb)),
               h0=np.zeros((B, M, m)), Jh=np.zeros((B, M, m, nb)))
    check(lib().bmpc_hmm_eval(context(device), M, m, _p(hc), B, _p(xb), _p(u), _p(xbk),
                              *(_p(out[k]) for k in ("xbp", "A", "B", "C", "h0", "Jh"))), "bmpc_hmm_eval")
    return out


def qp_arrays(P, q, A, l, u):
    """CSC arrays of one QP -- or of a batch sharing one pattern -- in bmpc_qp_solve's layout.

    ``P`` / ``A`` are scipy sparse or dense matrices (or equal-length sequences of them); only
    the upper triangle of P is kept (OSQP's interface does the same, PredictiveControllers.py:
    325).  A batch's pattern is the union of its members' patterns."""
    import scipy.sparse as sp
    many = isinstance(P, (list, tuple))
    B = len(P) if many else 1
    same = many and all(p is P[0] for p in P) and all(a is A[0] for a in A)   # one matrix pair, B right sides
    Ps = [sp.triu(sp.csc_matrix(p), format="csc") for p in ([P[0]] if same else P if many else [P])]
    As = [sp.csc_matrix(a) for a in ([A[0]] if same else A if many else [A])]
    n = Ps[0].shape[1]
    m = As[0].shape[0]

    def pattern(ms):
        pat = sp.csc_matrix(ms[0].shape)
        for mat in ms:
            pat = pat + sp.csc_matrix((np.ones(mat.nnz), mat.indices, mat.indptr), shape=mat.shape)
        pat = sp.csc_matrix(pat)
        pat.sort_indices()
        rows = pat.indices.astype(np.int64)
        cols = np.repeat(np.arange(pat.shape[1]), np.diff(pat.indptr))
        vals = np.stack([np.asarray(sp.csr_matrix(mat)[rows, cols]).reshape(-1) for mat in ms]) if len(rows) else \
            np.zeros((len(ms), 0))
        return pat.indptr.astype(np.int32), pat.indices.astype(np.int32), vals

    Pp, Pi, Px = pattern(Ps)
    Ap, Ai, Ax = pattern(As) if m else (np.zeros(n + 1, np.int32), np.zeros(0, np.int32), np.zeros((len(As), 0)))
    if same:
        Px, Ax = np.repeat(Px, B, axis=0), np.repeat(Ax, B, axis=0)
    def f2(a, k):
        a = np.asarray(a, np.float64)
        return np.ascontiguousarray(np.broadcast_to(a.reshape(-1, k) if k else np.zeros((B, 0)), (B, k)))
    return dict(n=n, m=m, Pp=Pp, Pi=Pi, Ap=Ap, Ai=Ai, Px=np.ascontiguousarray(Px), q=f2(q, n),
                Ax=np.ascontiguousarray(Ax), l=f2(l, m), u=f2(u, m))


def qp_solve(P, q, A, l, u, max_iter: int = 100, eps: float = 1e-10, device: int = 0):
    """OSQP-form QP(s)  min 1/2 x'Px + q'x  s.t. l <= Ax <= u  on the GPU (bmpc_qp_solve:
    interior point on the band-ordered KKT matrix, one wave per problem).  Returns
    dict(x [B][n], y [B][m], status [B] (1 solved, -2 max_iter, -8 numerics), iters [B],
    info = (KKT dimension, bandwidth, inequality rows, band entries))."""
    a = qp_arrays(P, q, A, l, u)
    B, n, m = a["q"].shape[0], a["n"], a["m"]
    x, y = np.zeros((B, n)), np.zeros((B, max(m, 1)))
    st, it, info = np.zeros(B, np.int32), np.zeros(B, np.int32), np.zeros(4, np.int32)
    check(lib().bmpc_qp_solve(context(device), n, m, _p(a["Pp"]), _p(a["Pi"]), _p(a["Ap"]), _p(a["Ai"]), B,
                              _p(a["Px"]), _p(a["q"]), _p(a["Ax"]), _p(a["l"]), _p(a["u"]), int(max_iter),
                              float(eps), _p(x), _p(y), _p(st), _p(it), _p(info)), "bmpc_qp_solve")
    return dict(x=x, y=y[:, :m], status=st, iters=it, info=info)
