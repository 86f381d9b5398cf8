"""Restatement of the ECOS interior-point algorithm (oracle; test-only).

The reference calls ``ecos.solve(c, G, h, dims, A, b, verbose=False)``
(``MPC_branch.py:2136``) and treats ``exitFlag >= 0`` as feasible (``:2141``).
ECOS is an un-vendored third-party C library with no pinned version in the reference
 and is absent from this image, so this module restates its *published*
algorithm (Domahidi, Chu, Boyd, "ECOS: An SOCP solver for embedded systems", ECC 2013):

* homogeneous self-dual embedding in (x, y, z, s, tau, kappa);
* Nesterov-Todd scaling for the LP and second-order cones;
* Mehrotra predictor-corrector with sigma = (1 - alpha_aff)^3;
* the three KKT solves per iteration sharing one factorisation
  (RHS1 = [-c; b; h] for the tau direction, affine, combined);
* ECOS default tolerances (feastol = abstol = reltol = 1e-8, inaccurate 1e-4/5e-5),
  maxit = 100, step factor gamma = 0.99, and its exit codes
  (0 optimal, 1 primal infeasible, 2 dual infeasible, 10+ inaccurate, -1 maxit,
  -2 numerics): optimal at the full tolerances; at maxit, or when a step fails
  numerically (ECOS backtracks to its best iterate), inaccurate if the best iterate meets
  the reduced tolerances, else -1 / -2.  No other early exit.

* ECOS's Ruiz equilibration of [A; G] (``ECOS_setup``, ECOS 2.0.x ``equil.c``; :func:`equilibration`).

Linear algebra is a sparse LU of the full KKT matrix
``[[0, A', G'], [A, 0, 0], [G, 0, -W'W]]`` (ECOS uses a sparse LDL' with static
regularisation; the solution of the KKT system is the same) with iterative refinement.
Parity of the *iterates* against ECOS is unpinned (no recorded ECOS output exists);
the returned point is certified by its own KKT residuals.

**Declared non-ECOS ingredient: the rotated-cone row boost** (:func:`boost_rows`, applied after
the equilibration).  The CVaR cones' first and last rows are (1 - a, ..., 1 + a) with |a| up to
~1e3 (``MPC_branch.py:1948-1964``); the oracle and the kernel (``k_tree`` writes the per-cone
beta = 1/2 log(max(1, sum xbar'Q xbar + ubar'R ubar)), ``oracle.tree.CVaRController.cone_boost``)
pre-multiply those two rows by the Lorentz boost T_beta, a cone automorphism: the feasible set,
the optimum and the returned (unboosted) x, y, z, s are unchanged, but the NT scaling, the initial
point and the exit tests' residual norms are formed in the boosted coordinates.  ECOS has no such
step.  Kept after the round-6 A/B (``tools/boost_experiment.py``, ``profiles/r06/boost_ab.log``):
with equilibration on and beta = 0 this restatement reaches ECOS's full tolerances on 1 of the 26
solver problems the six CVaR recordings hold (25 with the boost) at 46.7 iterations on average
(29.9), on none of 288 seeded closed-loop solves (223 with it; 43.0 vs 27.0 iterations), and the
kernel algorithm (host build, -DBMPC_CONE_BOOST=0) on 9 of the 184 recorded highway steps (181 with
it): the boost is what makes this restatement's (and the kernel's) cone arithmetic reach 1e-8 on
these rows.  The recordings' exit codes are therefore those of ECOS's algorithm
plus this boost.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

FEASTOL = 1e-8
ABSTOL = 1e-8
RELTOL = 1e-8
FEASTOL_INACC = 1e-4
ABSTOL_INACC = 5e-5
RELTOL_INACC = 5e-5
MAXIT = 100
GAMMA = 0.99
STEPMIN = 1e-6
STEPMAX = 0.999
SIGMAMIN = 1e-4
SIGMAMAX = 1.0

ECOS_OPTIMAL, ECOS_PINF, ECOS_DINF, ECOS_INACC_OFFSET = 0, 1, 2, 10
ECOS_MAXIT, ECOS_NUMERICS = -1, -2
DENSE_DEBUG = False


class Cones:
    def __init__(self, dims):
        self.l = int(dims['l'])
        self.q = [int(v) for v in dims.get('q', [])]
        self.off = []
        o = self.l
        for qd in self.q:
            self.off.append(o)
            o += qd
        self.m = o
        self.deg = self.l + len(self.q)

    def soc(self, v, k):
        o = self.off[k]
        return v[o:o + self.q[k]]


# ---- Jordan algebra helpers --------------------------------------------------------------
def _jprod(C, u, v):
    out = np.empty_like(u)
    out[:C.l] = u[:C.l] * v[:C.l]
    for k in range(len(C.q)):
        o, q = C.off[k], C.q[k]
        a, b = u[o:o + q], v[o:o + q]
        out[o] = a @ b
        out[o + 1:o + q] = a[0] * b[1:] + b[0] * a[1:]
    return out


def _jdiv(C, lam, v):
    """x with lam o x = v."""
    out = np.empty_like(v)
    out[:C.l] = v[:C.l] / lam[:C.l]
    for k in range(len(C.q)):
        o, q = C.off[k], C.q[k]
        l, w = lam[o:o + q], v[o:o + q]
        rho = cone_res(l)
        x0 = (l[0] * w[0] - l[1:] @ w[1:]) / rho
        out[o] = x0
        out[o + 1:o + q] = (w[1:] - x0 * l[1:]) / l[0]
    return out


def _unit(C):
    e = np.zeros(C.m)
    e[:C.l] = 1.0
    for o in C.off:
        e[o] = 1.0
    return e


def _bring2cone(C, r):
    """ECOS ``bring2cone``: s = r + (1 + alpha) e with alpha the worst cone residual."""
    alpha = -0.99
    if C.l:
        mn = -np.min(r[:C.l])
        if mn >= 0 and mn > alpha:
            alpha = mn
    for k in range(len(C.q)):
        v = C.soc(r, k)
        cres = v[0] - np.linalg.norm(v[1:])
        if cres <= 0 and -cres > alpha:
            alpha = -cres
    s = r.copy()
    s[:C.l] += 1.0 + alpha
    for o in C.off:
        s[o] += 1.0 + alpha
    return s


def cone_res(v):
    """v0^2 - ||v1||^2 evaluated as (v0-|v_k|)(v0+|v_k|) - sum_{i!=k} v_i^2, k = argmax |v_i|,
    which avoids squaring the dominant component."""
    if len(v) == 1:
        return v[0] * v[0]
    a = np.abs(v[1:])
    k = int(np.argmax(a)) + 1
    rest = v[1:] @ v[1:] - v[k] * v[k]
    return (v[0] - abs(v[k])) * (v[0] + abs(v[k])) - rest


class Scaling:
    """Nesterov-Todd scaling W (symmetric) with W z = W^{-1} s = lambda."""

    def __init__(self, C, s, z):
        self.C = C
        self.dl = np.sqrt(s[:C.l] / z[:C.l])           # W for LP = diag(sqrt(s/z))
        self.eta, self.wb, self.wbar = [], [], []
        for k in range(len(C.q)):
            sk, zk = C.soc(s, k), C.soc(z, k)
            sres = cone_res(sk)
            zres = cone_res(zk)
            if not (sres > 0 and zres > 0):
                raise FloatingPointError("iterate outside the second-order cone")
            sn, zn = math.sqrt(sres), math.sqrt(zres)
            sb, zb = sk / sn, zk / zn
            gam = math.sqrt((1.0 + sb @ zb) / 2.0)
            wb = sb.copy()
            wb[0] += zb[0]
            wb[1:] -= zb[1:]
            wb /= 2.0 * gam                          # wbar' J wbar = 1
            v = wb.copy()
            v[0] += 1.0
            v /= math.sqrt(2.0 * (wb[0] + 1.0))     # (2vv'-J)^2 = 2 wbar wbar' - J
            self.wbar.append(wb)
            self.wb.append(v)
            self.eta.append(math.sqrt(sn / zn))

    def W(self, v):
        out = np.empty_like(v)
        C = self.C
        out[:C.l] = self.dl * v[:C.l]
        for k in range(len(C.q)):
            o, q = C.off[k], C.q[k]
            wb, x = self.wb[k], v[o:o + q]
            Jx = x.copy(); Jx[1:] = -Jx[1:]
            out[o:o + q] = self.eta[k] * (2.0 * wb * (wb @ x) - Jx)
        return out

    def Winv(self, v):
        out = np.empty_like(v)
        C = self.C
        out[:C.l] = v[:C.l] / self.dl
        for k in range(len(C.q)):
            o, q = C.off[k], C.q[k]
            wb, x = self.wb[k], v[o:o + q]
            Jwb = wb.copy(); Jwb[1:] = -Jwb[1:]
            Jx = x.copy(); Jx[1:] = -Jx[1:]
            out[o:o + q] = (2.0 * Jwb * (Jwb @ x) - Jx) / self.eta[k]
        return out

    def Winv_block(self, k):
        """Dense W_k^{-1} = (2 Jv (Jv)' - J) / eta of cone k."""
        v = self.wb[k].copy()
        v[1:] = -v[1:]
        M = 2.0 * np.outer(v, v)
        q = len(v)
        M[0, 0] -= 1.0
        M[np.arange(1, q), np.arange(1, q)] += 1.0
        return M / self.eta[k]

    def W2_blocks(self):
        """Diagonal of W^2 on the LP part and dense W_k^2 per cone."""
        blocks = []
        for k in range(len(self.C.q)):
            q = self.C.q[k]
            wb = self.wbar[k]
            M = 2.0 * np.outer(wb, wb)
            M[0, 0] -= 1.0
            M[np.arange(1, q), np.arange(1, q)] += 1.0
            blocks.append(self.eta[k] ** 2 * M)
        return self.dl ** 2, blocks


def _max_step(C, lam, d):
    """Largest alpha with lam + alpha d in the cone (lam interior)."""
    amax = np.inf
    if C.l:
        dl = d[:C.l]
        neg = dl < 0
        if np.any(neg):
            amax = min(amax, np.min(-lam[:C.l][neg] / dl[neg]))
    for k in range(len(C.q)):
        o, q = C.off[k], C.q[k]
        l, dk = lam[o:o + q], d[o:o + q]
        ln2 = cone_res(l)
        if ln2 <= 0:
            return 0.0
        ln = math.sqrt(ln2)
        lb = l / ln
        rho0 = lb[0] * dk[0] - lb[1:] @ dk[1:]
        fac = (rho0 + dk[0]) / (lb[0] + 1.0)
        rho1 = dk[1:] - fac * lb[1:]
        t = np.linalg.norm(rho1) - rho0
        if t > 0:
            amax = min(amax, ln / t)
    return amax


def _line_search(C, lam, ds, dz, tau, dtau, kap, dkap):
    """Largest step keeping (lam + a ds, lam + a dz, tau, kappa) interior, capped at STEPMAX.

    Unlike a STEPMIN floor, a step is never forced past the boundary: a (near) zero step is
    reported to the caller, which treats it as a numerical stall."""
    a = min(_max_step(C, lam, ds), _max_step(C, lam, dz))
    if dtau < 0:
        a = min(a, -tau / dtau)
    if dkap < 0:
        a = min(a, -kap / dkap)
    return max(0.0, min(a, STEPMAX))


class KKT:
    """Sparse LU of the W-scaled KKT matrix

        [[0, A', G'W^-1], [A, 0, 0], [W^-1 G, 0, -I]]   in (dx, dy, W dz),

    which is the system [[0, A', G'], [A, 0, 0], [G, 0, -W'W]] of ECOS with the cone rows
    scaled by W^-1 (better conditioned: the scaling enters as a square root), followed by
    iterative refinement.
    """

    def __init__(self, A, G, C):
        self.A, self.G, self.C = A, G.tocsr(), C
        self.n = G.shape[1]
        self.p = A.shape[0]
        self.mm = G.shape[0]

    def factor(self, W):
        C = self.C
        self.Wsc = W
        Gl = sp.diags(1.0 / W.dl) @ self.G[:C.l]
        blocks = [Gl]
        for k in range(len(C.q)):
            o, q = C.off[k], C.q[k]
            Gk = self.G[o:o + q]
            cols = np.unique(Gk.indices)
            Gd = Gk[:, cols].toarray()
            Bk = sp.csr_matrix(W.Winv_block(k) @ Gd)
            Bk = sp.csr_matrix((Bk.data, cols[Bk.indices], Bk.indptr), shape=(q, self.n))
            blocks.append(Bk)
        Gs = sp.vstack(blocks).tocsc()
        self.Gs = Gs
        Z = sp.csc_matrix((self.n, self.n))
        K = sp.bmat([[Z, self.A.T, Gs.T],
                     [self.A, None, None],
                     [Gs, None, -sp.eye(self.mm)]], format='csc')
        self.K = K
        if DENSE_DEBUG:
            import scipy.linalg as sla
            lu = sla.lu_factor(K.toarray())
            self.lu = type('LU', (), {'solve': staticmethod(lambda r: sla.lu_solve(lu, r))})
        else:
            self.lu = spla.splu(K, permc_spec='COLAMD')

    def solve(self, rx, ry, rz, nitref=3):
        """Solve [[0,A',G'],[A,0,0],[G,0,-W^2]] [x;y;z] = [rx;ry;rz]."""
        rhs = np.concatenate([rx, ry, self.Wsc.Winv(rz)])
        sol = self.lu.solve(rhs)
        nrm = max(1.0, np.linalg.norm(rhs, np.inf))
        for _ in range(nitref):
            r = rhs - self.K @ sol
            if np.linalg.norm(r, np.inf) <= 1e-14 * nrm:
                break
            sol += self.lu.solve(r)
        n, p = self.n, self.p
        return sol[:n], sol[n:n + p], self.Wsc.Winv(sol[n + p:])


def _cone_basis(C, k):
    o, q = C.off[k], C.q[k]
    for i in range(q):
        e = np.zeros(C.m)
        e[o + i] = 1.0
        yield e


class _Identity:
    def __init__(self, C):
        self.C = C
        self.dl = np.ones(C.l)

    def Winv(self, v):
        return v.copy()

    def Winv_block(self, k):
        return np.eye(self.C.q[k])


def boost_rows(C, G, h, beta):
    """Apply the Lorentz boost T_b (a cone automorphism, T_b Q = Q) to the first/last rows of
    each cone: (G, h) -> (T G, T h).  The feasible set and the optimum are unchanged; it only
    balances the rotated-cone rows (1-a, ..., 1+a) of MPC_branch.py:1948-1964 whose |a| ~ 1e3
    would otherwise cost ~3 digits in every cone residual.  Returns new (G, h)."""
    G = G.tolil(copy=True)
    h = h.copy()
    for k, b in enumerate(beta):
        if b == 0.0:
            continue
        o, q = C.off[k], C.q[k]
        ch, sh = math.cosh(b), math.sinh(b)
        r0 = G[o].toarray().ravel()
        rl = G[o + q - 1].toarray().ravel()
        G[o] = ch * r0 + sh * rl
        G[o + q - 1] = sh * r0 + ch * rl
        h0, hl = h[o], h[o + q - 1]
        h[o], h[o + q - 1] = ch * h0 + sh * hl, sh * h0 + ch * hl
    return G.tocsc(), h


def unboost_dual(C, z, beta):
    """Dual of the original cone rows: z_orig = T' z (T symmetric for a boost)."""
    z = z.copy()
    for k, b in enumerate(beta):
        if b == 0.0:
            continue
        o, q = C.off[k], C.q[k]
        ch, sh = math.cosh(b), math.sinh(b)
        z0, zl = z[o], z[o + q - 1]
        z[o], z[o + q - 1] = ch * z0 + sh * zl, sh * z0 + ch * zl
    return z


EQUIL_ITERS = 3      # ECOS glblopts.h EQUIL_ITERS (RUIZ_EQUIL)
EQUILIBRATE = True   # module default of ecos_solve(equilibrate=...): ECOS equilibrates (ECOS_setup)


def equilibration(A, G, C, iters=EQUIL_ITERS):
    """ECOS's Ruiz equilibration of [A; G] (ECOS 2.0.x ``equil.c``, ``use_ruiz_equilibration``,
    run by ``ECOS_setup`` before the first iteration; restated, ECOS is not in this image):
    ``iters`` rounds of -- column max-abs over A and G, row max-abs of A and of G, the rows of
    each second-order cone given the SUM of their row maxima (one factor per cone keeps the cone
    invariant), square roots (values below 1e-6 -> 1), rows and columns divided by them, the
    factors accumulated.  Returns (xequil, Aequil, Gequil): the solver then works on
    c / xequil, diag(1/Aequil) A diag(1/xequil), b / Aequil, diag(1/Gequil) G diag(1/xequil),
    h / Gequil, and ``backscale`` returns x / xequil, y / Aequil, z / Gequil, s * Gequil."""
    A = sp.csr_matrix(A, dtype=float, copy=True)
    G = sp.csr_matrix(G, dtype=float, copy=True)
    n = G.shape[1]
    xe, ae, ge = np.ones(n), np.ones(A.shape[0]), np.ones(G.shape[0])

    def rowmax(M):
        return np.asarray(abs(M).max(axis=1).todense()).ravel() if M.shape[0] else np.zeros(0)

    for _ in range(iters):
        xt = np.asarray(abs(G).max(axis=0).todense()).ravel()
        if A.shape[0]:
            xt = np.maximum(xt, np.asarray(abs(A).max(axis=0).todense()).ravel())
        at, gt = rowmax(A), rowmax(G)
        for o, q in zip(C.off, C.q):
            gt[o:o + q] = gt[o:o + q].sum()
        xt, at, gt = (np.where(np.abs(v) < 1e-6, 1.0, np.sqrt(v)) for v in (xt, at, gt))
        A = sp.diags(1.0 / at) @ A @ sp.diags(1.0 / xt)
        G = sp.diags(1.0 / gt) @ G @ sp.diags(1.0 / xt)
        xe, ae, ge = xe * xt, ae * at, ge * gt
    return xe, ae, ge


def ecos_solve(prob, maxit=MAXIT, feastol=FEASTOL, abstol=ABSTOL, reltol=RELTOL, verbose=False, equilibrate=None):
    """Solve min c'x s.t. Ax = b, Gx + s = h, s in K. Returns (x, info).

    ``equilibrate`` (default: module EQUILIBRATE) scales the data as ECOS_setup does
    (:func:`equilibration`) and returns the back-scaled point; ``prob.cone_boost`` (optional,
    per cone) then applies :func:`boost_rows` to the (scaled) cone rows."""
    C = Cones(prob.dims)
    beta = list(getattr(prob, 'cone_boost', None) or [0.0] * len(C.q))
    c, A, b = prob.c, prob.A.tocsc(), prob.b
    G0, h0 = prob.G.tocsc(), prob.h
    if EQUILIBRATE if equilibrate is None else equilibrate:
        xe, ae, ge = equilibration(A, G0, C)
        c, b, h0 = c / xe, b / ae, h0 / ge
        A = (sp.diags(1.0 / ae) @ A @ sp.diags(1.0 / xe)).tocsc()
        G0 = (sp.diags(1.0 / ge) @ G0 @ sp.diags(1.0 / xe)).tocsc()
    else:
        xe, ae, ge = np.ones(len(c)), np.ones(A.shape[0]), np.ones(G0.shape[0])
    G, h = boost_rows(C, G0, h0, beta)
    n, p, m = G.shape[1], A.shape[0], G.shape[0]
    kkt = KKT(A, G, C)
    e = _unit(C)

    # ---- initial point (W = I) ----
    kkt.factor(_Identity(C))
    x, _, zt = kkt.solve(np.zeros(n), b, h)
    s = _bring2cone(C, -zt)
    _, y, zt = kkt.solve(-c, np.zeros(p), np.zeros(m))
    z = _bring2cone(C, zt)
    tau, kap = 1.0, 1.0

    resx0 = max(1.0, np.linalg.norm(c))
    resy0 = max(1.0, np.linalg.norm(b))
    resz0 = max(1.0, np.linalg.norm(h))
    info = dict(exitFlag=ECOS_MAXIT, iter=0)
    best = None          # (score, iterate, stats)

    def pack(code, it, st, xs, ys, zs, ss, ts):
        info.update(st, exitFlag=code, iter=it)
        info['x'], info['y'] = xs / ts / xe, ys / ts / ae
        info['s'] = unboost_dual(C, ss / ts, [-v for v in beta]) * ge   # T^-1 = T_{-b}
        info['z'] = unboost_dual(C, zs / ts, beta) / ge
        return info['x'], info

    for it in range(maxit + 1):
        # residuals
        rx = A.T @ y + G.T @ z + c * tau
        ry = b * tau - A @ x
        rz = h * tau - G @ x - s
        cx, by, hz = c @ x, b @ y, h @ z
        rt = kap + cx + by + hz
        nx, ny, nz, ns = (np.linalg.norm(v) for v in (x, y, z, s))
        mu = (s @ z + kap * tau) / (C.deg + 1)
        gap = (s @ z) / (tau * tau)
        pcost = cx / tau
        dcost = -(hz + by) / tau
        if pcost < 0:
            relgap = gap / (-pcost)
        elif dcost > 0:
            relgap = gap / dcost
        else:
            relgap = np.nan
        nry = np.linalg.norm(ry) / max(resy0 + nx, 1.0) if p else 0.0
        nrz = np.linalg.norm(rz) / max(resz0 + nx + ns, 1.0)
        pres = max(nry, nrz) / tau
        dres = np.linalg.norm(rx) / max(resx0 + ny + nz, 1.0) / tau
        nrx_h = np.linalg.norm(A.T @ y + G.T @ z)
        pinfres = nrx_h / max(ny + nz, 1.0) if (hz + by) / max(ny + nz, 1.0) < -reltol else np.nan
        dinfres = (max(np.linalg.norm(A @ x) / max(nx, 1.0),
                       np.linalg.norm(G @ x + s) / max(nx + ns, 1.0))
                   if cx / max(nx, 1.0) < -reltol else np.nan)
        stats = dict(pres=pres, dres=dres, gap=gap, relgap=relgap, pcost=pcost,
                     dcost=dcost, mu=mu, tau=tau, kap=kap, pinfres=pinfres, dinfres=dinfres)
        if verbose:
            print(f"it {it:3d} pcost {pcost:+.9e} dcost {dcost:+.9e} gap {gap:.2e} "
                  f"pres {pres:.2e} dres {dres:.2e} k/t {kap / tau:.2e}")

        def exit_check(ft, at, rt_):
            if not (tau > 0 and kap >= 0):
                return None
            if ((-cx > 0 or -by - hz >= -at) and pres < ft and dres < ft
                    and (gap < at or (not np.isnan(relgap) and relgap < rt_))):
                return ECOS_OPTIMAL
            if not np.isnan(dinfres) and dinfres < ft and tau < kap:
                return ECOS_DINF
            if ((not np.isnan(pinfres) and pinfres < ft and tau < kap)
                    or (tau < ft and kap < ft and not np.isnan(pinfres) and pinfres < ft)):
                return ECOS_PINF
            return None

        # ECOS safeguard: remember the best iterate by its worst residual
        score = max(pres, dres, relgap if not np.isnan(relgap) else np.inf)
        if best is None or score < best[0]:
            best = (score, it, stats, x.copy(), y.copy(), z.copy(), s.copy(), tau)

        code = exit_check(feastol, abstol, reltol)
        if code is None and it == maxit:
            code2 = exit_check(FEASTOL_INACC, ABSTOL_INACC, RELTOL_INACC)
            code = ECOS_MAXIT if code2 is None else code2 + ECOS_INACC_OFFSET
        if code is not None:
            return pack(code, it, stats, x, y, z, s, tau)

        try:
            # scaling + factorisation
            W = Scaling(C, s, z)
            lam = W.W(z)
            kkt.factor(W)
            x1, y1, z1 = kkt.solve(-c, b, h)
            den = kap / tau - (c @ x1 + b @ y1 + h @ z1)

            # affine direction: ds = -lam o lam, eta = 1
            xi = -lam
            x2, y2, z2 = kkt.solve(-rx, ry, rz - W.W(xi))
            dk_aff = -kap * tau
            dtau_a = (rt + dk_aff / tau + c @ x2 + b @ y2 + h @ z2) / den
            dz_a = z2 + dtau_a * z1
            Wdz_a = W.W(dz_a)
            dsW_a = xi - Wdz_a
            dkap_a = (dk_aff - kap * dtau_a) / tau
            a_aff = _line_search(C, lam, dsW_a, Wdz_a, tau, dtau_a, kap, dkap_a)
            sigma = min(SIGMAMAX, max(SIGMAMIN, (1.0 - a_aff) ** 3))
            eta = 1.0 - sigma

            # combined direction
            ds_comb = -_jprod(C, lam, lam) - _jprod(C, dsW_a, Wdz_a) + sigma * mu * e
            xi = _jdiv(C, lam, ds_comb)
            x2, y2, z2 = kkt.solve(-eta * rx, eta * ry, eta * rz - W.W(xi))
            dk_c = -kap * tau - dtau_a * dkap_a + sigma * mu
            dtau = (eta * rt + dk_c / tau + c @ x2 + b @ y2 + h @ z2) / den
            dx = x2 + dtau * x1
            dy = y2 + dtau * y1
            dz = z2 + dtau * z1
            Wdz = W.W(dz)
            dsW = xi - Wdz
            dkap = (dk_c - kap * dtau) / tau
            alpha = _line_search(C, lam, dsW, Wdz, tau, dtau, kap, dkap) * GAMMA
            if not alpha > 1e-10:
                raise FloatingPointError("step length collapsed")
            ds = W.W(dsW)
            if verbose:
                print(f"      a_aff {a_aff:.3f} alpha {alpha:.3f} sigma {sigma:.2e}")
            if not (np.all(np.isfinite(dx)) and np.isfinite(dtau)):
                raise FloatingPointError("non-finite direction")
            x = x + alpha * dx
            y = y + alpha * dy
            z = z + alpha * dz
            s = s + alpha * ds
            tau += alpha * dtau
            kap += alpha * dkap
        except (FloatingPointError, ZeroDivisionError, ValueError, RuntimeError):
            # numerical failure: fall back to the best iterate (ECOS backtracking)
            _, bit, bst, bx_, by_, bz_, bs_, btau = best
            x, y, z, s, tau = bx_, by_, bz_, bs_, btau
            pres, dres, relgap = bst['pres'], bst['dres'], bst['relgap']
            gap = bst['gap']
            cx, by, hz = c @ x, b @ y, h @ z
            code2 = exit_check(FEASTOL_INACC, ABSTOL_INACC, RELTOL_INACC)
            code = ECOS_NUMERICS if code2 is None else code2 + ECOS_INACC_OFFSET
            return pack(code, it, bst, x, y, z, s, tau)
    raise AssertionError("unreachable")


def kkt_residuals(prob, x, y, z, s):
    """Optimality certificate of a returned point (independent of the solver)."""
    c, G, h, A, b = prob.c, prob.G, prob.h, prob.A, prob.b
    C = Cones(prob.dims)
    r_dual = np.linalg.norm(A.T @ y + G.T @ z + c) / max(1.0, np.linalg.norm(c))
    r_eq = np.linalg.norm(A @ x - b) / max(1.0, np.linalg.norm(b))
    r_ineq = np.linalg.norm(G @ x + s - h) / max(1.0, np.linalg.norm(h))
    # cone membership of s and z
    worst = 0.0
    if C.l:
        worst = min(worst, float(np.min(s[:C.l])), float(np.min(z[:C.l])))
    for k in range(len(C.q)):
        for v in (C.soc(s, k), C.soc(z, k)):
            worst = min(worst, float(v[0] - np.linalg.norm(v[1:])))
    gap = float(s @ z)
    return dict(dual=r_dual, eq=r_eq, ineq=r_ineq, cone=worst, gap=gap,
                pcost=float(c @ x), dcost=float(-(b @ y) - h @ z))
