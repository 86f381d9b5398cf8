"""High-accuracy stand-in for OSQP + polish (oracle; test-only).

The reference builds a fresh ``OSQP()`` per solve with ``polish=True``
(``MPC_branch.py:476-481``) and treats ``status_val == 1`` as feasible (``:482``).
OSQP (un-vendored, unpinned, absent) is an ADMM method whose *polished* output is the
exact QP optimum up to ~1e-9 when polishing succeeds, so this oracle returns that optimum
with a Mehrotra primal-dual interior-point method instead of restating ADMM.

OSQP's Python interface keeps only the upper triangle of ``P``; the reference hands it a
non-symmetric ``P`` (``Hu[0:d,0:d] += dR`` broadcast, ``MPC_branch.py:312``), so
``P_eff = triu(P) + triu(P, 1)'`` here.  That interface behaviour is itself unpinned
 and recorded as such.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


def osqp_upper(P):
    U = sp.triu(sp.csc_matrix(P), format="csc")
    return (U + sp.triu(U, 1).T).tocsc()


INF = 1e20    # |bound| >= INF is infinite (OSQP_INFTY = 1e30)


def osqp_like_solve(prob, tol=1e-10, maxit=100, verbose=False):
    """min 1/2 x'Px + q'x  s.t. l <= Ax <= u (OSQP's form): rows with l == u are equalities,
    every other finite bound is a one-sided row (a'x <= u, -a'x <= -l), free rows drop."""
    P = osqp_upper(prob.P)
    q = prob.q
    A = sp.csr_matrix(prob.A)
    l, u = np.asarray(prob.l, float), np.asarray(prob.u, float)
    fl, fu = l > -INF, u < INF
    eq = fl & fu & (l == u)
    up, lo = fu & ~eq, fl & ~eq
    E, e = A[eq].tocsc(), u[eq]
    G = sp.vstack([A[up], -A[lo]]).tocsc()
    g = np.concatenate([u[up], -l[lo]])
    n, p, m = P.shape[0], E.shape[0], G.shape[0]

    def kkt(dsz):
        K = sp.bmat([[P, E.T, G.T], [E, None, None], [G, None, -sp.diags(dsz)]], format="csc")
        return K, spla.splu(K, permc_spec="COLAMD")

    def solve(K, lu, rhs):
        x = lu.solve(rhs)
        for _ in range(3):
            r = rhs - K @ x
            if np.linalg.norm(r, np.inf) < 1e-15 * max(1.0, np.linalg.norm(rhs, np.inf)):
                break
            x += lu.solve(r)
        return x[:n], x[n:n + p], x[n + p:]

    K, lu = kkt(np.ones(m))
    x, y, z = solve(K, lu, np.concatenate([-q, e, g]))
    s = g - G @ x
    a = max(0.0, -np.min(s)) if m else 0.0
    s = s + a + 1.0
    z = np.maximum(np.abs(z), 1.0)
    status = -2
    ninf = lambda v: float(np.max(np.abs(v))) if len(v) else 0.0
    nq = max(1.0, ninf(q))
    for it in range(maxit):
        rd = P @ x + q + E.T @ y + G.T @ z
        re = E @ x - e
        rg = G @ x + s - g
        mu = s @ z / m if m else 0.0
        if verbose:
            print(it, ninf(rd), ninf(re), ninf(rg), mu)
        # rg against max(|g|, |s|): OSQP scales the primal residual by max(|Ax|, |z|), and
        # G x + s - g cancels to the rounding floor of s, which |g| does not bound
        if (ninf(rd) < tol * nq and ninf(re) < tol * max(1, ninf(e))
                and ninf(rg) < tol * max(1, ninf(g), ninf(s)) and mu < tol):
            status = 1
            break
        K, lu = kkt(s / z)
        dx, dy, dz = solve(K, lu, np.concatenate([-rd, -re, -rg + s]))
        ds = -s - (s / z) * dz

        def amax(v, dv):
            neg = dv < 0
            return min(1.0, np.min(-v[neg] / dv[neg])) if np.any(neg) else 1.0

        aa = min(amax(s, ds), amax(z, dz))
        mua = (s + aa * ds) @ (z + aa * dz) / m if m else 0.0
        sig = (mua / mu) ** 3 if mu > 0 else 0.0
        corr = (ds * dz - sig * mu) / z if m else np.zeros(0)
        dx, dy, dz = solve(K, lu, np.concatenate([-rd, -re, -rg + s + corr]))
        ds = -s - (s / z) * dz - corr
        a = 0.99 * min(amax(s, ds), amax(z, dz))
        x, y, z, s = x + a * dx, y + a * dy, z + a * dz, s + a * ds
    return x, dict(status_val=status, iter=it, y_eq=y, z_ineq=z, s=s)
