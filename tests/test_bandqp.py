"""The batched QP solver (csrc/bmpc_bandqp.h, C ABI bmpc_qp_solve) against the oracle.

OSQP (the reference's QP solver, PredictiveControllers.py:320-340) is absent; the oracle
``oracle/qp_ipm.osqp_like_solve`` returns the exact optimum OSQP's polish targets.  Checked
on CPU through the host build of the same template (tests/hostsim), on the GPU through
libbmpc.so: seeded random QPs with every row class OSQP accepts (equalities, one-sided,
two-sided, free rows), an unconstrained problem, the belief-MPC problems the reference's
own PredictiveControllers assembled (tests/golden/belief_*.npz), the optimality conditions
of the returned dual, and the host analysis' error paths.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from common import coo, golden
from bmpc.plan import qp_arrays
from oracle.qp_ipm import osqp_like_solve
from oracle.tree import QPProblem

X_TOL = 1e-7     # both methods stop at 1e-10 residuals / gap; x agrees to ~1e-12 in practice


def random_qp(n, m, meq, ntwo, rng, nfree=0, density=0.3):
    Mx = sp.random(n, n, 0.2, random_state=rng).toarray()
    P = Mx @ Mx.T + 0.01 * np.eye(n)
    A = sp.random(m, n, density, random_state=rng).toarray()
    x0 = rng.normal(size=n)
    Ax0 = A @ x0
    l = np.full(m, -np.inf)
    u = Ax0 + rng.uniform(0.0, 1.0, m)
    l[:meq] = u[:meq] = Ax0[:meq]
    l[meq:meq + ntwo] = Ax0[meq:meq + ntwo] - rng.uniform(0.0, 1.0, ntwo)
    if nfree:
        l[m - nfree:], u[m - nfree:] = -np.inf, np.inf
    return P, rng.normal(size=n), A, l, u


def oracle_solve(P, q, A, l, u):
    """Split two-sided rows into two one-sided rows (oracle form), drop free rows."""
    rows, lo, hi = [], [], []
    for i in range(A.shape[0]):
        if np.isfinite(l[i]) and l[i] == u[i]:
            rows.append(A[i]), lo.append(l[i]), hi.append(u[i])
            continue
        if np.isfinite(u[i]):
            rows.append(A[i]), lo.append(-np.inf), hi.append(u[i])
        if np.isfinite(l[i]):
            rows.append(-A[i]), lo.append(-np.inf), hi.append(-l[i])
    Ao = sp.csc_matrix(np.array(rows)) if rows else sp.csc_matrix((0, P.shape[0]))
    lo, hi = np.array(lo, float), np.array(hi, float)
    x, info = osqp_like_solve(QPProblem(sp.csc_matrix(P), np.asarray(q, float), Ao, lo, hi,
                                        int(np.sum(~np.isfinite(lo)))))
    return x, info


def check_kkt(P, q, A, l, u, x, y, tol=1e-7):
    """Stationarity with OSQP's dual convention, primal feasibility, complementarity."""
    P = np.asarray(P.todense() if sp.issparse(P) else P)
    A = np.asarray(A.todense() if sp.issparse(A) else A)
    scale = max(1.0, np.abs(q).max())
    assert np.abs(P @ x + q + A.T @ y).max() <= tol * scale
    Ax = A @ x
    assert np.all(Ax <= u + tol * np.maximum(1, np.abs(u))) and np.all(Ax >= l - tol * np.maximum(1, np.abs(l)))
    # y > 0 only at an active upper bound, y < 0 only at an active lower bound
    act_u = np.isfinite(u) & (np.abs(Ax - u) <= 1e-6 * np.maximum(1, np.abs(u)))
    act_l = np.isfinite(l) & (np.abs(Ax - l) <= 1e-6 * np.maximum(1, np.abs(l)))
    assert np.all((y <= 1e-6) | act_u) and np.all((y >= -1e-6) | act_l)


CASES = [  # n, m, equalities, two-sided rows, free rows (the oracle needs >= 1 equality and >= 1 inequality)
    (30, 40, 5, 3, 0), (20, 25, 1, 0, 0), (25, 14, 10, 0, 0), (40, 60, 8, 10, 4), (12, 30, 1, 12, 2)]


def _host(**a):
    import hostsim_lib as H
    return H.qp_solve(a["n"], a["m"], a["Pp"], a["Pi"], a["Ap"], a["Ai"], a["Px"], a["q"], a["Ax"], a["l"], a["u"])


def test_host_build_matches_oracle_on_random_qps():
    rng = np.random.default_rng(11)
    for n, m, meq, ntwo, nfree in CASES:
        P, q, A, l, u = random_qp(n, m, meq, ntwo, rng, nfree)
        r = _host(**qp_arrays(P, q, A, l, u))
        xo, info = oracle_solve(P, q, A, l, u)
        assert r["status"][0] == 1 and info["status_val"] == 1
        np.testing.assert_allclose(r["x"][0], xo, atol=X_TOL * max(1, np.abs(xo).max()))
        check_kkt(P, q, A, l, u, r["x"][0], r["y"][0])
        assert r["info"][0] == n + meq + (m - meq - nfree) + ntwo    # KKT dimension


def test_host_build_unconstrained_and_equality_only():
    rng = np.random.default_rng(5)
    P, q, _, _, _ = random_qp(15, 1, 0, 0, rng)
    r = _host(**qp_arrays(P, q, np.zeros((0, 15)), np.zeros(0), np.zeros(0)))
    np.testing.assert_allclose(r["x"][0], np.linalg.solve(P, -q), rtol=1e-10, atol=1e-10)
    P, q, A, l, u = random_qp(15, 6, 6, 0, rng)
    r = _host(**qp_arrays(P, q, A, l, u))
    K = np.block([[P, A.T], [A, np.zeros((6, 6))]])
    sol = np.linalg.solve(K, np.concatenate([-q, u]))
    np.testing.assert_allclose(r["x"][0], sol[:15], atol=1e-9)
    np.testing.assert_allclose(r["y"][0], sol[15:], atol=1e-8)


def test_host_build_batch_shares_the_pattern():
    """A batch with one pattern and different values equals the problems solved one by one."""
    rng = np.random.default_rng(3)
    P, q, A, l, u = random_qp(20, 30, 4, 5, rng)
    Ps = [P * s for s in (1.0, 2.0, 0.5)]
    qs = [q, -q, 2 * q]
    r = _host(**qp_arrays(Ps, qs, [A] * 3, np.tile(l, (3, 1)), np.tile(u, (3, 1))))
    for b in range(3):
        xo, _ = oracle_solve(Ps[b], qs[b], A, l, u)
        np.testing.assert_allclose(r["x"][b], xo, atol=X_TOL * max(1, np.abs(xo).max()))


def test_host_build_window_and_in_lds_factorisations_agree():
    """Small batches factor the band in place in LDS, batches of more problems than CUs stream it
    through the ring window; both apply every column's updates in the same order, so a problem
    gets the same numbers either way (the host build runs both column-at-a-time kernels)."""
    rng = np.random.default_rng(8)
    P, q, A, l, u = random_qp(18, 24, 3, 4, rng)
    B = 260   # > 256 CUs of the analysis default: the window path
    qs = q[None, :] + 0.1 * rng.normal(size=(B, len(q)))
    big = _host(**qp_arrays([P] * B, qs, [A] * B, np.tile(l, (B, 1)), np.tile(u, (B, 1))))
    for b in (0, 131, B - 1):
        one = _host(**qp_arrays(P, qs[b], A, l, u))
        assert big["status"][b] == one["status"][0] == 1
        np.testing.assert_array_equal(big["x"][b], one["x"][0])
        np.testing.assert_array_equal(big["iters"][b], one["iters"][0])


def belief_problems():
    for name in ("belief_m1", "belief_m2"):
        g = golden(name)
        for t in (int(k) for k in g["keep"]):
            p = f"s{t}_"
            sol = g["traj_sol"][t]
            yield name, t, coo(g, p + "P"), g[p + "q"], coo(g, p + "A"), g[p + "l"], g[p + "u"], sol[~np.isnan(sol)]


def test_host_build_solves_reference_belief_problems():
    """The QPs the reference's PredictiveControllers.MPC handed to OSQP: same optimum as the
    oracle run behind the reference (recorded), narrow band after the ordering."""
    for name, t, P, q, A, l, u, sol in belief_problems():
        r = _host(**qp_arrays(P, q, A, l, u))
        assert r["status"][0] == 1, (name, t)
        np.testing.assert_allclose(r["x"][0], sol, atol=1e-7 * max(1, np.abs(sol).max()), err_msg=f"{name} s{t}")
        nk, bw = r["info"][:2]
        assert bw < 40 and nk > 4 * bw, (name, t, nk, bw)     # an MPC's stage structure: a narrow band


def test_analysis_rejects_bad_input():
    import hostsim_lib as H
    rng = np.random.default_rng(2)
    P, q, A, l, u = random_qp(6, 4, 1, 0, rng)
    a = qp_arrays(P, q, A, l, u)
    Pl = sp.csc_matrix(np.tril(P))           # lower-triangular entries are not OSQP's form
    Pl.sort_indices()
    with pytest.raises(RuntimeError, match="upper triangular"):
        H.qp_solve(6, 4, Pl.indptr, Pl.indices, a["Ap"], a["Ai"], Pl.data, q, a["Ax"], l, u)
    # a row that is an equality in one problem and an inequality in another
    l2, u2 = np.tile(l, (2, 1)), np.tile(u, (2, 1))
    l2[1, 0] = u2[1, 0] - 1.0
    b = qp_arrays([P, P], [q, q], [A, A], l2, u2)
    with pytest.raises(RuntimeError, match="classified differently"):
        _host(**b)
    with pytest.raises(RuntimeError, match="l > u"):
        _host(**qp_arrays(P, q, A, u + 1.0, u))
    # a dense 200-variable P: bandwidth 199 does not fit the LDS window
    Pd = np.eye(200) + 0.01
    with pytest.raises(RuntimeError, match="LDS"):
        _host(**qp_arrays(Pd, np.ones(200), np.zeros((0, 200)), np.zeros(0), np.zeros(0)))


# ---- libbmpc.so on the GPU -------------------------------------------------------------------
@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from bmpc import plan
    plan.context(0)
    return plan


@pytest.mark.gpu
def test_gpu_matches_oracle_on_random_qps(gpu):
    rng = np.random.default_rng(11)
    for n, m, meq, ntwo, nfree in CASES:
        P, q, A, l, u = random_qp(n, m, meq, ntwo, rng, nfree)
        r = gpu.qp_solve(P, q, A, l, u)
        xo, _ = oracle_solve(P, q, A, l, u)
        assert r["status"][0] == 1
        np.testing.assert_allclose(r["x"][0], xo, atol=X_TOL * max(1, np.abs(xo).max()))
        check_kkt(P, q, A, l, u, r["x"][0], r["y"][0])


@pytest.mark.gpu
def test_gpu_batch_and_belief_problems(gpu):
    rng = np.random.default_rng(3)
    P, q, A, l, u = random_qp(30, 40, 4, 5, rng)
    B = 96
    scales = rng.uniform(0.5, 2.0, B)
    qs = rng.normal(size=(B, 30))
    r = gpu.qp_solve([P * s for s in scales], qs, [A] * B, np.tile(l, (B, 1)), np.tile(u, (B, 1)))
    assert np.all(r["status"] == 1)
    for b in (0, 17, B - 1):
        xo, _ = oracle_solve(P * scales[b], qs[b], A, l, u)
        np.testing.assert_allclose(r["x"][b], xo, atol=X_TOL * max(1, np.abs(xo).max()))
    for name, t, P, q, A, l, u, sol in belief_problems():
        r = gpu.qp_solve(P, q, A, l, u)
        assert r["status"][0] == 1, (name, t)
        np.testing.assert_allclose(r["x"][0], sol, atol=1e-7 * max(1, np.abs(sol).max()), err_msg=f"{name} s{t}")


@pytest.mark.gpu
def test_gpu_large_batch_window_path_and_cache(gpu):
    """More problems than CUs (the factor streamed through the LDS window, in the workspace) and
    repeated calls on one pattern (the cached analysis): solutions equal the oracle's, and a
    call whose bounds classify the rows differently gets an analysis of its own."""
    rng = np.random.default_rng(5)
    P, q, A, l, u = random_qp(24, 30, 3, 4, rng)
    B = 300
    qs = q[None, :] + 0.1 * rng.normal(size=(B, len(q)))
    for rep in range(2):   # the second call hits the cache
        r = gpu.qp_solve([P] * B, qs, [A] * B, np.tile(l, (B, 1)), np.tile(u, (B, 1)))
        assert np.all(r["status"] == 1), rep
        for b in (0, 150, B - 1):
            xo, _ = oracle_solve(P, qs[b], A, l, u)
            np.testing.assert_allclose(r["x"][b], xo, atol=X_TOL * max(1, np.abs(xo).max()))
    u2 = u.copy()
    fin = np.where(np.isfinite(u2) & np.isfinite(l) & (u2 > l))[0]
    u2[fin[0]] = np.inf   # a two-sided row becomes one-sided: another row class
    r = gpu.qp_solve(P, q, A, l, u2)
    xo, _ = oracle_solve(P, q, A, l, u2)
    assert r["status"][0] == 1
    np.testing.assert_allclose(r["x"][0], xo, atol=X_TOL * max(1, np.abs(xo).max()))
