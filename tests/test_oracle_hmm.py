"""Pin the oracle's HMM belief-model restatement (oracle/hmm.py; reference module
HMM_backup_dyn.py is text-only): sympy-exact Jacobians of a transcription
of calc_xp_expr (:238-276), and central differences for a larger belief."""
import numpy as np
import sympy as sp

from oracle.hmm import HMMModel


def sym_hmm(M, m, dt, xbackup, L=4.0, W=2.5, ylb=0.0, yub=7.2, col_alpha=5.0, s1=2.0, tau=0.3):
    nb = 4 + M * m
    xb = sp.symbols(f"xb0:{nb}", real=True)
    u = sp.symbols("u0:2", real=True)
    x = xb[0:4]
    b = [[xb[4 + j * M + i] for j in range(m)] for i in range(M)]

    def smin(a, c, g):
        return (sp.exp(-g * a) * a + sp.exp(-g * c) * c) / (sp.exp(-g * a) + sp.exp(-g * c))

    xp = [x[0] + x[2] * sp.cos(x[3]) * dt, x[1] + x[2] * sp.sin(x[3]) * dt, x[2] + u[0] * dt, x[3] + u[1] * dt]
    size = [L + 1, W + 0.2]
    hs, bp = [], [[None] * m for _ in range(M)]
    for i in range(M):
        h = []
        for j in range(m):
            xr = xbackup[m * i + j]
            dx = (sp.Abs(x[0] - xr[0]) - size[0]) / size[0]
            dy = (sp.Abs(x[1] - xr[1]) - size[1]) / size[1]
            vc = (dx * sp.exp(dx) + dy * sp.exp(dy)) / (sp.exp(dx) + sp.exp(dy))
            lb = smin(xr[1] - ylb, yub - xr[1], 5)
            h.append(smin(vc, lb, col_alpha))
        hs.append(h)
        ms = [(sp.exp(s1 * hj) - 1) / (sp.exp(s1 * hj) + 1) * 0.5 + 0.5 for hj in h]
        tot = sum(ms)
        for c in range(m):
            bp[i][c] = sum(b[i][r] * ((1 - tau) * ms[c] / tot + (tau if r == c else 0)) for r in range(m))
    xbp = xp + [bp[i][j] for j in range(m) for i in range(M)]
    return xb, u, xbp, hs


def test_hmm_linearization_vs_sympy():
    rng = np.random.default_rng(0)
    M, m, dt = 1, 2, 0.1
    xbackup = np.array([[6.0, 5.4, 18.0, 0.0], [3.0, 1.9, 15.0, 0.0]])
    xb_s, u_s, xbp, hs = sym_hmm(M, m, dt, xbackup)
    args = list(xb_s) + list(u_s)
    fA = sp.lambdify(args, sp.Matrix(xbp).jacobian(sp.Matrix(xb_s)).tolist(), "math")
    fB = sp.lambdify(args, sp.Matrix(xbp).jacobian(sp.Matrix(u_s)).tolist(), "math")
    fx = sp.lambdify(args, xbp, "math")
    fJ = sp.lambdify(args, sp.Matrix(hs[0]).jacobian(sp.Matrix(xb_s)).tolist(), "math")
    fh = sp.lambdify(args, hs[0], "math")
    mdl = HMMModel(M, m, dt)
    for _ in range(3):
        xb = np.concatenate([[rng.uniform(-3, 3), rng.uniform(0, 7), rng.uniform(10, 25), rng.normal(0, .05)],
                             rng.dirichlet(np.ones(m))])
        u = np.array([rng.uniform(-3, 3), rng.uniform(-.2, .2)])
        A, B, C, h0, Jh, xv = mdl.linearize(xb, u, xbackup)
        a = list(xb) + list(u)
        np.testing.assert_allclose(A, np.array(fA(*a), float), atol=1e-13)
        np.testing.assert_allclose(B, np.array(fB(*a), float), atol=1e-13)
        np.testing.assert_allclose(xv, np.array(fx(*a), float), atol=1e-13)
        np.testing.assert_allclose(C, xv - A @ xb - B @ u, atol=1e-13)
        J = np.array(fJ(*a), float)
        np.testing.assert_allclose(Jh[0], J, atol=1e-13)
        np.testing.assert_allclose(h0[0], np.array(fh(*a), float) - J @ xb, atol=1e-12)


def test_hmm_central_differences_two_agents():
    rng = np.random.default_rng(1)
    M, m = 2, 3
    mdl = HMMModel(M, m, 0.1)
    xbackup = np.column_stack([rng.uniform(-5, 15, M * m), rng.uniform(0, 7, M * m),
                               rng.uniform(10, 25, M * m), np.zeros(M * m)])
    xb = np.concatenate([[0.5, 3.0, 20.0, 0.02], rng.dirichlet(np.ones(m), M).T.ravel()])
    u = np.array([0.5, -0.05])
    A, B, C, h0, Jh, xv = mdl.linearize(xb, u, xbackup)
    for k in range(mdl.nb):
        e = np.zeros(mdl.nb)
        e[k] = 1e-6
        fd = (mdl.linearize(xb + e, u, xbackup)[5] - mdl.linearize(xb - e, u, xbackup)[5]) / 2e-6
        np.testing.assert_allclose(A[:, k], fd, atol=1e-7)
    # belief rows stay stochastic: columns of the b block of A sum (over each agent) like H
    bp = xv[4:].reshape(m, M).T
    np.testing.assert_allclose(bp.sum(axis=1), xb[4:].reshape(m, M).T.sum(axis=1), atol=1e-12)


def _hmm_case(seed, M, m, B):
    rng = np.random.default_rng(seed)
    xbk = np.column_stack([rng.uniform(-5, 15, (B * M * m)), rng.uniform(0, 7, B * M * m),
                           rng.uniform(10, 25, B * M * m), np.zeros(B * M * m)]).reshape(B, M * m, 4)
    xb = np.column_stack([rng.uniform(-3, 3, B), rng.uniform(0, 7, B), rng.uniform(10, 25, B), rng.normal(0, .05, B),
                          np.stack([rng.dirichlet(np.ones(m), M).T.ravel() for _ in range(B)])])
    u = np.column_stack([rng.uniform(-3, 3, B), rng.uniform(-.2, .2, B)])
    return xb, u, xbk


HC = (0.1, 4.0, 2.5, 0.0, 7.2, 5.0, 2.0, 0.3)


def check_hmm_against_oracle(out, M, m, xb, u, xbk, tol=1e-12):
    mdl = HMMModel(M, m, HC[0], L=HC[1], W=HC[2], ylb=HC[3], yub=HC[4], col_alpha=HC[5], s1=HC[6], tran_diag=HC[7])
    for p in range(xb.shape[0]):
        A, B, C, h0, Jh, xv = mdl.linearize(xb[p], u[p], xbk[p])
        for got, ref in ((out["A"][p], A), (out["B"][p], B), (out["C"][p], C), (out["xbp"][p], xv),
                         (out["h0"][p], h0), (out["Jh"][p], Jh)):
            np.testing.assert_allclose(got, ref, rtol=tol, atol=tol)


def test_hmm_device_code_on_host():
    """csrc/bmpc_hmm.h compiled for the host (test-only build) vs the oracle."""
    import hostsim_lib as H
    for M, m in ((1, 3), (2, 3), (4, 4)):
        xb, u, xbk = _hmm_case(M * 10 + m, M, m, 16)
        check_hmm_against_oracle(H.hmm_eval(M, m, HC, xb, u, xbk), M, m, xb, u, xbk)
