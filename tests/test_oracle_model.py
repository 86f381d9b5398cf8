"""Pin the oracle's model restatement: the reference's CasADi graphs cannot run here
(casadi absent), so the NumPy restatement is checked against (1) sympy-exact
derivatives of the same SX-branch expressions and (2) central finite differences."""
import numpy as np
import pytest
import sympy as sp

from oracle.model import (BRAKE, LC, MAINTAIN, HighwayModel, Policy, QuadrupedModel, highway_policies,
                          quadruped_policies)


def sym_highway(N, dt, pols, L=4.0, W=2.5, s1=2.0, N_lane=3):
    """sympy transcription of calc_xp_expr (highway_branch_dyn.py:363-398), SX branches."""
    x = sp.symbols("x0:4", real=True)
    z = sp.symbols("z0:4", real=True)

    def f(s, u):
        return [s[2] * sp.cos(s[3]), s[2] * sp.sin(s[3]), u[0], u[1]]

    def pol(p, s):
        if p.kind == MAINTAIN:
            return [sp.Integer(0), -p.params[0] * s[3]]
        if p.kind == BRAKE:
            e1, e2 = sp.exp(5 * -7), sp.exp(5 * -s[2])
            return [(e1 * -7 + e2 * -s[2]) / (e1 + e2), -p.params[0] * s[3]]
        t = p.params
        return [-0.8558 * (s[2] - t[2]), -0.3162 * (s[1] - t[1]) - 3.9889 * (s[3] - t[3])]

    def roll(s, p):
        out = []
        for _ in range(N):
            fu = f(s, pol(p, s))
            s = [s[i] + fu[i] * dt for i in range(4)]
            out.append(s)
        return out

    def smin(v, g):
        return sum(sp.exp(-g * a) * a for a in v) / sum(sp.exp(-g * a) for a in v)

    def vcol(a, b, size):
        dx = sp.Abs(a[0] - b[0]) - size[0]
        dy = sp.Abs(a[1] - b[1]) - size[1]
        return (dx * sp.exp(dx) + dy * sp.exp(dy)) / (sp.exp(dx) + sp.exp(dy))

    lb, ub = W / 2, N_lane * 3.6 - W / 2
    x1 = roll(list(x), pols[0])
    hi = []
    for p in pols:
        x2 = roll(list(z), p)
        h = [vcol(x2[k], x1[k], [L + 2, W + 0.2]) for k in range(N)]
        h += [smin([x2[k][1] - lb, ub - x2[k][1]], 5) for k in range(N)]
        hi.append(smin(h, 5))
    mm = [sp.exp(s1 * ((sp.exp(h) - 1) / (sp.exp(h) + 1) * 0.5 + 0.5)) for h in hi]
    p = [v / sum(mm) for v in mm]
    hcol = vcol(x, z, [L + 1, W + 0.2])
    return x, z, p, hcol


@pytest.mark.parametrize("seed", [0])
def test_highway_branch_prob_and_collision_vs_sympy(seed):
    rng = np.random.default_rng(seed)
    N, dt = 2, 0.1
    pols = highway_policies(0.1, [0, 5.4, 20, 0])
    m = HighwayModel(N, dt, pols)
    xs, zs, p, hcol = sym_highway(N, dt, pols)
    args = list(xs) + list(zs)
    fp = sp.lambdify(args, p, "math", cse=True)
    fdp = sp.lambdify(args, [sp.diff(p[0], xj) for xj in xs], "math", cse=True)   # row 0 (cost)
    fh = sp.lambdify(args, hcol, "math")
    fdh = sp.lambdify(args, [sp.diff(hcol, xj) for xj in xs], "math")
    for _ in range(3):
        xv = np.array([rng.uniform(-3, 3), rng.uniform(1, 6), rng.uniform(15, 25), rng.normal(0, .05)])
        zv = xv + np.array([rng.uniform(2, 15), rng.uniform(-4, 4), rng.uniform(-3, 3), 0.0])
        a = list(xv) + list(zv)
        pv, dpv = m.branch_eval(xv, zv)
        np.testing.assert_allclose(pv, fp(*a), atol=1e-13)
        np.testing.assert_allclose(dpv[0], np.array(fdp(*a)), atol=1e-11)
        h0, dh = m.col_eval(xv, zv)
        dhs = np.array(fdh(*a))
        np.testing.assert_allclose(dh, dhs, atol=1e-13)
        assert abs(h0 - (fh(*a) - dhs @ xv)) < 1e-12


def test_highway_linearization_vs_sympy_and_fd():
    m = HighwayModel(20, 0.1, highway_policies(0.1, [0, 1.8, 20, 0]))
    x = sp.symbols("x0:4", real=True)
    u = sp.symbols("u0:2", real=True)
    xp = [x[0] + x[2] * sp.cos(x[3]) * 0.1, x[1] + x[2] * sp.sin(x[3]) * 0.1, x[2] + u[0] * 0.1, x[3] + u[1] * 0.1]
    xv, uv = np.array([1.0, 2.0, 18.0, 0.07]), np.array([0.5, -0.1])
    A, B, C, xpv = m.dyn_linearization(xv, uv)
    sub = {**dict(zip(x, xv)), **dict(zip(u, uv))}
    As = np.array([[float(sp.diff(e, v).subs(sub)) for v in x] for e in xp])
    Bs = np.array([[float(sp.diff(e, v).subs(sub)) for v in u] for e in xp])
    np.testing.assert_allclose(A, As, atol=1e-15)
    np.testing.assert_allclose(B, Bs, atol=1e-15)
    np.testing.assert_allclose(C, xpv - A @ xv - B @ uv, atol=1e-14)


def test_branch_eval_central_differences():
    m = HighwayModel(20, 0.1, highway_policies(0.1, [0, 5.4, 20, 0]))
    x, z = np.array([0.0, 1.8, 20.0, 0.01]), np.array([5.0, 5.4, 20.0, 0.0])
    p, dp = m.branch_eval(x, z)
    assert abs(p.sum() - 1) < 1e-14
    for j in range(4):
        e = np.zeros(4)
        e[j] = 1e-6
        fd = (m.branch_eval(x + e, z)[0] - m.branch_eval(x - e, z)[0]) / 2e-6
        np.testing.assert_allclose(dp[:, j], fd, atol=1e-7)


def test_quadruped_vs_finite_differences():
    m = QuadrupedModel(25, 0.2, quadruped_policies(0.2))
    x, z = np.array([0.0, 1.8, 0.1]), np.array([2.5, 2.5, -np.pi / 2])
    p, dp = m.branch_eval(x, z)
    for j in range(3):
        e = np.zeros(3)
        e[j] = 1e-6
        fd = (m.branch_eval(x + e, z)[0] - m.branch_eval(x - e, z)[0]) / 2e-6
        np.testing.assert_allclose(dp[:, j], fd, atol=1e-7)
    h0, dh = m.col_eval(x, z)
    np.testing.assert_allclose(dh, [np.sign(x[0] - z[0]), np.sign(x[1] - z[1]), 0.0])
    zp = m.zpred_eval(z)
    assert zp.shape == (25, 6)
    np.testing.assert_allclose(zp[:, 3:], np.tile(z, (25, 1)))   # stop policy keeps the obstacle


def test_brake_policy_uses_sx_constants():
    """backup_brake SX branch = softmax([-7,-v],5) (highway_branch_dyn.py:117), not (-5,3)."""
    from oracle.model import policy_u
    u = policy_u(Policy(BRAKE, (0.1,)), [0, 0, 3.0, 0.2])
    e1, e2 = np.exp(-35.0), np.exp(-15.0)
    assert abs(u[0] - (e1 * -7 + e2 * -3) / (e1 + e2)) < 1e-15
    assert abs(u[1] + 0.02) < 1e-15
    lc = policy_u(Policy(LC, (0, 5.4, 20, 0)), [0, 1.8, 18.0, 0.1])
    assert abs(lc[0] - (-0.8558 * (18 - 20))) < 1e-15
