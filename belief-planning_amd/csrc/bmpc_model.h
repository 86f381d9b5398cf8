// bmpc_model.h -- closed-form predictive models with forward-mode duals.
//
// Replaces the CasADi SX graphs of the reference (built in calc_xp_expr and evaluated
// through casadi.Function): highway_branch_dyn.py:363-398, quadruped_branch_dyn.py:218-248.
// SX-branch semantics are kept (see oracle/model.py for the quirk list).  Derivatives
// (A, B, dp/dx, dh/dx) come from dual numbers carried through the same expressions, so
// a lane needs no graph, no tape and no global memory.
#pragma once

#include "bmpc_core.h"

namespace bmpc {

template <int K>
struct Dual {
  double v;
  double g[K];
};

template <int K>
BMPC_HD Dual<K> dconst(double v) {
  Dual<K> r;
  r.v = v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = 0.0;
  return r;
}
template <int K>
BMPC_HD Dual<K> dvar(double v, int i) {
  Dual<K> r = dconst<K>(v);
  r.g[i] = 1.0;
  return r;
}
template <int K>
BMPC_HD Dual<K> operator+(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = a.g[i] + b.g[i];
  return r;
}
template <int K>
BMPC_HD Dual<K> operator-(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = a.g[i] - b.g[i];
  return r;
}
template <int K>
BMPC_HD Dual<K> operator-(const Dual<K>& a) {
  Dual<K> r;
  r.v = -a.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = -a.g[i];
  return r;
}
template <int K>
BMPC_HD Dual<K> operator*(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = a.g[i] * b.v + b.g[i] * a.v;
  return r;
}
template <int K>
BMPC_HD Dual<K> operator/(const Dual<K>& a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a.v / b.v;
  const double bb = b.v * b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = (a.g[i] * b.v - b.g[i] * a.v) / bb;
  return r;
}
template <int K>
BMPC_HD Dual<K> operator+(const Dual<K>& a, double b) {
  Dual<K> r = a;
  r.v = a.v + b;
  return r;
}
template <int K>
BMPC_HD Dual<K> operator+(double b, const Dual<K>& a) {
  return a + b;
}
template <int K>
BMPC_HD Dual<K> operator-(const Dual<K>& a, double b) {
  Dual<K> r = a;
  r.v = a.v - b;
  return r;
}
template <int K>
BMPC_HD Dual<K> operator-(double b, const Dual<K>& a) {
  Dual<K> r;
  r.v = b - a.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = -a.g[i];
  return r;
}
template <int K>
BMPC_HD Dual<K> operator*(const Dual<K>& a, double b) {
  Dual<K> r;
  r.v = a.v * b;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = a.g[i] * b;
  return r;
}
template <int K>
BMPC_HD Dual<K> operator*(double b, const Dual<K>& a) {
  return a * b;
}
template <int K>
BMPC_HD Dual<K> operator/(const Dual<K>& a, double b) {
  Dual<K> r;
  r.v = a.v / b;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = a.g[i] / b;
  return r;
}
template <int K>
BMPC_HD Dual<K> operator/(double a, const Dual<K>& b) {
  Dual<K> r;
  r.v = a / b.v;
  const double bb = b.v * b.v;
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = -a * b.g[i] / bb;
  return r;
}
template <int K>
BMPC_HD Dual<K> dexp(const Dual<K>& a) {
  Dual<K> r;
  r.v = exp(a.v);
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = a.g[i] * r.v;
  return r;
}
template <int K>
BMPC_HD Dual<K> dcos(const Dual<K>& a) {
  Dual<K> r;
  r.v = cos(a.v);
  const double s = -sin(a.v);
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = s * a.g[i];
  return r;
}
template <int K>
BMPC_HD Dual<K> dsin(const Dual<K>& a) {
  Dual<K> r;
  r.v = sin(a.v);
  const double c = cos(a.v);
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = c * a.g[i];
  return r;
}
template <int K>
BMPC_HD Dual<K> dfabs(const Dual<K>& a) {  // CasADi: d|x| = sign(x), sign(0) = 0
  Dual<K> r;
  r.v = fabs(a.v);
  const double sg = a.v > 0.0 ? 1.0 : (a.v < 0.0 ? -1.0 : 0.0);
#pragma unroll
  for (int i = 0; i < K; ++i) r.g[i] = sg * a.g[i];
  return r;
}
BMPC_HD double dexp(double a) { return exp(a); }
BMPC_HD double dcos(double a) { return cos(a); }
BMPC_HD double dsin(double a) { return sin(a); }
BMPC_HD double dfabs(double a) { return fabs(a); }
BMPC_HD double val(double a) { return a; }
template <int K>
BMPC_HD double val(const Dual<K>& a) {
  return a.v;
}
template <class S>
BMPC_HD S lift(double v) {
  return S(v);
}
template <>
BMPC_HD Dual<1> lift<Dual<1>>(double v) {
  return dconst<1>(v);
}
template <>
BMPC_HD Dual<3> lift<Dual<3>>(double v) {
  return dconst<3>(v);
}
template <>
BMPC_HD Dual<4> lift<Dual<4>>(double v) {
  return dconst<4>(v);
}
template <>
BMPC_HD Dual<6> lift<Dual<6>>(double v) {
  return dconst<6>(v);
}

// softmax over two values with gamma: sum(exp(g v) v) / sum(exp(g v))  (SX branch, :158-162)
template <class S>
BMPC_HD S softmax2(const S& a, const S& b, double g) {
  S ea = dexp(a * g), eb = dexp(b * g);
  return (ea * a + eb * b) / (ea + eb);
}
template <class S>
BMPC_HD S softmin2(const S& a, const S& b, double g) {
  S ea = dexp(a * (-g)), eb = dexp(b * (-g));
  return (ea * a + eb * b) / (ea + eb);
}

// ------------------------------------------------------------------------------------
// Lane reference of the psiref-tracking backups: casadi.interpolant(name, 'linear', [grid],
// values) (main_branch.py:78-82), linear on each grid cell, the end cells extended beyond the
// grid.  The cell of t is the last grid point <= t, clamped to [0, n-2].
// ------------------------------------------------------------------------------------
struct LaneRef {
  const double* g;   // grid (increasing), n points
  const double* v;   // values at the grid points
  int n;             // 0: no reference
};

BMPC_HD int lref_cell(const LaneRef& R, double t) {
  int lo = 0, hi = R.n - 1;   // invariant: g[lo] <= t < g[hi] once clamped
  if (!(t >= R.g[1])) return 0;
  if (t >= R.g[R.n - 2]) return R.n - 2;
  lo = 1;
  hi = R.n - 2;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (R.g[mid] <= t) lo = mid;
    else hi = mid;
  }
  return lo;
}

// psiref(t): v_i + (t - g_i) / (g_{i+1} - g_i) * (v_{i+1} - v_i); its derivative is the cell's
// slope (exact on each cell, as CasADi's linear plugin)
template <class S>
BMPC_HD S lref_eval(const LaneRef& R, const S& t) {
  const int i = lref_cell(R, val(t));
  const double g0 = R.g[i], g1 = R.g[i + 1], v0 = R.v[i], v1 = R.v[i + 1];
  return (t - g0) / (g1 - g0) * (v1 - v0) + v0;
}

// ------------------------------------------------------------------------------------
// Highway: x = (X, Y, v, psi), u = (a, r)           highway_branch_dyn.py:17-398
// ------------------------------------------------------------------------------------
struct Highway {
  static constexpr int NX = 4, NU = 2;
  static constexpr bool kTransform = false;   // no per-ego S / bx (see HighwayMerge)

  template <class S, class T>
  BMPC_HD static void f(const S* x, const T* u, S* xd) {  // dubin (:17-34)
    xd[0] = x[2] * dcos(x[3]);
    xd[1] = x[2] * dsin(x[3]);
    xd[2] = lift<S>(0.0) + u[0];
    xd[3] = lift<S>(0.0) + u[1];
  }

  // backup policy inputs, SX branches (:54-67, :108-119, :136-146, :80-88); the psiref
  // kinds follow the MX branches of the same functions (:66-77, :89-96, :122-130) with
  // psiref(X) from the lane reference R
  template <class S>
  BMPC_HD static void policy(const bmpc_policy& p, const S* x, S* u, const LaneRef& R = LaneRef{}) {
    switch (p.kind) {
      case BMPC_POL_MAINTAIN_PSIREF:
        u[0] = lift<S>(0.0);
        u[1] = lref_eval(R, x[0]) - x[3] * p.p[0];
        break;
      case BMPC_POL_MAINTAIN_TRACKV_PSIREF:
        u[0] = (p.p[1] - x[2]) * 0.5;
        u[1] = lref_eval(R, x[0]) - x[3] * p.p[0];
        break;
      case BMPC_POL_BRAKE_PSIREF:
        u[0] = softmax2(lift<S>(-5.0), -x[2], 3.0);
        u[1] = lref_eval(R, x[0]) - x[3] * p.p[0];
        break;
      case BMPC_POL_MAINTAIN:
        u[0] = lift<S>(0.0);
        u[1] = x[3] * (-p.p[0]);
        break;
      case BMPC_POL_BRAKE:
        u[0] = softmax2(lift<S>(-7.0), -x[2], 5.0);
        u[1] = x[3] * (-p.p[0]);
        break;
      case BMPC_POL_LC:
        u[0] = (x[2] - p.p[2]) * (-0.8558);
        u[1] = (x[1] - p.p[1]) * (-0.3162) - (x[3] - p.p[3]) * 3.9889;
        break;
      case BMPC_POL_MAINTAIN_TRACKV:
        u[0] = (p.p[1] - x[2]) * 0.5;
        u[1] = x[3] * (-p.p[0]);
        break;
      default:
        u[0] = lift<S>(0.0);
        u[1] = lift<S>(0.0);
    }
  }

  // veh_col SX branch (:228-235), one row, no clipping
  template <class S>
  BMPC_HD static S veh_col(const S& a0, const S& a1, double b0, double b1, double s0, double s1) {
    S dx = dfabs(a0 - b0) - s0;
    S dy = dfabs(a1 - b1) - s1;
    S ex = dexp(dx), ey = dexp(dy);
    return (dx * ex + dy * ey) / (ex + ey);
  }
  template <class S>
  BMPC_HD static S veh_col(const S& a0, const S& a1, const S& b0, const S& b1, double s0, double s1) {
    S dx = dfabs(a0 - b0) - s0;
    S dy = dfabs(a1 - b1) - s1;
    S ex = dexp(dx), ey = dexp(dy);
    return (dx * ex + dy * ey) / (ex + ey);
  }

  // collision h of col_eval (:386): veh_col(x', z', [L+1, W+0.2], 1)
  template <class S>
  BMPC_HD static S col_h(const double* mc, const S* x, const double* z) {
    return veh_col(x[0], x[1], z[0], z[1], mc[0] + 1.0, mc[1] + 0.2);
  }

  // hi of one policy: BF_traj(obstacle rollout, ego rollout) (:337-349)
  //   h = [veh_col(obs_k, ego_k, [L+2, W+0.2]) k<N ; lane_bdry_h(obs_k, LB) k<N]; softmin_5
  // streamed in the same summation order as the SX graph.
  template <class S>
  BMPC_HD static S bf_traj(const double* mc, double dt, int N, const bmpc_policy& ego_pol,
                           const bmpc_policy& obs_pol, const S* x0, const double* z0, const LaneRef& R = LaneRef{}) {
    const double s0 = mc[0] + 2.0, s1 = mc[1] + 0.2;
    const double lb = mc[1] / 2.0, ub = mc[3] * 3.6 - mc[1] / 2.0;
    S xe[4], ue[2], fe[4];
    double zo[4], uo[2], fo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xe[i] = x0[i], zo[i] = z0[i];
    S num = lift<S>(0.0), den = lift<S>(0.0);
    for (int k = 0; k < N; ++k) {
      policy(ego_pol, xe, ue, R);
      f(xe, ue, fe);
#pragma unroll
      for (int i = 0; i < 4; ++i) xe[i] = xe[i] + fe[i] * dt;
      policy(obs_pol, zo, uo, R);
      f(zo, uo, fo);
#pragma unroll
      for (int i = 0; i < 4; ++i) zo[i] = zo[i] + fo[i] * dt;
      S h = veh_col(lift<S>(zo[0]), lift<S>(zo[1]), xe[0], xe[1], s0, s1);
      S e = dexp(h * (-5.0));
      num = num + e * h;
      den = den + e;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) zo[i] = z0[i];
    for (int k = 0; k < N; ++k) {
      policy(obs_pol, zo, uo, R);
      f(zo, uo, fo);
#pragma unroll
      for (int i = 0; i < 4; ++i) zo[i] = zo[i] + fo[i] * dt;
      const double h = softmin2(zo[1] - lb, ub - zo[1], 5.0);
      const double e = exp(h * (-5.0));
      num = num + e * h;
      den = den + e;
    }
    return num / den;
  }

  // branch_prob (:355-359): softsat(h,1) then exp(s1*.) normalised
  template <class S>
  BMPC_HD static S prob_weight(const double* mc, const S& h) {
    S e = dexp(h);
    S ss = (e - 1.0) / (e + 1.0) * 0.5 + 0.5;
    return dexp(ss * mc[2]);
  }
};

// ------------------------------------------------------------------------------------
// HighwayMerge: PredictiveModel_merge (highway_branch_dyn.py:400-502) as the merge scene's
// controller uses it (pred_model[0], main_branch.py:85-88: maintain_trackV(v0) / brake, no
// psiref): the highway dynamics, policies, collision row and branch probabilities, but
// BF_traj (:463-467) is softmin_5 over veh_col(obs_k, ego_k, [L+1, W+0.2]) alone -- no
// lane-boundary term.  Its plans carry a per-ego state transformation (kTransform).
// ------------------------------------------------------------------------------------
struct HighwayMerge : Highway {
  static constexpr bool kTransform = true;

  template <class S>
  BMPC_HD static S bf_traj(const double* mc, double dt, int N, const bmpc_policy& ego_pol,
                           const bmpc_policy& obs_pol, const S* x0, const double* z0, const LaneRef& R = LaneRef{}) {
    const double s0 = mc[0] + 1.0, s1 = mc[1] + 0.2;
    S xe[4], ue[2], fe[4];
    double zo[4], uo[2], fo[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xe[i] = x0[i], zo[i] = z0[i];
    S num = lift<S>(0.0), den = lift<S>(0.0);
    for (int k = 0; k < N; ++k) {
      policy(ego_pol, xe, ue, R);
      f(xe, ue, fe);
#pragma unroll
      for (int i = 0; i < 4; ++i) xe[i] = xe[i] + fe[i] * dt;
      policy(obs_pol, zo, uo, R);
      f(zo, uo, fo);
#pragma unroll
      for (int i = 0; i < 4; ++i) zo[i] = zo[i] + fo[i] * dt;
      S h = veh_col(lift<S>(zo[0]), lift<S>(zo[1]), xe[0], xe[1], s0, s1);
      S e = dexp(h * (-5.0));
      num = num + e * h;
      den = den + e;
    }
    return num / den;
  }
};

// HighwayT: the highway model in a plan that takes solve's S / Fx / bx (BMPC_PLAN_TRANSFORM;
// MPC_branch.py:2043-2057 accepts them for any model): same model functions, the per-ego
// transform path of the solver (kTransform).
struct HighwayT : Highway {
  static constexpr bool kTransform = true;
};

// ------------------------------------------------------------------------------------
// Quadruped: x = (X, Y, theta), u = (vx, vy, omega)   quadruped_branch_dyn.py:14-248
// ------------------------------------------------------------------------------------
struct Quadruped {
  static constexpr int NX = 3, NU = 3;
  static constexpr bool kTransform = false;

  template <class S, class T>
  BMPC_HD static void f(const S* x, const T* u, S* xd) {  // quad_kinetics (:14-27)
    S c = dcos(x[2]), s = dsin(x[2]);
    xd[0] = c * u[0] - s * u[1];
    xd[1] = s * u[0] + c * u[1];
    xd[2] = lift<S>(0.0) + u[2];
  }

  template <class S>
  BMPC_HD static void policy(const bmpc_policy& p, const S* x, S* u, const LaneRef& = LaneRef{}) {
    (void)x;
    u[0] = lift<S>(p.kind == BMPC_POL_FORWARD ? p.p[0] : 0.0);  // backup_forward/stop (:34-54)
    u[1] = lift<S>(0.0);
    u[2] = lift<S>(0.0);
  }

  // robot_col SX branch (:135-144): |dx| + |dy| - (L1+L2)/2 - tol   (mc = L1 W1 L2 W2 tol s1)
  template <class S, class T>
  BMPC_HD static S robot_col(const double* mc, const S& a0, const S& a1, const T& b0, const T& b1) {
    return dfabs(a0 - b0) + dfabs(a1 - b1) - ((mc[0] + mc[2]) / 2.0) - mc[4];
  }

  template <class S>
  BMPC_HD static S col_h(const double* mc, const S* x, const double* z) {
    return robot_col(mc, x[0], x[1], z[0], z[1]);
  }

  // BF_traj (:204-211): softmin_5 over robot_col(obs_k, ego_k)
  template <class S>
  BMPC_HD static S bf_traj(const double* mc, double dt, int N, const bmpc_policy& ego_pol,
                           const bmpc_policy& obs_pol, const S* x0, const double* z0, const LaneRef& R = LaneRef{}) {
    S xe[3], ue[3], fe[3];
    double zo[3], uo[3], fo[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) xe[i] = x0[i], zo[i] = z0[i];
    S num = lift<S>(0.0), den = lift<S>(0.0);
    for (int k = 0; k < N; ++k) {
      policy(ego_pol, xe, ue, R);
      f(xe, ue, fe);
#pragma unroll
      for (int i = 0; i < 3; ++i) xe[i] = xe[i] + fe[i] * dt;
      policy(obs_pol, zo, uo, R);
      f(zo, uo, fo);
#pragma unroll
      for (int i = 0; i < 3; ++i) zo[i] = zo[i] + fo[i] * dt;
      S h = robot_col(mc, lift<S>(zo[0]), lift<S>(zo[1]), xe[0], xe[1]);
      S e = dexp(h * (-5.0));
      num = num + e * h;
      den = den + e;
    }
    return num / den;
  }

  template <class S>
  BMPC_HD static S prob_weight(const double* mc, const S& h) {  // no softsat (:212-216)
    return dexp(h * mc[5]);
  }
};

// ------------------------------------------------------------------------------------
// model entry points used by the tree update and bmpc_model_eval
// ------------------------------------------------------------------------------------

// x+ = x + f(x,u) dt and its Jacobians (dyn_linearization, highway_branch_dyn.py:284-291)
template <class M>
BMPC_HD void linearize(double dt, const double* x, const double* u, double* A, double* B,
                       double* C, double* xp) {
  constexpr int NX = M::NX, NU = M::NU, K = NX + NU;
  Dual<K> xs[NX], us[NU], fx[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) xs[i] = dvar<K>(x[i], i);
#pragma unroll
  for (int i = 0; i < NU; ++i) us[i] = dvar<K>(u[i], NX + i);
  M::f(xs, us, fx);
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    Dual<K> r = xs[i] + fx[i] * dt;
    xp[i] = r.v;
    double ax = 0.0, bu = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      A[i * NX + j] = r.g[j];
      ax += r.g[j] * x[j];
    }
#pragma unroll
    for (int j = 0; j < NU; ++j) {
      B[i * NU + j] = r.g[NX + j];
      bu += r.g[NX + j] * u[j];
    }
    C[i] = (r.v - ax) - bu;  // C = xp - A@x - B@u
  }
}

template <class M>
BMPC_HD void step(double dt, const double* x, const double* u, double* xp) {
  constexpr int NX = M::NX;
  double f[NX];
  M::f(x, u, f);
#pragma unroll
  for (int i = 0; i < NX; ++i) xp[i] = x[i] + f[i] * dt;
}

// zpred column block of one policy: rows x_1..x_N of propagate_backup (:174-187)
template <class M>
BMPC_HD void rollout(double dt, int N, const bmpc_policy& pol, const double* z0, double* out,
                     int row_stride, const LaneRef& R = LaneRef{}) {
  constexpr int NX = M::NX, NU = M::NU;
  double z[NX], u[NU], f[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) z[i] = z0[i];
  for (int k = 0; k < N; ++k) {
    M::policy(pol, z, u, R);
    M::f(z, u, f);
#pragma unroll
    for (int i = 0; i < NX; ++i) z[i] = z[i] + f[i] * dt;
#pragma unroll
    for (int i = 0; i < NX; ++i) out[k * row_stride + i] = z[i];
  }
}

// branch_eval (:298-301): p[m] and dp[m][NX] at (x, z)
template <class M>
BMPC_HD void branch_eval(const double* mc, double dt, int N, int m, const bmpc_policy* pol,
                         const double* x, const double* z, double* p, double* dp, const LaneRef& R = LaneRef{}) {
  constexpr int NX = M::NX;
  Dual<NX> xs[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) xs[i] = dvar<NX>(x[i], i);
  Dual<NX> wts[BMPC_MAX_M];
  Dual<NX> sum = dconst<NX>(0.0);
  for (int i = 0; i < m; ++i) {
    Dual<NX> h = M::bf_traj(mc, dt, N, pol[0], pol[i], xs, z, R);
    wts[i] = M::prob_weight(mc, h);
  }
  for (int i = 0; i < m; ++i) sum = sum + wts[i];
  for (int i = 0; i < m; ++i) {
    Dual<NX> pi = wts[i] / sum;
    p[i] = pi.v;
    if (dp)
#pragma unroll
      for (int j = 0; j < NX; ++j) dp[i * NX + j] = pi.g[j];
  }
}

// col_eval (:322-325): h0 = h - dh.x, dh
template <class M>
BMPC_HD void col_eval(const double* mc, const double* x, const double* z, double* h0, double* dh) {
  constexpr int NX = M::NX;
  Dual<NX> xs[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) xs[i] = dvar<NX>(x[i], i);
  Dual<NX> h = M::col_h(mc, xs, z);
  double dot = 0.0;
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    dh[j] = h.g[j];
    dot += h.g[j] * x[j];
  }
  *h0 = h.v - dot;
}

}  // namespace bmpc
