// bmpc_env.h -- the closed-loop highway overtake scene, one scene per ego.
//
// Restates Highway_env_branch.Highway_env.step (Highway_env_branch.py:83-184) and the
// collision rule of Highway_sim (:421-429) for the two-vehicle sim_overtake scene
// (:719-725); oracle/env.py is its CPU oracle.  One env_step_ego advances one ego's scene
// by one control step around the controller solve:
//   post(t-1): Euler step of the ego with uPred[0] of the last solve and of the obstacle with
//              the backup input chosen at t-1 (vehicle.step :39-41, used at :170-182);
//   collision: Highway_sim's sticky flag, tested before env.step(t) (:421-429);
//   pre(t):    the obstacle's backup choice -- argmax over the model's backup rollouts of the
//              clipped NumPy veh_col / lane_bdry_h safety value (:137-149) --, the lane
//              bookkeeping with the update_backup re-targeting of the lane-change policy
//              (:93-118), and the x_ref rule (:153-167): the inputs of the next solve.
// The obstacle's input uses the env's construction-time backup list (NumPy branches, :60,
// :149); the rollouts use the model's list as it was before this step's update (SX
// branches, zpred_eval at :95 precedes update_backup at :118).
#pragma once

#include "bmpc_model.h"

namespace bmpc {

// per-ego scene state (doubles), resident on the device between steps
enum {
  ENV_X = 0,        // ego state (X, Y, v, psi)
  ENV_Z = 4,        // obstacle state
  ENV_UOBS = 8,     // obstacle input chosen by pre(t), applied by post(t)
  ENV_LANE0 = 10,   // laneidx of the ego / of the obstacle (:96-101)
  ENV_LANE1 = 11,
  ENV_COLL = 12,    // Highway_sim collision flag (sticky)
  ENV_OBSPOL = 13,  // obstacle backup index chosen by the last pre()
  ENV_STEPS = 14,   // control steps taken
  ENV_STRIDE = BMPC_ENV_STRIDE
};

// per-ego closed-loop statistics (doubles, accumulated over the steps)
enum {
  ENVS_J = 0, ENVS_J2, ENVS_INFEAS, ENVS_ITERS, ENVS_SOLVES, ENVS_COLL_STEPS, ENVS_COLLIDED,
  ENVS_STRIDE = BMPC_ENV_NSTAT
};

// NumPy veh_col (highway_branch_dyn.py:243-254): rows clipped to +-5, alpha = 1
BMPC_HD double env_veh_col(double a0, double a1, double b0, double b1, double s0, double s1) {
  const double dx = fmin(fmax(fabs(a0 - b0) - s0, -5.0), 5.0);
  const double dy = fmin(fmax(fabs(a1 - b1) - s1, -5.0), 5.0);
  const double ex = exp(dx), ey = exp(dy);
  return (dx * ex + dy * ey) / (ex + ey);
}

// NumPy lane_bdry_h (highway_branch_dyn.py:195-214): softmin_5([y - lb, ub - y])
BMPC_HD double env_lane_bdry(double y, double lb, double ub) {
  const double a = y - lb, b = ub - y;
  const double ea = exp(-5.0 * a), eb = exp(-5.0 * b);
  return (ea * a + eb * b) / (ea + eb);
}

// NumPy branches of the env's backup list (highway_branch_dyn.py:67, :121, :148)
BMPC_HD void env_policy_u(int kind, const double* x, double Kpsi, const double* target, double* u) {
  if (kind == 0) {
    u[0] = 0.0;
    u[1] = -Kpsi * x[3];
  } else if (kind == 1) {   // softmax([-5, -v], 3)
    const double a = -5.0, b = -x[2];
    const double ea = exp(3.0 * a), eb = exp(3.0 * b);
    u[0] = (ea * a + eb * b) / (ea + eb);
    u[1] = -Kpsi * x[3];
  } else {
    u[0] = -0.8558 * (x[2] - target[2]);
    u[1] = -0.3162 * (x[1] - target[1]) - 3.9889 * (x[3] - target[3]);
  }
}

// One scene step of one ego (see the header comment).  st: ENV_STRIDE doubles; pol: the
// ego's m model policies (the lane-change target is re-targeted in place, update_backup);
// u0: uPred[0] of the last solve (unused at t == 0); x_out, z_out, xref_out: the next
// solve's inputs.
BMPC_HD void env_step_ego(const bmpc_env_desc& E, double dt, int N, int m, int t, double* st,
                          bmpc_policy* pol, const double* u0, double* x_out, double* z_out,
                          double* xref_out) {
  double* x = st + ENV_X;
  double* z = st + ENV_Z;
  if (t > 0) {   // post(t-1): vehicle.step of ego and obstacle
    double xp[4], zp[4];
    step<Highway>(dt, x, u0, xp);
    step<Highway>(dt, z, st + ENV_UOBS, zp);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = xp[i], z[i] = zp[i];
  }
  if (st[ENV_COLL] == 0.0) {   // Highway_sim, before env.step(t)
    const double dis = fmax(fabs(x[0] - z[0]) - E.vlen, fabs(x[1] - z[1]) - E.vwid);
    if (dis < 0.0) st[ENV_COLL] = 1.0;
  }
  // safety value of every obstacle backup against the ego's backup-0 rollout (the ego's
  // backupidx is never changed): min over the rows of veh_col and lane_bdry_h of the ego
  const double s0 = E.L + 1.0, s1 = E.W + 0.2;
  const double lb = E.W / 2.0, ub = E.n_lane * 3.6 - E.W / 2.0;
  double hi[BMPC_MAX_M], zo[BMPC_MAX_M][4], xe[4];
  double lane_min = 1e300;
#pragma unroll
  for (int i = 0; i < 4; ++i) xe[i] = x[i];
  for (int j = 0; j < m; ++j) {
    hi[j] = 1e300;
#pragma unroll
    for (int i = 0; i < 4; ++i) zo[j][i] = z[i];
  }
  for (int k = 0; k < N; ++k) {
    double ue[2], fe[4];
    Highway::policy(pol[0], xe, ue);
    Highway::f(xe, ue, fe);
#pragma unroll
    for (int i = 0; i < 4; ++i) xe[i] = xe[i] + fe[i] * dt;
    lane_min = fmin(lane_min, env_lane_bdry(xe[1], lb, ub));
    for (int j = 0; j < m; ++j) {
      double uo[2], fo[4];
      Highway::policy(pol[j], zo[j], uo);
      Highway::f(zo[j], uo, fo);
#pragma unroll
      for (int i = 0; i < 4; ++i) zo[j][i] = zo[j][i] + fo[i] * dt;
      hi[j] = fmin(hi[j], env_veh_col(xe[0], xe[1], zo[j][0], zo[j][1], s0, s1));
    }
  }
  int best = 0;
  for (int j = 0; j < m; ++j) {
    hi[j] = fmin(hi[j], lane_min);
    if (hi[j] > hi[best]) best = j;   // np.argmax: the first maximum
  }
  // lane bookkeeping (Python round = half to even = rint) and update_backup re-targeting
  for (int i = 0; i < 2; ++i) {
    const double* v = i == 0 ? x : z;
    const double nl = rint((v[1] - 1.8) / 3.6);
    double& lane = st[ENV_LANE0 + i];
    if (t == 0 || (nl != lane && fabs(v[1] - 1.8 - 3.6 * nl) < 1.4)) {
      lane = nl;
      if (i == 1) {
        const double l0 = st[ENV_LANE0], l1 = st[ENV_LANE1];
        const double tl = l0 < l1 ? l1 - 1.0 : l0 > l1 ? l1 + 1.0 : l1 > 0.0 ? l1 - 1.0 : l1 + 1.0;
        for (int j = 0; j < m; ++j)
          if (pol[j].kind == BMPC_POL_LC) {
            pol[j].p[0] = 0.0;
            pol[j].p[1] = 1.8 + 3.6 * tl;
            pol[j].p[2] = E.v0;
            pol[j].p[3] = 0.0;
          }
      }
    }
  }
  st[ENV_OBSPOL] = (double)best;
  env_policy_u(best, z, E.Kpsi, E.target, st + ENV_UOBS);
  // x_ref rule (:153-167)
  const double Ydes = x[0] < z[0] ? 1.8 + st[ENV_LANE0] * 3.6 : z[1];
  const double vdes = (fabs(x[1] - Ydes) < 1.0 && x[0] > z[0] + 3.0) ? E.v0 : z[2] + (z[0] + 1.5 - x[0]);
#pragma unroll
  for (int i = 0; i < 4; ++i) x_out[i] = x[i], z_out[i] = z[i];
  xref_out[0] = 0.0;
  xref_out[1] = Ydes;
  xref_out[2] = vdes;
  xref_out[3] = 0.0;
  st[ENV_STEPS] += 1.0;
}

// statistics of the last solve and of the scene (bench / closed-loop summaries)
BMPC_HD void env_accumulate(const double* st, double J, int status, int iters, bool cvar, double* acc) {
  acc[ENVS_J] += J;
  acc[ENVS_J2] += J * J;
  acc[ENVS_INFEAS] += (cvar ? status < 0 : status != 1) ? 1.0 : 0.0;
  acc[ENVS_ITERS] += (double)iters;
  acc[ENVS_SOLVES] += 1.0;
  acc[ENVS_COLL_STEPS] += st[ENV_COLL];
  acc[ENVS_COLLIDED] = st[ENV_COLL];
}

}  // namespace bmpc
