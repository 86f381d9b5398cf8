// bmpc_plan.cpp -- host-side plan construction (see bmpc_plan.h).
#include <stdlib.h>
#include "bmpc_plan.h"

#include <algorithm>

#include <math.h>
#include <string.h>

#include <deque>

namespace bmpc {

namespace {

// symmetric PSD square root via Jacobi eigen-decomposition (scipy.linalg.sqrtm fallback of
// MPC_branch.py:1628-1631 when the Cholesky of a singular weight fails)
void sqrtm_sym(const double* A, int n, double* out) {
  double a[BMPC_MAX_N][BMPC_MAX_N], v[BMPC_MAX_N][BMPC_MAX_N];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      a[i][j] = A[i * n + j];
      v[i][j] = i == j ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 100; ++sweep) {
    double off = 0.0;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) off += a[i][j] * a[i][j];
    if (off < 1e-30) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        if (fabs(a[p][q]) < 1e-300) continue;
        const double th = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < n; ++k) {
          const double akp = a[k][p], akq = a[k][q];
          a[k][p] = c * akp - s * akq;
          a[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = a[p][k], aqk = a[q][k];
          a[p][k] = c * apk - s * aqk;
          a[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = v[k][p], vkq = v[k][q];
          v[k][p] = c * vkp - s * vkq;
          v[k][q] = s * vkp + c * vkq;
        }
      }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int k = 0; k < n; ++k) s += v[i][k] * sqrt(fmax(a[k][k], 0.0)) * v[j][k];
      out[i * n + j] = s;
    }
}

// W with W'W = M: chol(M)' if M is positive definite, else sqrtm(M) (MPC_branch.py:1628-1636)
void weight_root(const double* M, int n, double* W) {
  double L[BMPC_MAX_N][BMPC_MAX_N];
  bool ok = true;
  for (int i = 0; i < n && ok; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = M[i * n + j];
      for (int k = 0; k < j; ++k) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (!(s > 0.0)) {
          ok = false;
          break;
        }
        L[i][i] = sqrt(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
  if (ok) {
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) W[i * n + j] = j >= i ? L[j][i] : 0.0;   // L'
  } else {
    sqrtm_sym(M, n, W);
  }
}

}  // namespace

void HostPlan::point_tables(const int32_t* base) {
  size_t i = 0;
#define BMPC_TOPO_POINT_(n) plan.t.n = (gint*)(base + blob_off[i]), plan.toff[i] = (int)blob_off[i], ++i;
  BMPC_TOPO_FIELDS(BMPC_TOPO_POINT_)
#undef BMPC_TOPO_POINT_
  plan.ntab = (int)blob.size();
}

std::string build_plan(const bmpc_plan_desc& desc, HostPlan& hp) {
  Plan& P = hp.plan;
  memset(&P, 0, sizeof(P));
  P.desc = desc;
  const int n = desc.n, d = desc.d, N = desc.N, NB = desc.NB, m = desc.m;
  if (desc.controller != BMPC_CTRL_CVAR && desc.controller != BMPC_CTRL_PROX && desc.controller != BMPC_CTRL_QP &&
      desc.controller != BMPC_CTRL_ROBUST)
    return "unknown controller";
  const bool robust = desc.controller == BMPC_CTRL_ROBUST;
  if (desc.model == BMPC_MODEL_HIGHWAY || desc.model == BMPC_MODEL_HIGHWAY_MERGE) {
    if (n != 4 || d != 2) return "highway model needs n=4, d=2";
    if (desc.model == BMPC_MODEL_HIGHWAY_MERGE && desc.controller != BMPC_CTRL_CVAR)
      return "the merge model (state transformation S) is supported with the CVaR controller";
    if ((desc.flags & BMPC_PLAN_TRANSFORM) && desc.controller != BMPC_CTRL_CVAR)
      return "BMPC_PLAN_TRANSFORM (solve's S / Fx / bx) needs the CVaR controller";
  } else if (desc.model == BMPC_MODEL_QUADRUPED) {
    if (n != 3 || d != 3) return "quadruped model needs n=3, d=3";
    if (desc.flags & BMPC_PLAN_TRANSFORM) return "BMPC_PLAN_TRANSFORM is supported for the highway models";
  } else {
    return "unknown model";
  }
  if (N < 2 || NB < 1 || m < 1 || m > BMPC_MAX_M) return "need N >= 2, NB >= 1, 1 <= m <= 4";
  if (desc.nFx < 0 || desc.nFx > BMPC_MAX_FX || desc.nFu < 0 || desc.nFu > BMPC_MAX_FU)
    return "too many constraint rows";
  if (!(desc.dt > 0.0)) return "dt must be positive";
  // robustMPC: the QP is a chain (one leaf root branch of N*NB+1 nodes + terminal node); the
  // scenario tree only shapes the obstacle predictions (MPC_branch.py:1301-1302,1336-1360)
  const int NBt = robust ? 0 : NB;
  P.n = n, P.d = d, P.N = N, P.NB = NBt, P.m = m, P.nFx = desc.nFx, P.nFu = desc.nFu;
  P.zNB = NB;
  P.Ncol = 1;
  if (robust)
    for (int k = 0; k < NB; ++k) P.Ncol *= m;
  if (P.Ncol > 64) return "too many obstacle predictions (m^NB > 64)";
  P.Nc = desc.nFx + P.Ncol;
  if (P.desc.maxit <= 0) P.desc.maxit = 100;
  if (!(P.desc.feastol > 0)) P.desc.feastol = 1e-8;
  if (!(P.desc.abstol > 0)) P.desc.abstol = 1e-8;
  if (!(P.desc.reltol > 0)) P.desc.reltol = 1e-8;

  // ---- BFS topology (MPC_branch.inittree :1678-1747) ----------------------------------
  hp.br_depth = {0};
  hp.br_len = {robust ? N * NB + 1 : 1};
  hp.br_parent = {-1};
  hp.br_ndx = {0};
  hp.br_ndu = {0};
  hp.br_child0 = {-1};
  int cx = hp.br_len[0] + (NBt == 0 ? 1 : 0), cu = hp.br_len[0];   // root nodes (+ terminal if a leaf)
  std::deque<int> q{0};
  while (!q.empty()) {
    const int b = q.front();
    q.pop_front();
    if (hp.br_depth[b] >= NBt) continue;
    hp.br_child0[b] = (int)hp.br_depth.size();
    for (int i = 0; i < m; ++i) {
      const int c = (int)hp.br_depth.size();
      hp.br_depth.push_back(hp.br_depth[b] + 1);
      hp.br_len.push_back(N);
      hp.br_parent.push_back(b);
      hp.br_child0.push_back(-1);
      hp.br_ndx.push_back(cx);
      hp.br_ndu.push_back(cu);
      cx += hp.br_depth[c] == NBt ? N + 1 : N;
      cu += N;
      q.push_back(c);
    }
  }
  const int nbr = (int)hp.br_depth.size();
  P.T = cx, P.U = cu, P.nbranch = nbr;
  P.bdim = 0;
  for (int b = 0; b < nbr; ++b) P.bdim += hp.br_depth[b] < NBt;
  P.ncones = 1;
  for (int b = 0; b < nbr; ++b)
    if (hp.br_depth[b] < NBt) P.ncones += m;
  if (P.ncones > 32) return "too many cones (m^NB too large)";

  // ---- nodes ------------------------------------------------------------------------------
  const int T = P.T, U = P.U;
  hp.x_u.assign(T, -1);
  hp.x_srcu.assign(T, -1);
  hp.x_srcx.assign(T, -1);
  hp.x_cone.assign(T, -1);
  hp.x_conepos.assign(T, -1);
  hp.x_branch.assign(T, -1);
  hp.u_x.assign(U, -1);
  hp.u_cone.assign(U, -1);
  std::vector<int> level(T, 0);
  std::vector<std::vector<int>> succ(T);
  for (int b = 0; b < nbr; ++b) {
    const int len = hp.br_len[b], ndx = hp.br_ndx[b], ndu = hp.br_ndu[b];
    const bool leaf = hp.br_depth[b] == NBt;
    const int lvl0 = b == 0 ? 0 : 1 + (hp.br_depth[b] - 1) * N;
    for (int j = 0; j < len; ++j) {
      hp.x_u[ndx + j] = ndu + j;
      hp.u_x[ndu + j] = ndx + j;
      hp.x_branch[ndx + j] = b;
      level[ndx + j] = lvl0 + j;
      if (j > 0) {
        hp.x_srcu[ndx + j] = ndu + j - 1;
        hp.x_srcx[ndx + j] = ndx + j - 1;
        succ[ndx + j - 1].push_back(ndx + j);
      }
    }
    if (b > 0) {
      const int p = hp.br_parent[b];
      const int lx = hp.br_ndx[p] + hp.br_len[p] - 1, lu = hp.br_ndu[p] + hp.br_len[p] - 1;
      hp.x_srcu[ndx] = lu;
      hp.x_srcx[ndx] = lx;
      succ[lx].push_back(ndx);
    }
    if (leaf) {
      const int tn = ndx + len;
      hp.x_branch[tn] = b;
      hp.x_srcu[tn] = ndu + len - 1;
      hp.x_srcx[tn] = ndx + len - 1;
      level[tn] = lvl0 + len;
      succ[ndx + len - 1].push_back(tn);
    }
  }
  int maxlvl = 0;
  for (int k = 0; k < T; ++k) maxlvl = level[k] > maxlvl ? level[k] : maxlvl;
  P.nlevels = maxlvl + 1;
  hp.lvl_off.assign(P.nlevels + 1, 0);
  for (int k = 0; k < T; ++k) hp.lvl_off[level[k] + 1]++;
  for (int l = 0; l < P.nlevels; ++l) hp.lvl_off[l + 1] += hp.lvl_off[l];
  hp.lvl_nodes.assign(T, 0);
  {
    std::vector<int> fill(hp.lvl_off.begin(), hp.lvl_off.end() - 1);
    for (int k = 0; k < T; ++k) hp.lvl_nodes[fill[level[k]]++] = k;
  }
  hp.succ_off.assign(T + 1, 0);
  hp.succ.clear();
  for (int k = 0; k < T; ++k) {
    hp.succ_off[k] = (int)hp.succ.size();
    for (int c : succ[k]) hp.succ.push_back(c);
  }
  hp.succ_off[T] = (int)hp.succ.size();
  if (hp.succ.empty()) hp.succ.push_back(0);

  // ---- layouts (reference sol['x'] and row order) ----------------------------------------
  const int bd = P.bdim;
  P.oX = 0;
  P.oU = T * n;
  P.oRho = P.oU + U * d;
  P.oSig = P.oRho + bd;
  P.oMup = P.oRho + 2 * bd;
  P.oMum = P.oRho + bd * (2 + m);
  P.oS = P.oRho + bd * (2 * m + 2);
  P.oJ = P.oS + T * P.Nc;
  P.nv = P.oJ + 1;
  P.neq = T * n + bd;
  P.rFx = 0;
  P.rFu = T * P.Nc;
  P.rRisk = P.rFu + U * P.nFu;
  P.rPos = P.rRisk + bd * (2 * m + 1);
  P.nlp = P.rPos + T * P.Nc;
  P.ng = bd * (2 * m + 2) + 1;
  P.nsm = P.ng + bd + P.ncones;
  P.cgrp = 64;
  while (P.cgrp > 1 && P.cgrp * P.ncones > 64) P.cgrp >>= 1;

  // ---- cones (buildIneqConstr :1940-1984): children of non-leaf branches, then the root ----
  int row = P.nlp, k = 0;
  for (int b = 0; b < nbr; ++b) {
    if (hp.br_depth[b] >= NBt) continue;
    for (int i = 0; i < m; ++i) {
      const int c = hp.br_child0[b] + i;
      hp.cone_b.push_back(b);
      hp.cone_i.push_back(i);
      hp.cone_c.push_back(c);
      const int qd = 2 + N * n + N * d;
      hp.cone_q.push_back(qd);
      hp.cone_off.push_back(row);
      row += qd;
      for (int j = 0; j < N; ++j) {
        hp.x_cone[hp.br_ndx[c] + j] = k;
        hp.x_conepos[hp.br_ndx[c] + j] = j;
        hp.u_cone[hp.br_ndu[c] + j] = k;
      }
      ++k;
    }
  }
  hp.cone_b.push_back(-1);
  hp.cone_i.push_back(-1);
  hp.cone_c.push_back(-1);
  hp.cone_q.push_back(2 + d);
  hp.cone_off.push_back(row);
  hp.u_cone[0] = k;
  row += 2 + d;
  P.nrows = row;
  P.maxq = 0;
  for (int q : hp.cone_q) P.maxq = q > P.maxq ? q : P.maxq;
  // widen the cone groups (more rounds) until the widest cone fits the fused cone passes'
  // registers, 8 rows per lane (bmpc_ipm.h cone_regs): NB = 2 plans' 13 cones of 2 + N (n + d)
  // rows otherwise run the unfused chain of whole-vector passes
  while (P.cgrp < 64 && P.maxq > 8 * P.cgrp) P.cgrp <<= 1;
  if (desc.controller != BMPC_CTRL_CVAR) {
    // BranchMPCProx's / BranchMPC's OSQP vector z = [X | U | S] and rows [Fx-type | Fu | -S] (MPC_branch.py:185-370)
    P.oS = T * n + U * d;
    P.oRho = P.oSig = P.oMup = P.oMum = P.oS;   // no CVaR globals
    P.oJ = P.oS + T * P.Nc;     // (no J; keeps "oS..oJ" = slack range for shared loops)
    P.ncones = 0;
    P.nv = P.oJ;
    P.neq = T * n;
    P.rFx = 0;
    P.rFu = T * P.Nc;
    P.rRisk = P.rFu + U * P.nFu;
    P.rPos = P.rRisk;
    P.nlp = P.rPos + T * P.Nc;
    P.nrows = P.nlp;
    P.ng = 0;
    P.nsm = 0;
  }
  // LDS of the solver kernels (doubles): a 64-double reduction area, the tree-solve scratch
  // (CVaR IPM: the pre-pass slack terms, T * Nc doubles, while the whole stays within 9,984
  // bytes = 16 egos per CU), then the dense coupling system (matrix, pivots, rhs).  A lean-LDS
  // launch (bmpc_hip.hip, choose_lds_rich) keeps only the part before the coupling system and
  // finds the system in the slab (Layout::coup) -- deep trees, whose 50 x 50 system would
  // otherwise leave 7 egos per CU.
  // (matrix, pivots and the two right-hand sides of a paired back half)
  const int ncoup = P.nsm * P.nsm + 3 * P.nsm;
  // the first area holds W1 and Wu (filled at kernel start; the IPM's cone passes index their
  // rows per lane), at least the 64 doubles of the former reduction area
  P.lds_red = 0;
  P.lds_w = 0;
  P.lds_wu = P.lds_w + n * n;
  P.lds_fx = P.lds_wu + d * d;
  P.lds_fu = P.lds_fx + P.nFx * n;
  P.nconst = P.lds_fu + P.nFu * d;
  P.lds_scr = std::max(64, (P.nconst + 7) & ~7);
  // (plans whose staging does not fit form each node's slack terms inside the tree solve's sweep)
  P.nscr = desc.controller == BMPC_CTRL_CVAR && P.lds_scr + ncoup + T * P.Nc <= 1248 ? T * P.Nc : 0;
  // pivots and right-hand sides before the matrix: lean launches keep those in LDS too (the
  // substitutions' dependent chains then run on LDS; only the matrix moves to the slab)
  P.lds_piv = P.lds_scr + P.nscr;
  P.lds_rhs = P.lds_piv + P.nsm;
  P.lds_rhs2 = P.lds_rhs + P.nsm;   // the pair's second right-hand side (kkt_back_pair)
  P.lds_M = P.lds_rhs2 + P.nsm;
  P.nlds = P.lds_M + P.nsm * P.nsm;
  P.nlds_lean = P.lds_M;
  if (P.nscr > 0 && P.nlds > 1248) return "internal: the tree-solve LDS staging overflows the 16-egos-per-CU budget";

  // ---- weights -----------------------------------------------------------------------------
  double Qm[BMPC_MAX_N * BMPC_MAX_N], Rm[BMPC_MAX_D * BMPC_MAX_D];
  for (int i = 0; i < n * n; ++i) Qm[i] = desc.Q[i];
  for (int i = 0; i < d * d; ++i) Rm[i] = desc.R[i];
  weight_root(Qm, n, P.W1);
  weight_root(Rm, d, P.Wu);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = 0.0;
      for (int r = 0; r < n; ++r) s += P.W1[r * n + i] * P.W1[r * n + j];
      P.QQ[i * n + j] = s;
    }
  for (int i = 0; i < d; ++i)
    for (int j = 0; j < d; ++j) {
      double s = 0.0;
      for (int r = 0; r < d; ++r) s += P.Wu[r * d + i] * P.Wu[r * d + j];
      P.RR[i * d + j] = s;
    }

  // ---- concatenated tables -------------------------------------------------------------------
#define BMPC_TOPO_HOSTVEC_(n) &hp.n,
  std::vector<int32_t>* tabs[] = {BMPC_TOPO_FIELDS(BMPC_TOPO_HOSTVEC_)};   // same order as Topo
#undef BMPC_TOPO_HOSTVEC_
  hp.blob.clear();
  hp.blob_off.clear();
  for (auto* v : tabs) {
    hp.blob_off.push_back(hp.blob.size());
    hp.blob.insert(hp.blob.end(), v->begin(), v->end());
  }
  hp.point_tables(hp.blob.data());

  // ---- per-ego workspace layout --------------------------------------------------------------
  Layout& L = hp.lay;
  size_t o = 0;
  auto take = [&](size_t cnt) {
    const size_t r = o;
    o += (cnt + 7) & ~(size_t)7;   // 64-byte aligned slices
    return r;
  };
  const int nv = P.nv, neq = P.neq, nr = P.nrows, nc = P.ncones;
  L.uLin = take((size_t)(U + 1) * d);
  L.pprev = take((size_t)bd * m);
  L.misc = take(8 + BMPC_MAX_N);
  L.xpred = take((size_t)T * n);
  L.upred = take((size_t)U * d);
  L.sol = take(nv);
  L.xbar = take((size_t)T * n);
  L.zbar = take((size_t)T * n);
  L.ubar = take((size_t)U * d);
  L.Ad = take((size_t)U * n * n);
  L.Bd = take((size_t)U * n * d);
  L.Cd = take((size_t)U * n);
  L.dh = take((size_t)T * P.Ncol * n);
  L.h0 = take((size_t)T * P.Ncol);
  L.w = take(nbr);
  L.p = take((size_t)bd * m);
  L.dp = take((size_t)bd * m * n);
  L.boost = take(2 * (size_t)nc);   // the cone boosts beta_k, then e^-beta_k
  L.xref = take(n);
  L.x = take(nv);
  L.y = take(neq);
  L.z = take(nr);
  L.s = take(nr);
  L.lam = take(nr);
  L.z1 = take(nr);
  L.z2 = take(nr);
  L.dz = take(nr);
  L.ds = take(nr);
  L.rx = take(nv);
  L.rz = take(nr);
  L.hvec = take(nr);
  L.ta = take(nv);
  L.ta2 = take(nv);
  L.ya = take(neq);
  L.ra = take(nr);
  L.rb = take(nr);
  L.rc = take(nr);
  L.bestx = take(nv);
  L.xeq = take(nv);
  L.aeq = take(neq);
  L.geq = take(nr);
  L.k_r0 = take(nr);
  L.k_nv0 = take(nv);
  L.k_e1 = take(2 * (size_t)nv);    // two halves: the pair's refinement (kkt_refine_pair)
  L.k_e2 = take(2 * (size_t)neq);
  L.k_e3 = take(nr);
  L.k_t3 = take(nr);
  L.k_t3b = take(nr);
  L.k_cx = take(2 * (size_t)nv);
  L.k_cy = take(2 * (size_t)neq);
  L.k_cz = take(2 * (size_t)nr);
  L.k_nv1 = take(nv);
  L.dl = take(P.nlp);
  L.dli = take(P.nlp);
  L.eta = take(nc);
  L.wbar = take(nr);
  L.vnt = take(nr);
  L.hx = take((size_t)T * n * n);
  L.hu = take((size_t)U * d * d);
  L.sd = take((size_t)T * P.Nc * 2);
  L.P = take((size_t)T * n * n);
  L.Kg = take((size_t)U * d * n);
  L.Luu = take((size_t)U * d * d);
  // tree-solve right-hand sides (CVaR: the nc Woodbury columns plus the c-direction and affine
  // solves that ride in the same tree solve, kkt_coupling / kkt_solve_pair)
  const size_t nrhs = nc > 0 ? (size_t)nc + 2 : 1;
  L.kff = take(nrhs * U * d);
  L.lvec = take(nrhs * T * n);
  L.qx0 = take(nrhs * T * n);   // slack-eliminated x rhs of the tree sweeps (pre-pass plans)
  if (nc > 0) {
    // contiguous rhs / solution blocks of the merged tree solve, stride nv (z-space) / neq
    // (eq-space): g_1..g_nc | tz_c | tz_a,  col_1..col_nc | x1 | x2,  colnu_1..nc | y1 | y2,
    // and the eq-space rhs 0 (nc times) | bvec | ry
    L.gk = take((size_t)(nc + 2) * nv);
    const size_t colk = take((size_t)(nc + 2) * nv);
    L.colk = colk;
    L.x1 = colk + (size_t)nc * nv;
    L.x2 = L.x1 + nv;
    const size_t colnu = take((size_t)(nc + 2) * neq);
    L.colnu = colnu;
    L.y1 = colnu + (size_t)nc * neq;
    L.y2 = L.y1 + neq;
    const size_t zb = take((size_t)(nc + 2) * neq);
    L.zeros = zb;                        // nc all-zero eq-space vectors (never written)
    L.bvec = zb + (size_t)nc * neq;
    L.ry = L.bvec + neq;
  } else {
    L.gk = L.colk = L.colnu = take(0);
    L.x1 = take(nv);
    L.y1 = take(neq);
    L.x2 = take(nv);
    L.y2 = take(neq);
    L.ry = take(neq);
    L.bvec = take(neq);
    L.zeros = take(neq);   // all-zero eq-space vector (tree solves without an e term)
  }
  L.prof = take(PROF_COUNT);
  L.coup = take((size_t)P.nsm * P.nsm + 2 * (size_t)P.nsm);
  L.ist = take(64);
  if (desc.controller != BMPC_CTRL_CVAR) {   // QP-only arrays (augmented-state Riccati)
    const int NS = n + d;
    L.qo = take((size_t)U * d * d);
    L.qq = take(nv);
    L.Pa = take((size_t)T * NS * NS);
    L.Ka = take((size_t)U * d * NS);
    L.la = take((size_t)T * NS);
  } else {
    L.qo = L.qq = L.Pa = L.Ka = L.la = 0;
  }
  L.xform = take(XF_COUNT);
  L.xlin = robust ? take((size_t)T * n) : 0;
  L.zrob = robust ? take((size_t)(T - 1) * P.Ncol * n) : 0;
  L.stride = o;
  return "";
}

}  // namespace bmpc
