// hostsim.cpp -- TEST-ONLY host build of the GPU solver templates.
//
// Instantiates the wave-cooperative templates of belief-planning_amd/csrc with a 1-lane
// host executor so the CPU test suite can check the kernel *algorithm* against the oracle
// without a GPU.  It exports its own `hs_*` symbols (never the product C ABI) and is never
// loaded by the belief-planning_amd package: the product path is libbmpc.so (HIP) only.
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "bmpc_plan.h"
#include "bmpc_hmm.h"
#include "bmpc_solve.h"
#include "bmpc_ipm_ph.h"
#include "bmpc_env.h"
#include "bmpc_qpplan.h"

using namespace bmpc;

#ifndef BMPC_HOST_CONE_REGS
#define BMPC_HOST_CONE_REGS 256
#endif

#ifdef BMPC_HOST_COUNT_SYNC   // diagnostics: executor barriers and whole-executor reductions per solve
long long g_syncs = 0, g_reds = 0;
#define HS_CNT(c) (++(c))
#else
#define HS_CNT(c) ((void)0)
#endif
extern "C" long long hs_sync_count(int which) {
#ifdef BMPC_HOST_COUNT_SYNC
  return which == 0 ? g_syncs : g_reds;
#else
  return -1 + 0 * which;
#endif
}

namespace {
template <bool TR, bool CL = true>
struct HostExecT {
  static constexpr bool kTransform = TR;
  static constexpr bool kCoupLds = CL;   // coupling system in the LDS stand-in (else the slab, as lean launches)
  int lane = 0;
  int nlanes = 1;
  double* lds = nullptr;      // stands in for the wave's LDS scratch
  using tab_ptr = const int32_t*;
  const int32_t* tab = nullptr;   // ... and for its LDS copy of the topology tables
  double* eco = nullptr;      // ... and for the per-ego constants (kTransform)
  static constexpr int kTaskLanes = 1;
  // one lane holds a whole cone (fused IPM passes); -DBMPC_HOST_CONE_REGS=1 runs the unfused
  // chain instead (what the GPU takes for cones wider than 8 rows per group lane)
  static constexpr int kConeRegRows = BMPC_HOST_CONE_REGS;
  double tsum(double v) const { return v; }
  template <int S>
  double tget(double v) const { return v; }
  double gsum(double v, int) const { return v; }
  double gmax(double v, int) const { return v; }
  double gmin(double v, int) const { return v; }
  void sync() const { HS_CNT(g_syncs); }
  bool uniform(bool b) const { return b; }
  double sum(double v) const { HS_CNT(g_reds); return v; }
  double max(double v) const { HS_CNT(g_reds); return v; }
  double min(double v) const { HS_CNT(g_reds); return v; }
  template <int K>
  void sum_n(double*) const { HS_CNT(g_reds); }
  template <int K>
  void min_n(double*) const { HS_CNT(g_reds); }
};
using HostExec = HostExecT<false>;

// BMPC_HOST_PHASED=1: CVaR solves through the phase sequence of the GPU's phase-per-kernel IPM
template <class X, class M>
IpmResult hs_solve_ego(const X& ex, const Plan& P, const Layout& L, EgoView E, const double* x, const double* z,
                       const double* xref, bool phased, std::vector<double>& lds) {
  if (!phased || P.desc.controller != BMPC_CTRL_CVAR) return solve_ego<X, M>(ex, P, L, E, x, z, xref);
  tree_step<X, M>(ex, P, L, E, x, z, xref);
  return solve_ego_ipm_phased<X, M>(ex, P, L, E, lds.data(), (int)lds.size());
}

struct HS {
  HostPlan hp;
  int batch;
  std::vector<double> ws;
  std::vector<bmpc_policy> pol;
  std::vector<double> lref;   // lane reference (grid | values) of the psiref policies
};
thread_local std::string g_err;
}  // namespace

extern "C" {

const char* hs_last_error(void) { return g_err.c_str(); }

int hs_create(const bmpc_plan_desc* desc, int batch, void** out) {
  HS* h = new HS();
  g_err = build_plan(*desc, h->hp);
  if (!g_err.empty()) {
    delete h;
    return -22;
  }
  h->batch = batch;
  h->ws.assign(h->hp.lay.stride * (size_t)batch, 0.0);
  h->pol.assign((size_t)batch * desc->m, bmpc_policy{});
  *out = h;
  return 0;
}

int hs_destroy(void* p) {
  delete (HS*)p;
  return 0;
}

int hs_info(void* p, int32_t* info) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  info[BMPC_INFO_T] = P.T;
  info[BMPC_INFO_U] = P.U;
  info[BMPC_INFO_BDIM] = P.bdim;
  info[BMPC_INFO_NBRANCH] = P.nbranch;
  info[BMPC_INFO_NV] = P.nv;
  info[BMPC_INFO_NEQ] = P.neq;
  info[BMPC_INFO_NROWS] = P.nrows;
  info[BMPC_INFO_NCONES] = P.ncones;
  info[BMPC_INFO_LP] = P.nlp;
  info[BMPC_INFO_BATCH] = h->batch;
  info[BMPC_INFO_WS_DOUBLES] = (int32_t)h->hp.lay.stride;
  info[BMPC_INFO_SOLVER] = BMPC_KERNEL_NONE;   // the host build has no kernels
  return 0;
}

int hs_set_policies(void* p, const bmpc_policy* pol) {
  HS* h = (HS*)p;
  memcpy(h->pol.data(), pol, sizeof(bmpc_policy) * h->pol.size());
  return 0;
}

int hs_solve(void* p, const double* x, const double* z, const double* xref, double* upred,
             double* xpred, double* bw, double* J, int32_t* status, int32_t* iters) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  const Layout& L = h->hp.lay;
  // egos are independent: one OpenMP thread per ego slice (OMP_NUM_THREADS; 1 without -fopenmp)
#pragma omp parallel
  {
  HostExec ex;
  HostExecT<true> exm;
  HostExecT<false, false> exl;          // BMPC_HOST_LEAN=1: the lean-LDS launch's slab coupling system
  const char* lean_env = getenv("BMPC_HOST_LEAN");
  const bool lean = lean_env && atoi(lean_env) != 0;
  const char* ph_env = getenv("BMPC_HOST_PHASED");
  const bool phased = ph_env && atoi(ph_env) != 0;
  std::vector<double> lds(P.nlds), eco(ECO_COUNT);
  for (int i = 0; i < P.nconst; ++i) lds[P.lds_w + i] = plan_const(P, i);
  ex.lds = exm.lds = exl.lds = lds.data();
  ex.tab = exm.tab = exl.tab = P.t.br_depth;      // the host blob (first table at offset 0)
  exm.eco = eco.data();
#pragma omp for schedule(dynamic, 4)
  for (int e = 0; e < h->batch; ++e) {
    EgoView E{h->ws.data() + L.stride * e, h->pol.data() + (size_t)e * P.m};
    IpmResult r;
    if (P.desc.model == BMPC_MODEL_HIGHWAY && (P.desc.flags & BMPC_PLAN_TRANSFORM))
      r = hs_solve_ego<HostExecT<true>, HighwayT>(exm, P, L, E, x + e * P.n, z + e * P.n, xref + e * P.n, phased, lds);
    else if (P.desc.model == BMPC_MODEL_HIGHWAY && lean && !phased)
      r = solve_ego<HostExecT<false, false>, Highway>(exl, P, L, E, x + e * P.n, z + e * P.n, xref + e * P.n);
    else if (P.desc.model == BMPC_MODEL_HIGHWAY)
      r = hs_solve_ego<HostExec, Highway>(ex, P, L, E, x + e * P.n, z + e * P.n, xref + e * P.n, phased, lds);
    else if (P.desc.model == BMPC_MODEL_HIGHWAY_MERGE)
      r = hs_solve_ego<HostExecT<true>, HighwayMerge>(exm, P, L, E, x + e * P.n, z + e * P.n, xref + e * P.n, phased, lds);
    else
      r = hs_solve_ego<HostExec, Quadruped>(ex, P, L, E, x + e * P.n, z + e * P.n, xref + e * P.n, phased, lds);
    const double* ws = E.ws;
    if (upred) memcpy(upred + (size_t)e * P.U * P.d, ws + L.upred, sizeof(double) * P.U * P.d);
    if (xpred) memcpy(xpred + (size_t)e * P.T * P.n, ws + L.xpred, sizeof(double) * P.T * P.n);
    if (bw) memcpy(bw + (size_t)e * (P.nbranch - 1), ws + L.w + 1, sizeof(double) * (P.nbranch - 1));
    if (J) J[e] = P.desc.controller != BMPC_CTRL_CVAR ? r.pcost : ws[L.sol + P.oJ];
    if (status) status[e] = r.exit_flag;
    if (iters) iters[e] = r.iters;
  }
  }
  return 0;
}

int hs_set_warm_start(void* p, const double* uLin, const double* pprev, const double* jcons,
                      const double* oldu) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  const Layout& L = h->hp.lay;
  for (int e = 0; e < h->batch; ++e) {
    double* ws = h->ws.data() + L.stride * e;
    memcpy(ws + L.uLin, uLin + (size_t)e * (P.U + 1) * P.d, sizeof(double) * (P.U + 1) * P.d);
    if (pprev) memcpy(ws + L.pprev, pprev + (size_t)e * P.bdim * P.m, sizeof(double) * P.bdim * P.m);
    if (jcons) ws[L.misc + MISC_JCONS] = jcons[e];
    if (oldu) memcpy(ws + L.misc + MISC_OLDU, oldu + (size_t)e * P.d, sizeof(double) * P.d);
    ws[L.misc + MISC_INIT] = 1.0;
  }
  return 0;
}

int hs_set_robust_warm_start(void* p, const double* xlin, const double* ulin, const double* oldu) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  const Layout& L = h->hp.lay;
  for (int e = 0; e < h->batch; ++e) {
    double* ws = h->ws.data() + L.stride * e;
    memcpy(ws + L.xlin, xlin + (size_t)e * P.T * P.n, sizeof(double) * P.T * P.n);
    memcpy(ws + L.uLin, ulin + (size_t)e * P.U * P.d, sizeof(double) * P.U * P.d);
    memcpy(ws + L.misc + MISC_OLDU, oldu + (size_t)e * P.d, sizeof(double) * P.d);
    ws[L.misc + MISC_INIT] = 1.0;
  }
  return 0;
}

// bmpc_set_transform of the host build (same slab slots)
int hs_set_transform(void* p, const double* S, const uint8_t* s_on, const double* bx) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  const Layout& L = h->hp.lay;
  const int n = P.n;
  for (int e = 0; e < h->batch; ++e) {
    double* xf = h->ws.data() + L.stride * e + L.xform;
    for (int i = 0; i < n * n; ++i) xf[XF_S + i] = S ? S[(size_t)e * n * n + i] : 0.0;
    xf[XF_SON] = (S && (!s_on || s_on[e])) ? 1.0 : 0.0;
    if (bx) {
      for (int i = 0; i < P.nFx; ++i) xf[XF_BX + i] = bx[(size_t)e * P.nFx + i];
      xf[XF_BXSET] = 1.0;
    }
  }
  return 0;
}

// bmpc_set_fx of the host build (solve's Fx argument, kept until the next one)
int hs_set_fx(void* p, const double* Fx) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  const Layout& L = h->hp.lay;
  for (int e = 0; e < h->batch; ++e) {
    double* xf = h->ws.data() + L.stride * e + L.xform;
    for (int i = 0; i < P.nFx * P.n; ++i) xf[XF_FX + i] = Fx[(size_t)e * P.nFx * P.n + i];
    xf[XF_FXSET] = 1.0;
  }
  return 0;
}

// BranchTree.dp of every non-leaf branch [batch][bdim][m][n] (bmpc_get_branch_dp)
int hs_get_branch_dp(void* p, double* dp) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  const Layout& L = h->hp.lay;
  const size_t k = (size_t)P.bdim * P.m * P.n;
  for (int e = 0; e < h->batch; ++e) memcpy(dp + e * k, h->ws.data() + L.stride * e + L.dp, sizeof(double) * k);
  return 0;
}

// debugging aids: raw workspace of ego e and the Layout offsets (sizeof(Layout)/8 size_t)
double* hs_ws_ptr(void* p, int e) {
  HS* h = (HS*)p;
  return h->ws.data() + h->hp.lay.stride * e;
}
int hs_layout(void* p, size_t* out) {
  HS* h = (HS*)p;
  memcpy(out, &h->hp.lay, sizeof(Layout));
  return (int)(sizeof(Layout) / sizeof(size_t));
}

int hs_reset(void* p, const uint8_t* mask) {
  HS* h = (HS*)p;
  const Layout& L = h->hp.lay;
  for (int e = 0; e < h->batch; ++e)
    if (!mask || mask[e]) h->ws[L.stride * e + L.misc + MISC_INIT] = 0.0;
  return 0;
}

int hs_get_tree(void* p, double* xbar, double* ubar, double* zbar, double* w, double* pr,
                double* sol) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  const Layout& L = h->hp.lay;
  for (int e = 0; e < h->batch; ++e) {
    const double* ws = h->ws.data() + L.stride * e;
    if (xbar) memcpy(xbar + (size_t)e * P.T * P.n, ws + L.xbar, sizeof(double) * P.T * P.n);
    if (zbar) memcpy(zbar + (size_t)e * P.T * P.n, ws + L.zbar, sizeof(double) * P.T * P.n);
    if (ubar) memcpy(ubar + (size_t)e * P.U * P.d, ws + L.ubar, sizeof(double) * P.U * P.d);
    if (w) memcpy(w + (size_t)e * P.nbranch, ws + L.w, sizeof(double) * P.nbranch);
    if (pr) memcpy(pr + (size_t)e * P.bdim * P.m, ws + L.p, sizeof(double) * P.bdim * P.m);
    if (sol) memcpy(sol + (size_t)e * P.nv, ws + L.sol, sizeof(double) * P.nv);
  }
  return 0;
}

int hs_set_lane_ref(void* hp, int nref, const double* grid, const double* values) {
  HS* h = (HS*)hp;
  h->lref.assign(grid, grid + nref);
  h->lref.insert(h->lref.end(), values, values + nref);
  h->hp.plan.lref = nref ? h->lref.data() : nullptr;
  h->hp.plan.nlref = nref;
  return 0;
}

int hs_model_eval_ref(const bmpc_plan_desc* D, const bmpc_policy* pol, int nref, const double* grid,
                      const double* values, int B, const double* x, const double* u, const double* z, double* A,
                      double* Bm, double* C, double* xp, double* p, double* dp, double* zpred, double* h0,
                      double* dh) {
  const int n = D->n, d = D->d, m = D->m, N = D->N;
  const LaneRef R{grid, values, nref};
  for (int b = 0; b < B; ++b) {
    const bmpc_policy* pb = pol + (size_t)b * m;
#define OFF(ptr, k) (ptr ? ptr + (size_t)b * (k) : nullptr)
    if (D->model == BMPC_MODEL_HIGHWAY)
      model_eval_point<Highway>(*D, pb, x + b * n, u + b * d, z + b * n, OFF(A, n * n), OFF(Bm, n * d),
                                OFF(C, n), OFF(xp, n), OFF(p, m), OFF(dp, m * n), OFF(zpred, N * m * n),
                                OFF(h0, 1), OFF(dh, n), R);
    else if (D->model == BMPC_MODEL_HIGHWAY_MERGE)
      model_eval_point<HighwayMerge>(*D, pb, x + b * n, u + b * d, z + b * n, OFF(A, n * n), OFF(Bm, n * d),
                                     OFF(C, n), OFF(xp, n), OFF(p, m), OFF(dp, m * n), OFF(zpred, N * m * n),
                                     OFF(h0, 1), OFF(dh, n), R);
    else
      model_eval_point<Quadruped>(*D, pb, x + b * n, u + b * d, z + b * n, OFF(A, n * n), OFF(Bm, n * d),
                                  OFF(C, n), OFF(xp, n), OFF(p, m), OFF(dp, m * n),
                                  OFF(zpred, N * m * n), OFF(h0, 1), OFF(dh, n), R);
#undef OFF
  }
  return 0;
}

int hs_model_eval(const bmpc_plan_desc* D, const bmpc_policy* pol, int B, const double* x,
                  const double* u, const double* z, double* A, double* Bm, double* C, double* xp,
                  double* p, double* dp, double* zpred, double* h0, double* dh) {
  const int n = D->n, d = D->d, m = D->m, N = D->N;
  for (int b = 0; b < B; ++b) {
    const bmpc_policy* pb = pol + (size_t)b * m;
#define OFF(ptr, k) (ptr ? ptr + (size_t)b * (k) : nullptr)
    if (D->model == BMPC_MODEL_HIGHWAY)
      model_eval_point<Highway>(*D, pb, x + b * n, u + b * d, z + b * n, OFF(A, n * n), OFF(Bm, n * d),
                                OFF(C, n), OFF(xp, n), OFF(p, m), OFF(dp, m * n), OFF(zpred, N * m * n),
                                OFF(h0, 1), OFF(dh, n));
    else if (D->model == BMPC_MODEL_HIGHWAY_MERGE)
      model_eval_point<HighwayMerge>(*D, pb, x + b * n, u + b * d, z + b * n, OFF(A, n * n), OFF(Bm, n * d),
                                     OFF(C, n), OFF(xp, n), OFF(p, m), OFF(dp, m * n), OFF(zpred, N * m * n),
                                     OFF(h0, 1), OFF(dh, n));
    else
      model_eval_point<Quadruped>(*D, pb, x + b * n, u + b * d, z + b * n, OFF(A, n * n), OFF(Bm, n * d),
                                  OFF(C, n), OFF(xp, n), OFF(p, m), OFF(dp, m * n),
                                  OFF(zpred, N * m * n), OFF(h0, 1), OFF(dh, n));
#undef OFF
  }
  return 0;
}


int hs_env_step(void* p, const bmpc_env_desc* env, int t, double* scene, const double* upred, const double* J,
                const int32_t* status, const int32_t* iters, double* x, double* z, double* xref, double* stats) {
  HS* h = (HS*)p;
  const Plan& P = h->hp.plan;
  for (int e = 0; e < h->batch; ++e) {
    double* st = scene + (size_t)e * ENV_STRIDE;
    if (t > 0 && stats && J && status && iters)
      env_accumulate(st, J[e], status[e], iters[e], P.desc.controller == BMPC_CTRL_CVAR, stats + (size_t)e * ENVS_STRIDE);
    env_step_ego(*env, P.desc.dt, P.N, P.m, t, st, h->pol.data() + (size_t)e * P.m,
                 upred ? upred + (size_t)e * P.U * P.d : nullptr, x + (size_t)e * 4, z + (size_t)e * 4,
                 xref + (size_t)e * 4);
  }
  return 0;
}

int hs_get_policies(void* p, bmpc_policy* out) {
  HS* h = (HS*)p;
  memcpy(out, h->pol.data(), sizeof(bmpc_policy) * h->pol.size());
  return 0;
}

int hs_hmm_eval(int M, int m, const double* hc, int B, const double* xb, const double* u, const double* xbackup,
                double* xbp, double* A, double* Bm, double* C, double* h0, double* Jh) {
  const int nb = 4 + M * m;
  for (int p = 0; p < B; ++p)
    hmm_linearize(M, m, hc, xb + (size_t)p * nb, u + (size_t)p * 2, xbackup + (size_t)p * M * m * 4,
                  xbp ? xbp + (size_t)p * nb : nullptr, A ? A + (size_t)p * nb * nb : nullptr,
                  Bm ? Bm + (size_t)p * nb * 2 : nullptr, C ? C + (size_t)p * nb : nullptr,
                  h0 ? h0 + (size_t)p * M * m : nullptr, Jh ? Jh + (size_t)p * M * m * nb : nullptr);
  return 0;
}

int hs_qp_solve(int n, int m, const int32_t* Pp, const int32_t* Pi, const int32_t* Ap, const int32_t* Ai, int batch,
                const double* Px, const double* q, const double* Ax, const double* l, const double* u, int max_iter,
                double eps, double* x, double* y, int32_t* status, int32_t* iters, int32_t* info) {
  HostBandQP h;
  g_err = bandqp_analyse(n, m, Pp, Pi, Ap, Ai, batch, l, u, max_iter, eps, h);
  if (!g_err.empty()) return -22;
  if (info) {
    info[0] = h.d.nk;
    info[1] = h.d.bw;
    info[2] = h.d.n_in;
    info[3] = h.d.nscat;
  }
  const int nnzP = Pp[n], nnzA = Ap[n];
  std::vector<double> vals(h.d.nvals + 1), cvals(h.d.ncvals), ws(h.d.stride), lds(bandqp_lds_doubles(h.d.nk, h.d.W, h.d.lb_lds));
  std::vector<double> ybuf(m + 1);
  HostExec ex;
  ex.lds = lds.data();
  for (int b = 0; b < batch; ++b) {
    for (int t = 0; t < nnzP; ++t) vals[t] = Px[(size_t)b * nnzP + t];
    for (int t = 0; t < nnzA; ++t) vals[nnzP + t] = Ax[(size_t)b * nnzA + t];
    for (int j = 0; j < n; ++j) cvals[j] = q[(size_t)b * n + j];
    for (int r = 0; r < m; ++r) {
      cvals[n + r] = l[(size_t)b * m + r];
      cvals[n + m + r] = u[(size_t)b * m + r];
    }
    int it = 0;
    status[b] = bandqp_solve(ex, h.d, vals.data(), cvals.data(), ws.data(), x + (size_t)b * n,
                             y ? y + (size_t)b * m : ybuf.data(), &it);
    if (iters) iters[b] = it;
  }
  return 0;
}

}  // extern "C"
