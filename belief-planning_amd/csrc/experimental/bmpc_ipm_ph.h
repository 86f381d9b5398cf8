// bmpc_ipm_ph.h -- the CVaR interior point of bmpc_ipm.h cut into phases, each run as a kernel
// of its own over the whole batch (phase-per-kernel IPM, bmpc_dev_ph.h).
//
// Why: the monolithic k_ipm calls its phases as out-of-line device functions, and the AMDGPU
// calling convention makes a callee save and restore every callee-saved VGPR it touches (the
// v40+ stripes: 48 of a 128-VGPR function, ~25 KB of scratch traffic per call and wave, ~24
// calls per IPM iteration).  A kernel saves nothing: here every phase is inlined into the
// kernel that runs it, so no phase pays a calling-convention round trip, and each kernel gets
// its own register allocation.
//
// The arithmetic is exactly ipm_solve's, operation for operation (the phased and the monolithic
// solve of an ego are bit-identical; tests/test_phased_*): ipm_solve's control flow is cut at
// the phase calls, and the scalars it carries across them (tau, kappa, the best iterate's
// scores, the affine step's sigma / eta, the refinement's scale and stop flags, ...) live in
// the ego's state block (Layout::ist), the factored coupling system between kernels in
// Layout::coup (copied into LDS by every kernel that solves with it).
//
// Per solve: INIT1 (h / b, W = I, first factorisation), INIT2 (coupling system), INIT3 (the two
// initial-point solves); per iteration it: RES (residuals, exit tests, best iterate, NT scaling),
// FAC (factorisation, right-hand sides of the c- and affine directions), CPL (Woodbury tree solve
// of nc + 2 right-hand sides, coupling LU), BKP (back halves of the two solves), RFP0 / RFP1
// (their refinement rounds), AFF (affine step, combined right-hand side), CMB (combined solve),
// RFC0 / RFC1 (its refinement rounds), UPD (step, or the backtrack exit); FIN unpacks.
#pragma once

#include "bmpc_solve.h"

namespace bmpc {

// per-ego IPM state (Layout::ist, doubles)
enum {
  IS_ACTIVE = 0,   // 1 while the ego iterates
  IS_OK,           // no phase of the current iteration has failed
  IS_EXIT, IS_ITERS, IS_PCOST,   // result
  IS_TAU, IS_KAP, IS_RESY0, IS_RESZ0,
  IS_BEST, IS_BEST_TAU, IS_BS_PRES, IS_BS_DRES, IS_BS_RELGAP, IS_BS_GAP, IS_BS_PCOST, IS_BS_OKCX,
  IS_NREF, IS_RT, IS_MU, IS_DEN, IS_DTAU_A, IS_DKAP_A, IS_SIGMA, IS_ETA1,
  IS_SC0, IS_SC1, IS_STOP0, IS_STOP1,   // refinement: scale and "stopped" per right-hand side
  IS_COUNT
};
static_assert(IS_COUNT <= 64, "Layout::ist holds 64 doubles");

enum {
  PH_INIT1 = 0, PH_INIT2, PH_INIT3, PH_RES, PH_FAC, PH_CPL, PH_BKP, PH_RFP0, PH_RFP1, PH_AFF, PH_CMB,
  PH_RFC0, PH_RFC1, PH_UPD, PH_FIN, PH_COUNT
};

template <class X>
BMPC_HD bool ph_flag(const X& ex, const gdouble* st, int slot) {
  return ex.uniform(st[slot] != 0.0);
}

// the factored coupling system between kernels: LDS matrix -> Layout::coup[0, nsm^2), LDS
// pivots -> Layout::coup[nsm^2, nsm^2 + nsm)
template <class X>
BMPC_HD void coup_save(const X& ex, const Ctx& C) {
  CPlan& P = *C.P;
  const int nm = P.nsm * P.nsm, n = nm + P.nsm;
  gdouble* dst = C.ws + C.L->coup;
  lane_batch<8>(ex, 0, n, [&](int i) { return (double)ex.lds[i < nm ? P.lds_M + i : P.lds_piv + (i - nm)]; },
                [&](int i, double v) { dst[i] = v; });
  ex.sync();
}
template <class X>
BMPC_HD void coup_load(const X& ex, const Ctx& C) {
  CPlan& P = *C.P;
  const int nm = P.nsm * P.nsm, n = nm + P.nsm;
  const gdouble* src = C.ws + C.L->coup;
  lane_batch<8>(ex, 0, n, [&](int i) { return src[i]; },
                [&](int i, double v) { ex.lds[i < nm ? P.lds_M + i : P.lds_piv + (i - nm)] = v; });
  ex.sync();
}

// ---- INIT1: h, b, identity scaling, first factorisation (ipm_solve's initial point) ----------
template <class X, int NX, int NU>
BMPC_HD void ph_init1(const X ex, const Ctx& C) {
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* st = ws + L.ist;
  if (BMPC_EQUIL) equilibrate<X, NX, NU>(ex, C);   // (ipm_solve: the same initial point and norms)
  build_hb<X, NX, NU>(ex, C, ws + L.hvec, ws + L.bvec);
  identity_scaling(ex, C);
  const bool ok = ex.uniform(kkt_factor<X, NX, NU>(ex, C, true));
  if (ex.lane == 0) {
    st[IS_ACTIVE] = 0.0;
    st[IS_OK] = ok ? 1.0 : 0.0;
    st[IS_EXIT] = ok ? (double)EXIT_MAXIT : (double)EXIT_NUMERICS;
    st[IS_ITERS] = 0.0;
    st[IS_PCOST] = 0.0;
  }
}

// ---- INIT2: the coupling system of the W = I factorisation -----------------------------------
template <class X, int NX, int NU>
BMPC_HD void ph_init2(const X ex, const Ctx& C) {
  gdouble* st = C.ws + C.L->ist;
  const bool ok = ex.uniform(kkt_coupling<X, NX, NU>(ex, C, 0));
  coup_save(ex, C);
  if (ex.lane == 0 && !ok) {
    st[IS_OK] = 0.0;
    st[IS_EXIT] = (double)EXIT_NUMERICS;
  }
}

// ---- INIT3: the two initial-point solves, bring2cone, the iteration's starting scalars -------
template <class X, int NX, int NU>
BMPC_HD void ph_init3(const X ex, const Ctx& C) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* st = ws + L.ist;
  coup_load(ex, C);
  const int nv = P.nv, neq = P.neq, nr = P.nrows;
  gdouble* tA = ws + L.ta;
  gdouble* ya = ws + L.ya;
  gdouble* ra = ws + L.ra;
  gdouble* z2 = ws + L.z2;
  gdouble* hv = ws + L.hvec;
  gdouble* bv = ws + L.bvec;
  // pass 0: [x; y2; z2] = K^-1 [0; b; h], s = bring2cone(-z2)
  // pass 1: [x2; y; z2] = K^-1 [-c; 0; 0], z = bring2cone(z2)      (one copy of the solve's code)
  for (int pass = 0; pass < 2; ++pass) {
    const bool p0 = ex.uniform(pass == 0);
    lane_batch<16>(ex, 0, nv, [&](int i) { return (!p0 && i == P.oJ) ? -1.0 : 0.0; }, [&](int i, double v) { tA[i] = v; });
    if (!p0) {
      lane_batch(ex, 0, neq, [&](int i) { return 0.0; }, [&](int i, double v) { ya[i] = v; });
      lane_batch<16>(ex, 0, nr, [&](int i) { return 0.0; }, [&](int i, double v) { ra[i] = v; });
    }
    ex.sync();
    const gdouble* r2 = uniform_ptr(p0 ? bv : ya);
    const gdouble* r3 = uniform_ptr(p0 ? hv : ra);
    gdouble* dx = uniform_ptr(ws + (p0 ? L.x : L.x2));
    gdouble* dy = uniform_ptr(ws + (p0 ? L.y2 : L.y));
    kkt_solve<X, NX, NU>(ex, C, tA, r2, r3, dx, dy, z2, BMPC_NITREF_INIT);
    const gdouble* gq = ws + L.geq;
    if (p0) {
      lane_batch<16>(ex, 0, nr, [&](int i) { return -(BMPC_EQUIL ? gq[i] : 1.0) * z2[i]; }, [&](int i, double v) { ra[i] = v; });
      ex.sync();
    } else if (BMPC_EQUIL) {
      lane_batch<16>(ex, 0, nr, [&](int i) { return gq[i] * z2[i]; }, [&](int i, double v) { z2[i] = v; });
      ex.sync();
    }
    gdouble* sz = uniform_ptr(ws + (p0 ? L.s : L.z));
    bring2cone(ex, C, uniform_ptr(p0 ? (const gdouble*)ra : (const gdouble*)z2), sz);
    if (BMPC_EQUIL) {   // s = ge s~, z = z~ / ge
      lane_batch<16>(ex, 0, nr, [&](int i) { return p0 ? gq[i] * sz[i] : sz[i] / gq[i]; }, [&](int i, double v) { sz[i] = v; });
      ex.sync();
    }
  }
  const gdouble* aq = ws + L.aeq;
  const gdouble* gq = ws + L.geq;
  const double resy0 = fmax(1.0, sqrt(lane_sum(ex, 0, neq, [&](int i) {
    const double v = BMPC_EQUIL ? bv[i] / aq[i] : bv[i];
    return v * v;
  })));
  const double resz0 = fmax(1.0, sqrt(lane_sum(ex, 0, nr, [&](int i) {
    const double v = BMPC_EQUIL ? hv[i] / gq[i] : hv[i];
    return v * v;
  })));
  if (ex.lane == 0) {
    st[IS_ACTIVE] = 1.0;
    st[IS_TAU] = 1.0;
    st[IS_KAP] = 1.0;
    st[IS_RESY0] = resy0;
    st[IS_RESZ0] = resz0;
    st[IS_BEST] = 1e300;
    st[IS_BEST_TAU] = 1.0;
    st[IS_BS_PRES] = st[IS_BS_DRES] = st[IS_BS_RELGAP] = st[IS_BS_GAP] = st[IS_BS_PCOST] = 0.0;
    st[IS_BS_OKCX] = 0.0;
  }
}

// ---- RES: residuals, the exit tests, the best iterate, then the NT scaling -------------------
template <class X, int NX, int NU>
BMPC_HD void ph_res(const X ex, const Ctx& C, int it) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* st = ws + L.ist;
  const int nv = P.nv, neq = P.neq, nr = P.nrows;
  gdouble* x = ws + L.x;
  gdouble* y = ws + L.y;
  gdouble* z = ws + L.z;
  gdouble* s = ws + L.s;
  gdouble* rx = ws + L.rx;
  gdouble* ry = ws + L.ry;
  gdouble* rz = ws + L.rz;
  gdouble* hv = ws + L.hvec;
  gdouble* bv = ws + L.bvec;
  gdouble* tA = ws + L.ta;
  gdouble* ra = ws + L.ra;
  gdouble* rb = ws + L.rb;
  const double feastol = P.desc.feastol, abstol = P.desc.abstol, reltol = P.desc.reltol;
  const double deg = (double)(P.nlp + P.ncones);
  const double tau = st[IS_TAU], kap = st[IS_KAP];
  const gdouble* xq = ws + L.xeq;
  const gdouble* aq = ws + L.aeq;
  const gdouble* gq = ws + L.geq;
  const double resx0 = BMPC_EQUIL ? fmax(1.0, 1.0 / xq[P.oJ]) : 1.0, resy0 = st[IS_RESY0], resz0 = st[IS_RESZ0];
  double best_score = st[IS_BEST];

  apply_AT<X, NX, NU>(ex, C, y, rx);
  apply_GT<X, NX, NU>(ex, C, z, tA);
  // (ipm_solve's passes: the equilibrated norms formed with the residuals)
  double acx[2] = {0.0, 0.0}, acy[3] = {0.0, 0.0, 0.0}, acz[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  struct R2b { double v, rs, xs; };
  lane_batch<8>(ex, 0, nv, [&](int i) {
    const double xi = x[i], q = BMPC_EQUIL ? xq[i] : 1.0;
    const double v = rx[i] + (tA[i] + (i == P.oJ ? tau : 0.0));
    return R2b{v, v / q, q * xi};
  }, [&](int i, R2b r) { rx[i] = r.v; acx[0] += r.rs * r.rs; acx[1] += r.xs * r.xs; });
  apply_A<X, NX, NU>(ex, C, x, ry);
  struct R4 { double v, rs, a, ys; };
  lane_batch<8>(ex, 0, neq, [&](int i) {
    const double yi = y[i], bi = bv[i], q = BMPC_EQUIL ? aq[i] : 1.0;
    const double v = bi * tau - ry[i];
    return R4{v, v / q, bi * yi, q * yi};
  }, [&](int i, R4 r) { ry[i] = r.v; acy[0] += r.rs * r.rs; acy[1] += r.a; acy[2] += r.ys * r.ys; });
  apply_G<X, NX, NU>(ex, C, x, rz);
  struct R7 { double v, rs, a, zs, ss, sz; };
  lane_batch<4>(ex, 0, nr, [&](int i) {
    const double zi = z[i], si = s[i], hi = hv[i], q = BMPC_EQUIL ? gq[i] : 1.0;
    const double v = hi * tau - rz[i] - si;
    return R7{v, v / q, hi * zi, q * zi, si / q, si * zi};
  }, [&](int i, R7 r) { rz[i] = r.v; acz[0] += r.rs * r.rs; acz[1] += r.a; acz[2] += r.zs * r.zs; acz[3] += r.ss * r.ss; acz[4] += r.sz; });
  ex.sync();
  const double cx = x[P.oJ];
  const double by = ex.sum(acy[1]), hz = ex.sum(acz[1]);
  const double rt = kap + cx + by + hz;
  const double nx = sqrt(ex.sum(acx[1])), ny = sqrt(ex.sum(acy[2]));
  const double nz = sqrt(ex.sum(acz[2])), ns = sqrt(ex.sum(acz[3]));
  const double sz = ex.sum(acz[4]);
  const double mu = (sz + kap * tau) / (deg + 1.0);
  const double gap = sz / (tau * tau);
  const double pcost = cx / tau, dcost = -(hz + by) / tau;
  double relgap = -1.0;
  if (pcost < 0.0) relgap = gap / (-pcost);
  else if (dcost > 0.0) relgap = gap / dcost;
  const double nry = neq ? sqrt(ex.sum(acy[0])) / fmax(resy0 + nx, 1.0) : 0.0;
  const double nrz = sqrt(ex.sum(acz[0])) / fmax(resz0 + nx + ns, 1.0);
  const double pres = fmax(nry, nrz) / tau;
  const double dres = sqrt(ex.sum(acx[0])) / fmax(resx0 + ny + nz, 1.0) / tau;
  double pinfres = -1.0, dinfres = -1.0;
  if (ex.uniform((hz + by) / fmax(ny + nz, 1.0) < -reltol)) {
    lane_batch<16>(ex, 0, nv, [&](int i) { return (rx[i] - (i == P.oJ ? tau : 0.0)) / (BMPC_EQUIL ? xq[i] : 1.0); },
                   [&](int i, double v) { ra[i] = v; });
    ex.sync();
    pinfres = sqrt(vdot(ex, ra, ra, nv)) / fmax(ny + nz, 1.0);
  }
  if (ex.uniform(cx / fmax(nx, 1.0) < -reltol)) {
    apply_A<X, NX, NU>(ex, C, x, rb);
    const double a1 = sqrt(lane_sum(ex, 0, neq, [&](int i) {
      const double v = rb[i] / (BMPC_EQUIL ? aq[i] : 1.0);
      return v * v;
    })) / fmax(nx, 1.0);
    apply_G<X, NX, NU>(ex, C, x, ra);
    lane_batch<16>(ex, 0, nr, [&](int i) { return (ra[i] + s[i]) / (BMPC_EQUIL ? gq[i] : 1.0); },
                   [&](int i, double v) { ra[i] = v; });
    ex.sync();
    const double a2 = sqrt(vdot(ex, ra, ra, nr)) / fmax(nx + ns, 1.0);
    dinfres = fmax(a1, a2);
  }
  auto check = [&](double ft, double at, double rtl) -> int {
    if (!(tau > 0.0 && kap >= 0.0)) return 99;
    if ((-cx > 0.0 || -by - hz >= -at) && pres < ft && dres < ft &&
        (gap < at || (relgap >= 0.0 && relgap < rtl)))
      return EXIT_OPTIMAL;
    if (dinfres >= 0.0 && dinfres < ft && tau < kap) return EXIT_DINF;
    if ((pinfres >= 0.0 && pinfres < ft && tau < kap) ||
        (tau < ft && kap < ft && pinfres >= 0.0 && pinfres < ft))
      return EXIT_PINF;
    return 99;
  };
  const double score = fmax(fmax(pres, dres), relgap >= 0.0 ? relgap : 1e300);
  if (ex.uniform(score < best_score)) {
    best_score = score;
    if (ex.lane == 0) {
      st[IS_BEST] = best_score;
      st[IS_BEST_TAU] = tau;
      st[IS_BS_PRES] = pres;
      st[IS_BS_DRES] = dres;
      st[IS_BS_RELGAP] = relgap;
      st[IS_BS_GAP] = gap;
      st[IS_BS_PCOST] = pcost;
      st[IS_BS_OKCX] = (-cx > 0.0 || -by - hz >= -5e-5) ? 1.0 : 0.0;
      ws[L.misc + MISC_BEST] = best_score;   // the monolithic kernel's guard mirror
      ws[L.misc + MISC_BEST + 1] = tau;
    }
    lane_batch<16>(ex, 0, nv, [&](int i) { return x[i]; }, [&](int i, double v) { ws[L.bestx + i] = v; });
    ex.sync();
  }
  int code = check(feastol, abstol, reltol);
  if (code == 99 && it == P.desc.maxit) {
    const int c2 = check(1e-4, 5e-5, 5e-5);
    code = c2 == 99 ? EXIT_MAXIT : c2 + EXIT_INACC;
  }
  if (ex.uniform(code != 99)) {
    lane_batch<16>(ex, 0, nv, [&](int i) { return x[i] / tau; }, [&](int i, double v) { ws[L.sol + i] = v; });
    ex.sync();
    if (ex.lane == 0) {
      st[IS_EXIT] = (double)code;
      st[IS_ITERS] = (double)it;
      st[IS_PCOST] = pcost;
      st[IS_ACTIVE] = 0.0;
    }
    return;
  }
  const bool ok = ex.uniform(compute_scaling(ex, C, s, z));
  const int nref = score < BMPC_REFSCORE2 ? BMPC_NITREF2 : score < BMPC_REFSCORE ? BMPC_NITREF : 0;
  if (ex.lane == 0) {
    st[IS_OK] = ok ? 1.0 : 0.0;
    st[IS_NREF] = (double)nref;
    st[IS_RT] = rt;
    st[IS_MU] = mu;
  }
}

// ---- FAC: factorisation and the right-hand sides of the c- and affine directions -------------
template <class X, int NX, int NU>
BMPC_HD void ph_fac(const X ex, const Ctx& C) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* st = ws + L.ist;
  const int nv = P.nv;
  const bool ok = ex.uniform(kkt_factor<X, NX, NU>(ex, C, false));
  if (ok) {
    gdouble* tA = ws + L.ta;
    gdouble* tA2 = ws + L.ta2;
    gdouble* rx = ws + L.rx;
    gdouble* rb = ws + L.rb;
    lane_batch<16>(ex, 0, nv, [&](int i) { return i == P.oJ ? -1.0 : 0.0; }, [&](int i, double v) { tA[i] = v; });
    lane_batch<16>(ex, 0, nv, [&](int i) { return -rx[i]; }, [&](int i, double v) { tA2[i] = v; });
    apply_W(ex, C, 0, ws + L.lam, rb, 1.0, ws + L.rz, 1.0);
    // kkt_solve_pair's right-hand sides: G'W^-1 (W^-1 r3) + r1 for both solves
    const size_t nvs = P.nv, nc = P.ncones;
    gdouble* tzc = ws + L.gk + nc * nvs;
    gdouble* tza = tzc + nvs;
    gdouble* tr = ws + L.k_r0;
    apply_Winv2(ex, C, ws + L.hvec, ws + L.k_t3, tr);
    apply_GT<X, NX, NU>(ex, C, tr, tzc, tA);
    apply_Winv2(ex, C, rb, ws + L.k_t3b, tr);
    apply_GT<X, NX, NU>(ex, C, tr, tza, tA2);
  }
  if (ex.lane == 0 && !ok) st[IS_OK] = 0.0;
}

// ---- CPL: Woodbury columns and the two directions' tree parts in one tree solve, coupling LU -
template <class X, int NX, int NU>
BMPC_HD void ph_cpl(const X ex, const Ctx& C) {
  gdouble* st = C.ws + C.L->ist;
  const bool ok = ex.uniform(kkt_coupling<X, NX, NU>(ex, C, 2));
  coup_save(ex, C);
  if (ex.lane == 0 && !ok) st[IS_OK] = 0.0;
}

// ---- BKP: back halves of the c- and affine solves (kkt_solve_pair) ----------------------------
template <class X, int NX, int NU>
BMPC_HD void ph_bkp(const X ex, const Ctx& C) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  const gdouble* st = ws + L.ist;
  coup_load(ex, C);
  const bool fin = ex.uniform(st[IS_NREF] == 0.0);
  const size_t nvs = P.nv, nc = P.ncones;
  gdouble* tzc = ws + L.gk + nc * nvs;
  gdouble* tza = tzc + nvs;
  // both back halves through one copy of the code
  for (int j = 0; j < 2; ++j) {
    const bool c = ex.uniform(j == 0);
    kkt_back<X, NX, NU, false>(ex, C, uniform_ptr(c ? tzc : tza), uniform_ptr(ws + (c ? L.bvec : L.ry)),
                               uniform_ptr(ws + (c ? L.k_t3 : L.k_t3b)), uniform_ptr(ws + (c ? L.x1 : L.x2)),
                               uniform_ptr(ws + (c ? L.y1 : L.y2)), uniform_ptr(ws + (c ? L.z1 : L.z2)), fin);
  }
}

// ---- RFP / RFC: one refinement round (kkt_refine's loop body) of the pair / combined solves ---
// SET 0: the c- and affine solves (two right-hand sides), SET 1: the combined solve.  Round r
// runs when r < nref and the right-hand side has not stopped; the final W^-1 of dz follows in
// the next phase (AFF / UPD).
template <class X, int NX, int NU, int SET>
BMPC_HD void ph_refine(const X ex, const Ctx& C, int round) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* st = ws + L.ist;
  coup_load(ex, C);
  gdouble* e1 = ws + L.k_e1;
  gdouble* e2 = ws + L.k_e2;
  gdouble* e3 = ws + L.k_e3;
  gdouble* cx = ws + L.k_cx;
  gdouble* cy = ws + L.k_cy;
  gdouble* cz = ws + L.k_cz;
  gdouble* tv = ws + L.k_nv1;
  constexpr int NR = SET == 0 ? 2 : 1;
  for (int j = 0; j < NR; ++j) {
    const bool a = ex.uniform(SET == 0 && j == 1);   // the affine solve of the pair
    const gdouble* r1 = uniform_ptr(ws + (a ? L.ta2 : L.ta));
    const gdouble* r2 = uniform_ptr(ws + (SET == 1 ? L.ya : a ? L.ry : L.bvec));
    const gdouble* r3h = uniform_ptr(ws + (a ? L.k_t3b : L.k_t3));
    gdouble* dx = uniform_ptr(ws + (SET == 1 || a ? L.x2 : L.x1));
    gdouble* dy = uniform_ptr(ws + (SET == 1 || a ? L.y2 : L.y1));
    gdouble* dz = uniform_ptr(ws + (SET == 1 || a ? L.z2 : L.z1));
    double sc;
    if (ex.uniform(round == 0)) {
      sc = ex.max(fmax(fmax(strided_partial<8, 1>(ex.lane, ex.nlanes, P.nv, [&](int i) { return fabs(r1[i]); }),
                            strided_partial<8, 1>(ex.lane, ex.nlanes, P.neq, [&](int i) { return fabs(r2[i]); })),
                       strided_partial<8, 1>(ex.lane, ex.nlanes, P.nrows, [&](int i) { return fabs(r3h[i]); })));
    } else {
      sc = st[IS_SC0 + j];
      if (ph_flag(ex, st, IS_STOP0 + j)) continue;
    }
    // e1 = r1 - A'dy - G'W^-1 dzh, e2 = r2 - A dx
    apply_W(ex, C, 1, dz, e3);
    apply_GT<X, NX, NU>(ex, C, e3, tv);
    apply_AT<X, NX, NU>(ex, C, dy, e1);
    lane_batch<16>(ex, 0, P.nv, [&](int i) { return r1[i] - e1[i] - tv[i]; }, [&](int i, double v) { e1[i] = v; });
    apply_A<X, NX, NU>(ex, C, dx, e2);
    lane_batch(ex, 0, P.neq, [&](int i) { return r2[i] - e2[i]; }, [&](int i, double v) { e2[i] = v; });
    ex.sync();
    const double err = ex.max(fmax(strided_partial<8, 1>(ex.lane, ex.nlanes, P.nv, [&](int i) { return fabs(e1[i]); }),
                                   strided_partial<8, 1>(ex.lane, ex.nlanes, P.neq, [&](int i) { return fabs(e2[i]); })));
    const bool stop = ex.uniform(!(err > BMPC_REFTOL * fmax(sc, 1.0)));
    if (!stop) {
      kkt_solve_once<X, NX, NU, true>(ex, C, e1, e2, nullptr, cx, cy, cz, false, false);
      lane_batch<16>(ex, 0, P.nv, [&](int i) { return dx[i] + cx[i]; }, [&](int i, double v) { dx[i] = v; });
      lane_batch(ex, 0, P.neq, [&](int i) { return dy[i] + cy[i]; }, [&](int i, double v) { dy[i] = v; });
      lane_batch<16>(ex, 0, P.nrows, [&](int i) { return dz[i] + cz[i]; }, [&](int i, double v) { dz[i] = v; });
      ex.sync();
    }
    if (ex.lane == 0) {
      st[IS_SC0 + j] = sc;
      st[IS_STOP0 + j] = stop ? 1.0 : 0.0;
    }
  }
}

// ---- AFF: affine step, sigma, the combined right-hand side and its G'W^-1 (kkt_solve's head) --
template <class X, int NX, int NU>
BMPC_HD void ph_aff(const X ex, const Ctx& C) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* st = ws + L.ist;
  const int nv = P.nv, neq = P.neq, nr = P.nrows;
  gdouble* lam = ws + L.lam;
  gdouble* x1 = ws + L.x1;
  gdouble* y1 = ws + L.y1;
  gdouble* z1 = ws + L.z1;
  gdouble* x2 = ws + L.x2;
  gdouble* y2 = ws + L.y2;
  gdouble* z2 = ws + L.z2;
  gdouble* ds = ws + L.ds;
  gdouble* rx = ws + L.rx;
  gdouble* ry = ws + L.ry;
  gdouble* rz = ws + L.rz;
  gdouble* hv = ws + L.hvec;
  gdouble* bv = ws + L.bvec;
  gdouble* tA = ws + L.ta;
  gdouble* ya = ws + L.ya;
  gdouble* rb = ws + L.rb;
  if (ph_flag(ex, st, IS_NREF)) {   // kkt_refine's final dz = W^-1 dzh of the pair
    apply_W(ex, C, 1, z1, z1);
    apply_W(ex, C, 1, z2, z2);
  }
  const double tau = st[IS_TAU], kap = st[IS_KAP], rt = st[IS_RT], mu = st[IS_MU];
  const double den = kap / tau - (x1[P.oJ] + dot2(ex, bv, y1, neq, hv, z1, nr));
  const double dk_aff = -kap * tau;
  const double dtau_a = (rt + dk_aff / tau + x2[P.oJ] + dot2(ex, bv, y2, neq, hv, z2, nr)) / den;
  affine_dirs(ex, C, z2, z1, dtau_a, lam, rb, ds);
  const double dkap_a = (dk_aff - kap * dtau_a) / tau;
  double a_aff = max_step2(ex, C, lam, ds, rb);
  if (dtau_a < 0.0) a_aff = fmin(a_aff, -tau / dtau_a);
  if (dkap_a < 0.0) a_aff = fmin(a_aff, -kap / dkap_a);
  a_aff = fmax(0.0, fmin(a_aff, 0.999));
  double sigma = (1.0 - a_aff) * (1.0 - a_aff) * (1.0 - a_aff);
  sigma = fmin(1.0, fmax(1e-4, sigma));
  const double eta1 = 1.0 - sigma;
  combined_rhs(ex, C, lam, ds, rb, rz, sigma * mu, eta1);
  lane_batch<16>(ex, 0, nv, [&](int i) { return -eta1 * rx[i]; }, [&](int i, double v) { tA[i] = v; });
  lane_batch(ex, 0, neq, [&](int i) { return eta1 * ry[i]; }, [&](int i, double v) { ya[i] = v; });
  ex.sync();
  // kkt_solve(tA, ya, rb -> x2, y2, z2): r3h = W^-1 rb, then G'W^-1 r3h + r1 (kkt_solve_once)
  apply_Winv2(ex, C, rb, ws + L.k_t3, ws + L.k_r0);
  apply_GT<X, NX, NU>(ex, C, ws + L.k_r0, ws + L.k_nv0, tA);
  if (ex.lane == 0) {
    st[IS_DEN] = den;
    st[IS_DTAU_A] = dtau_a;
    st[IS_DKAP_A] = dkap_a;
    st[IS_SIGMA] = sigma;
    st[IS_ETA1] = eta1;
  }
}

// ---- CMB: the combined solve's tree solve and back half ----------------------------------------
template <class X, int NX, int NU>
BMPC_HD void ph_cmb(const X ex, const Ctx& C) {
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  const gdouble* st = ws + L.ist;
  coup_load(ex, C);
  const bool fin = ex.uniform(st[IS_NREF] == 0.0);
  gdouble* tz = ws + L.k_nv0;
  tree_solve<X, NX, NU>(ex, C, 1, tz, 0, ws + L.ya, 0, ws + L.x2, 0, ws + L.y2, 0);
  kkt_back<X, NX, NU, false>(ex, C, tz, ws + L.ya, ws + L.k_t3, ws + L.x2, ws + L.y2, ws + L.z2, fin);
}

// ---- UPD: the combined step and the update, or ECOS's backtrack to the best iterate ----------
// returns true when the ego goes on to the next iteration
template <class X, int NX, int NU>
BMPC_HD bool ph_upd(const X ex, const Ctx& C, int it) {
  CPlan& P = *C.P;
  CLayout& L = *C.L;
  gdouble* ws = C.ws;
  gdouble* st = ws + L.ist;
  const int nv = P.nv, neq = P.neq, nr = P.nrows;
  gdouble* x = ws + L.x;
  gdouble* y = ws + L.y;
  gdouble* z = ws + L.z;
  gdouble* s = ws + L.s;
  gdouble* lam = ws + L.lam;
  gdouble* x1 = ws + L.x1;
  gdouble* y1 = ws + L.y1;
  gdouble* z1 = ws + L.z1;
  gdouble* x2 = ws + L.x2;
  gdouble* y2 = ws + L.y2;
  gdouble* z2 = ws + L.z2;
  gdouble* ds = ws + L.ds;
  gdouble* hv = ws + L.hvec;
  gdouble* bv = ws + L.bvec;
  gdouble* rb = ws + L.rb;
  gdouble* rc = ws + L.rc;
  bool ok = ph_flag(ex, st, IS_OK);
  double tau = st[IS_TAU], kap = st[IS_KAP];
  if (ok) {
    if (ph_flag(ex, st, IS_NREF)) apply_W(ex, C, 1, z2, z2);   // kkt_refine's final W^-1
    const double rt = st[IS_RT], mu = st[IS_MU], den = st[IS_DEN], dtau_a = st[IS_DTAU_A];
    const double dkap_a = st[IS_DKAP_A], sigma = st[IS_SIGMA], eta1 = st[IS_ETA1];
    const double dk_c = -kap * tau - dtau_a * dkap_a + sigma * mu;
    const double dtau = (eta1 * rt + dk_c / tau + x2[P.oJ] + dot2(ex, bv, y2, neq, hv, z2, nr)) / den;
    double nonfinite = 0.0;
    lane_batch<8>(ex, 0, nv, [&](int i) { return x2[i] + (dtau * x1[i]); }, [&](int i, double v) {
      x2[i] = v;
      if (!isfinite(v)) nonfinite = 1.0;
    });
    lane_batch(ex, 0, neq, [&](int i) { return y2[i] + (dtau * y1[i]); }, [&](int i, double v) { y2[i] = v; });
    ex.sync();
    combined_dirs(ex, C, z2, z1, dtau, ds, rb, rc);
    const double dkap = (dk_c - kap * dtau) / tau;
    double a = max_step2(ex, C, lam, ds, rb);
    if (dtau < 0.0) a = fmin(a, -tau / dtau);
    if (dkap < 0.0) a = fmin(a, -kap / dkap);
    a = fmin(a, 0.999);
    const double alpha = a * 0.99;
    const double fin = ex.max(nonfinite);
    ok = ex.uniform(fin == 0.0 && isfinite(dtau) && alpha > 1e-10);
    if (ok) {
      lane_batch<8>(ex, 0, nv, [&](int i) { return x[i] + (alpha * x2[i]); }, [&](int i, double v) { x[i] = v; });
      lane_batch(ex, 0, neq, [&](int i) { return y[i] + (alpha * y2[i]); }, [&](int i, double v) { y[i] = v; });
      struct ZS { double z, s; };
      lane_batch<4>(ex, 0, nr, [&](int i) { return ZS{z[i] + alpha * z2[i], s[i] + alpha * rc[i]}; },
                    [&](int i, ZS v) { z[i] = v.z; s[i] = v.s; });
      tau += alpha * dtau;
      kap += alpha * dkap;
      ex.sync();
    }
  }
  if (ok) {
    if (ex.lane == 0) {
      st[IS_TAU] = tau;
      st[IS_KAP] = kap;
    }
    return true;
  }
  // numerical failure: ECOS backtracks to the best iterate
  const double best_score = st[IS_BEST], best_tau = st[IS_BEST_TAU];
  int code;
  double pc = st[IS_BS_PCOST];
  if (best_score < 1e300 && (ws[L.misc + MISC_BEST] != best_score || ws[L.misc + MISC_BEST + 1] != best_tau)) {
    code = EXIT_GUARD;
    pc = 0.0;
  } else {
    const double bs_relgap = st[IS_BS_RELGAP];
    const bool inacc = st[IS_BS_OKCX] != 0.0 && st[IS_BS_PRES] < 1e-4 && st[IS_BS_DRES] < 1e-4 &&
                       (st[IS_BS_GAP] < 5e-5 || (bs_relgap >= 0.0 && bs_relgap < 5e-5));
    lane_batch<16>(ex, 0, nv, [&](int i) { return ws[L.bestx + i] / best_tau; }, [&](int i, double v) { ws[L.sol + i] = v; });
    ex.sync();
    code = inacc ? EXIT_OPTIMAL + EXIT_INACC : EXIT_NUMERICS;
  }
  if (ex.lane == 0) {
    st[IS_EXIT] = (double)code;
    st[IS_ITERS] = (double)it;
    st[IS_PCOST] = pc;
    st[IS_ACTIVE] = 0.0;
  }
  return false;
}

// the solve's result from the state block
BMPC_HD IpmResult ph_result(const gdouble* st) {
  return IpmResult{(int)st[IS_EXIT], (int)st[IS_ITERS], st[IS_PCOST]};
}

// Whether the kernel of phase ph (iteration it) runs for this ego: the gate every k_ph kernel
// applies on entry (bmpc_dev_ph.h).
BMPC_HD bool ph_gate(const gdouble* st, int ph) {
  if (ph == PH_INIT1 || ph == PH_FIN) return true;
  if (ph == PH_INIT2 || ph == PH_INIT3) return st[IS_OK] != 0.0;
  if (ph == PH_RES || ph == PH_UPD) return st[IS_ACTIVE] != 0.0;
  if (!(st[IS_ACTIVE] != 0.0 && st[IS_OK] != 0.0)) return false;
  if (ph == PH_RFP0 || ph == PH_RFC0) return st[IS_NREF] > 0.0;
  if (ph == PH_RFP1 || ph == PH_RFC1) return st[IS_NREF] > 1.0;
  return true;
}

// One phase of one ego (the body of kernel k_ph<M, ph>; LDS constants / tables already set up).
// Returns false from UPD when the ego stops iterating.
template <class X, int NX, int NU>
BMPC_HD bool ph_run(const X ex, const Ctx& C, int ph, int it) {
  switch (ph) {
    case PH_INIT1: ph_init1<X, NX, NU>(ex, C); break;
    case PH_INIT2: ph_init2<X, NX, NU>(ex, C); break;
    case PH_INIT3: ph_init3<X, NX, NU>(ex, C); break;
    case PH_RES: ph_res<X, NX, NU>(ex, C, it); break;
    case PH_FAC: ph_fac<X, NX, NU>(ex, C); break;
    case PH_CPL: ph_cpl<X, NX, NU>(ex, C); break;
    case PH_BKP: ph_bkp<X, NX, NU>(ex, C); break;
    case PH_RFP0: ph_refine<X, NX, NU, 0>(ex, C, 0); break;
    case PH_RFP1: ph_refine<X, NX, NU, 0>(ex, C, 1); break;
    case PH_AFF: ph_aff<X, NX, NU>(ex, C); break;
    case PH_CMB: ph_cmb<X, NX, NU>(ex, C); break;
    case PH_RFC0: ph_refine<X, NX, NU, 1>(ex, C, 0); break;
    case PH_RFC1: ph_refine<X, NX, NU, 1>(ex, C, 1); break;
    case PH_UPD: return ph_upd<X, NX, NU>(ex, C, it);
    default: break;
  }
  return true;
}

// The phase sequence of one ego in the GPU's launch order (host build: checks the cut of
// ipm_solve into phases; every phase's LDS contents are scrambled first, as a new kernel's are).
template <class X, int NX, int NU>
BMPC_HD IpmResult ipm_solve_phased(const X ex, const Ctx& C, double* lds_scratch, int nlds) {
  CPlan& P = *C.P;
  const gdouble* st = C.ws + C.L->ist;
  auto run = [&](int ph, int it) {
    if (!ph_gate(st, ph)) return true;
    for (int i = P.nconst; i < nlds; ++i) lds_scratch[i] = 1.2345e300;   // nothing survives a kernel boundary
    return ph_run<X, NX, NU>(ex, C, ph, it);
  };
  run(PH_INIT1, 0);
  run(PH_INIT2, 0);
  run(PH_INIT3, 0);
  for (int it = 0; it <= P.desc.maxit; ++it) {
    run(PH_RES, it);
    if (it == P.desc.maxit || !(st[IS_ACTIVE] != 0.0)) break;
    for (int ph = PH_FAC; ph < PH_UPD; ++ph) run(ph, it);
    run(PH_UPD, it);
    if (!(st[IS_ACTIVE] != 0.0)) break;
  }
  return ph_result(st);
}

}  // namespace bmpc

namespace bmpc {

// host build: solve_ego_ipm through the phase sequence
template <class X, class M>
BMPC_HD IpmResult solve_ego_ipm_phased(const X& ex, const Plan& P, const Layout& L, EgoView E, double* lds, int nlds) {
  double* ws = E.ws;
  ipm_prelude<X, M>(ex, P, L, ws);
  ipm_eco<X, M>(ex, P, L, ws);
  Ctx C;
  C.P = (CPlan*)&P;
  C.L = (CLayout*)&L;
  C.ws = (gdouble*)ws;
  const IpmResult r = ipm_solve_phased<X, M::NX, M::NU>(ex, C, lds, nlds);
  ipm_unpack<X, M>(ex, P, L, ws, r);
  return r;
}

}  // namespace bmpc
