// bmpc_bandqp.h -- batched convex QP in OSQP's problem form
//
//     minimise 1/2 x'Px + q'x   subject to   l <= Ax <= u
//
// the solver behind the belief LTV-MPC (PredictiveControllers.MPC.osqp_solve_qp,
// PredictiveControllers.py:310-340, which builds a fresh OSQP object per solve).  OSQP's
// ADMM is not restated: like the oracle (oracle/qp_ipm.py) the kernel returns the QP optimum
// by a Mehrotra predictor-corrector interior-point method.
//
// Rows are split by the host (bmpc_qpplan.cpp) into equalities (l == u) and one-sided
// inequality copies (a'x <= u, -a'x <= -l).  Each Newton step solves the quasidefinite KKT
// system
//
//     [ P + rI    E'     G'         ] [dx]
//     [ E        -rI                ] [dy]   (r: static regularisation, removed again by
//     [ G               -S/Z - rI   ] [dz]    iterative refinement on the true matrix)
//
// whose LDL' factorisation exists in ANY symmetric ordering.  The host orders the KKT
// matrix by reverse Cuthill-McKee; an MPC's stage structure then leaves a narrow band
// (bandwidth bw), so the factorisation costs nk*bw^2/2 instead of nk^3/3.
//
// Execution: one 64-lane wave per problem.  The factorisation streams the band through a
// (bw+1) x (bw+1) ring window in LDS -- each rank-1 update touches only rows k+1..k+bw, so
// every band entry is read from HBM once per factorisation; the factor itself stays in LDS
// when it fits beside the window (nk*(bw+1) doubles: 100 KB for the belief MPC's 400 x 32
// band), so the triangular sweeps of the solves read LDS; the solve vector lives in LDS too.  Everything else is O(nk*bw) per iteration.  Vectors are kept in
// "KKT space" (the permuted index of the x, y and z blocks) so every IPM vector operation
// is one strided loop.
//
// Written once for the executor X (bmpc_core.h): libbmpc.so runs it with the device wave,
// tests/hostsim with the 1-lane host executor.
#pragma once

#include <type_traits>

#include "bmpc_core.h"

namespace bmpc {

// -DBMPC_BQP_PROF (device builds, experiments): s_memtime cycles of the factorisation, the
// triangular sweeps and the mat-vecs of problem 0, printed at the end of its solve
#if defined(BMPC_BQP_PROF) && defined(__HIP_DEVICE_COMPILE__)
__device__ unsigned long long g_bqp_prof[8];
#define BQP_TIC(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define BQP_TOC(i, v) \
  if (blockIdx.x == 0 && threadIdx.x == 0) g_bqp_prof[i] += __builtin_amdgcn_s_memtime() - (v)
#else
#define BQP_TIC(v) ((void)0)
#define BQP_TOC(i, v) ((void)0)
#endif

enum { QPK_X = 0, QPK_EQ = 1, QPK_IN = 2 };

#ifndef BMPC_BQP_NB
#define BMPC_BQP_NB 8   // columns per block of the one-wave blocked band factorisation
#endif

// problem statuses (OSQP's status_val codes where one exists)
enum { QP_SOLVED = 1, QP_MAX_ITER = -2, QP_NUMERICS = -8 };

// The symbolic part shared by every problem of a batch (one sparsity pattern, one row
// classification); pointers refer to device memory on the GPU, host memory in hostsim.
struct BandQPDesc {
  int32_t n, m;          // variables, rows of A
  int32_t nk, bw, W;     // KKT dimension, bandwidth after ordering, W = bw + 1
  int32_t n_in;          // inequality copies (mu normaliser)
  int32_t nvals, ncvals; // values per problem: [Px; Ax] and [q; l; u]
  int32_t nscat, ncscat; // entries of the two scatter lists
  int32_t max_iter;
  int32_t lb_lds;        // the factor L D L' lives in LDS (it fits beside the window), else in the workspace
  double eps;            // convergence tolerance (oracle/qp_ipm.py's tol)
  const int32_t* kind;   // [nk] QPK_* of each KKT row
  const int32_t* scat;   // [nscat][3]: src in [Px; Ax], band index dst, sign
  const int32_t* cscat;  // [ncscat][3]: src in [q; l; u], KKT index dst, sign
  const int32_t* xmap;   // [n] KKT index of x_j
  const int32_t* ymap;   // [m][4]: KKT index and sign of the eq / upper copy, of the lower copy (-1 none)
  size_t stride;         // workspace doubles per problem
};

// workspace of one problem (doubles)
struct BandQPWs {
  double *Kb, *Lb, *c, *w, *s, *r, *dw, *rhs, *t1, *t2, *fdg, *tdg, *ds;
};

BMPC_HD size_t bandqp_stride(int nk, int W) { return 2 * (size_t)nk * W + 11 * (size_t)nk; }
// LDS: the column of multipliers (W) and the solve vector (nk), then either the factorisation
// window (W*W; the factor goes to the workspace) or (lb_lds) the whole band, factored in
// place (nk*W): no row streamed from global memory inside the column loop, and the
// triangular sweeps of an iteration read LDS
// (lb_lds adds the row signs (nk) and the blocked factorisation's panel copies, 2 * 64 * NB)
BMPC_HD size_t bandqp_lds_doubles(int nk, int W, bool lb_lds) {
  return (size_t)W + nk + (lb_lds ? (size_t)nk * W + nk + 2 * 64 * BMPC_BQP_NB : (size_t)W * W);
}

BMPC_HD BandQPWs bandqp_ws(const BandQPDesc& d, double* base) {
  BandQPWs v;
  const size_t nk = d.nk, band = nk * d.W;
  v.Kb = base;
  v.Lb = base + band;
  double* p = base + 2 * band;
  double** vecs[] = {&v.c, &v.w, &v.s, &v.r, &v.dw, &v.rhs, &v.t1, &v.t2, &v.fdg, &v.tdg, &v.ds};
  for (double** q : vecs) {
    *q = p;
    p += nk;
  }
  return v;
}

// out = K v, K the symmetric band matrix Kb with its diagonal replaced by dg.  A lane's row
// loads are issued in chunks of 8 (band entry and vector entry, indices clamped and the extra
// terms masked by a zero factor), two rows at a time, so two rows cost bw / 4 memory round
// trips instead of 4 bw; each row's terms are added in the order of a plain row loop (lower
// part, then upper part; masked terms add exact zeros).
template <class X>
BMPC_HD void bqp_matvec(const X& ex, const BandQPDesc& d, const double* Kb, const double* dg, const double* v,
                        double* out) {
  const int nk = d.nk, W = d.W, bw = d.bw, nl = ex.nlanes;
  constexpr int CH = 8;
  BQP_TIC(t0);
  // two rows per lane per trip (i and i + nl; the second clamped to i and dropped when past
  // nk): their chunk loads are in flight together
  for (int i0 = ex.lane; i0 < nk; i0 += 2 * nl) {
    const bool two = i0 + nl < nk;
    const int ri[2] = {i0, two ? i0 + nl : i0};
    double a[2], e[2][CH], x[2][CH];
    int k0[2], k1[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = ri[h];
      a[h] = dg[i] * v[i];
      k0[h] = i < bw ? i : bw;
      k1[h] = nk - 1 - i < bw ? nk - 1 - i : bw;
    }
    for (int kb = 1; kb <= bw; kb += CH) {   // lower part: row i, columns i - k
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const bool in = kb + u <= k0[h];
          e[h][u] = Kb[(size_t)ri[h] * W + (in ? kb + u : 0)];
          x[h][u] = v[in ? ri[h] - kb - u : ri[h]];
        }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < CH; ++u) a[h] += e[h][u] * (x[h][u] * (kb + u <= k0[h] ? 1.0 : 0.0));
    }
    for (int kb = 1; kb <= bw; kb += CH) {   // upper part: column i of the rows i + k below
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const bool in = kb + u <= k1[h];
          e[h][u] = Kb[(size_t)(in ? ri[h] + kb + u : ri[h]) * W + (in ? kb + u : 0)];
          x[h][u] = v[in ? ri[h] + kb + u : ri[h]];
        }
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int u = 0; u < CH; ++u) a[h] += e[h][u] * (x[h][u] * (kb + u <= k1[h] ? 1.0 : 0.0));
    }
    out[ri[0]] = a[0];
    if (two) out[ri[1]] = a[1];
  }
  ex.sync();
  BQP_TOC(2, t0);
}

// Rank-1 update pattern of one column: entry (a, b), 0 <= b <= a < last, of the active
// rows' lower triangle, flattened t = a(a+1)/2 + b and dealt round-robin over the lanes (a
// lane per row would leave lane a with a+1 dependent updates, the others idle)
template <class X, class F>
BMPC_HD void bqp_tri_for(const X& ex, int last, F f) {
  const int ntri = last * (last + 1) / 2;
  int a = 0, b = ex.lane;
  while (b > a) {
    b -= a + 1;
    ++a;
  }
  for (int t = ex.lane; t < ntri; t += ex.nlanes) {
    f(a, b);
    b += ex.nlanes;
    while (b > a) {
      b -= a + 1;
      ++a;
    }
  }
}

// the pivot of column k: a pivot of the wrong sign or below 1e-13 in magnitude is replaced
// by +-2e-7 (ECOS's dynamic regularisation constants)
BMPC_HD double bqp_pivot(const BandQPDesc& d, int k, double dk) {
  const double sg = d.kind[k] == QPK_X ? 1.0 : -1.0;
  return sg * dk >= 1e-13 ? dk : sg * 2e-7;
}

// Band LDL' of Kb with diagonal fdg (the regularised one) into Lb: row i of Lb holds
// L[i][i-k] for k = 1..bw and D[i] at k = 0.  Right-looking, rows k..k+bw of the active
// submatrix resident in the LDS ring window; the row that enters the window after column k
// is loaded before the column's arithmetic (its latency hides behind it).
template <class X, class LP>
BMPC_HD void bqp_factor(const X& ex, const BandQPDesc& d, const double* Kb, const double* fdg, LP* Lb) {
  const int nk = d.nk, W = d.W, bw = d.bw, nl = ex.nlanes;
  auto* lv = ex.lds;
  auto* win = ex.lds + W + nk;
  const int rows0 = nk < W ? nk : W;
  for (int t = ex.lane; t < rows0 * W; t += nl) {
    const int i = t / W, k = t - i * W;
    win[t] = k == 0 ? fdg[i] : Kb[(size_t)i * W + k];   // row i sits in slot i (i < W)
  }
  ex.sync();
  for (int k = 0; k < nk; ++k) {
    const int slot = k % W, nxt = k + W;
    double pre = 0.0;   // this lane's entry c = lane of row nxt (W <= nlanes; else loaded at retirement)
    if (nxt < nk && ex.lane < W) pre = ex.lane == 0 ? fdg[nxt] : Kb[(size_t)nxt * W + ex.lane];
    const double dk = bqp_pivot(d, k, win[slot * W]);
    const int last = nk - 1 - k < bw ? nk - 1 - k : bw;   // rows k+1 .. k+last
    for (int a = ex.lane; a < last; a += nl) {
      const int si = (k + 1 + a) % W;
      const double l = win[si * W + a + 1] / dk;
      win[si * W + a + 1] = l;
      lv[a] = l;
    }
    ex.sync();
    bqp_tri_for(ex, last, [&](int a, int b) { win[((k + 1 + a) % W) * W + a - b] -= lv[a] * dk * lv[b]; });
    ex.sync();
    // row k is final: retire it to Lb and put row k + W into its slot
    for (int c = ex.lane; c < W; c += nl) {
      Lb[(size_t)k * W + c] = c == 0 ? dk : win[slot * W + c];
      if (nxt < nk) win[slot * W + c] = c < nl ? pre : (c == 0 ? fdg[nxt] : Kb[(size_t)nxt * W + c]);
    }
    ex.sync();
  }
}

// The same factorisation with the whole band in LDS (lb_lds), factored in place: one copy
// in, then per column the multipliers and the rank-1 update, all LDS.
template <class X, class LP>
BMPC_HD void bqp_factor_lds(const X& ex, const BandQPDesc& d, const double* Kb, const double* fdg, LP* L) {
  const int nk = d.nk, W = d.W, bw = d.bw, nl = ex.nlanes;
  auto* lv = ex.lds;
  for (size_t t = ex.lane; t < (size_t)nk * W; t += nl) {
    const size_t i = t / W;
    L[t] = t == i * W ? fdg[i] : Kb[t];
  }
  ex.sync();
  for (int k = 0; k < nk; ++k) {
    const double dk = bqp_pivot(d, k, L[(size_t)k * W]);
    const int last = nk - 1 - k < bw ? nk - 1 - k : bw;
    for (int a = ex.lane; a < last; a += nl) {
      LP* e = L + (size_t)(k + 1 + a) * W + a + 1;
      const double l = *e / dk;
      *e = l;
      lv[a] = l;
    }
    if (ex.lane == 0) L[(size_t)k * W] = dk;
    ex.sync();
    bqp_tri_for(ex, last, [&](int a, int b) { L[(size_t)(k + 1 + a) * W + a - b] -= lv[a] * dk * lv[b]; });
    ex.sync();
  }
}

// out = (L D L')^{-1} b; column sweeps on the LDS solve vector
template <class X, class LP>
BMPC_HD void bqp_ldl_solve(const X& ex, const BandQPDesc& d, const LP* Lb, const double* b, double* out) {
  const int nk = d.nk, W = d.W, bw = d.bw, nl = ex.nlanes;
  auto* y = ex.lds + W;
  for (int i = ex.lane; i < nk; i += nl) y[i] = b[i];
  ex.sync();
  for (int k = 0; k < nk; ++k) {            // L y = b
    const double yk = y[k];
    const int last = nk - 1 - k < bw ? nk - 1 - k : bw;
    for (int a = 1 + ex.lane; a <= last; a += nl) y[k + a] -= Lb[(size_t)(k + a) * W + a] * yk;
    ex.sync();
  }
  for (int i = ex.lane; i < nk; i += nl) y[i] /= Lb[(size_t)i * W];
  ex.sync();
  for (int k = nk - 1; k > 0; --k) {        // L' x = y
    const double xk = y[k];
    const int last = k < bw ? k : bw;
    for (int a = 1 + ex.lane; a <= last; a += nl) y[k - a] -= Lb[(size_t)k * W + a] * xk;
    ex.sync();
  }
  for (int i = ex.lane; i < nk; i += nl) out[i] = y[i];
  ex.sync();
}

// out = K^{-1} b for the true matrix (Kb, diagonal tdg) through its regularised factor:
// up to three refinement steps, stopping at a 1e-15 relative residual (oracle/qp_ipm.py).
template <class X, class LP>
BMPC_HD void bqp_ldl_solve_any(const X& ex, const BandQPDesc& d, const LP* Lb, const double* b, double* out);

template <class X, class LP>
BMPC_HD void bqp_solve_refined(const X& ex, const BandQPDesc& d, const BandQPWs& v, const LP* Lb, const double* b,
                               double* out) {
  bqp_ldl_solve_any(ex, d, Lb, b, out);
  double bn = 0.0;
  for (int i = ex.lane; i < d.nk; i += ex.nlanes) bn = fmax(bn, fabs(b[i]));
  bn = ex.max(bn);
  for (int it = 0; it < 3; ++it) {
    bqp_matvec(ex, d, v.Kb, v.tdg, out, v.t1);
    double rn = 0.0;
    for (int i = ex.lane; i < d.nk; i += ex.nlanes) {
      v.t1[i] = b[i] - v.t1[i];
      rn = fmax(rn, fabs(v.t1[i]));
    }
    rn = ex.max(rn);
    ex.sync();
    if (rn < 1e-15 * fmax(1.0, bn)) break;
    bqp_ldl_solve_any(ex, d, Lb, v.t1, v.t2);
    for (int i = ex.lane; i < d.nk; i += ex.nlanes) out[i] += v.t2[i];
    ex.sync();
  }
}

// largest step in (0, 1] keeping s + a ds >= 0 and z + a dz >= 0 over the inequality rows
template <class X>
BMPC_HD double bqp_step(const X& ex, const BandQPDesc& d, const BandQPWs& v) {
  double a = 1.0;
  for (int i = ex.lane; i < d.nk; i += ex.nlanes) {
    if (d.kind[i] != QPK_IN) continue;
    if (v.ds[i] < 0) a = fmin(a, -v.s[i] / v.ds[i]);
    if (v.dw[i] < 0) a = fmin(a, -v.w[i] / v.dw[i]);
  }
  return ex.min(a);
}

// ---- one wave, band in LDS: blocked factorisation and sweeps ------------------------------
// The column-at-a-time kernels above chain two barriers and an LDS round trip per column (and
// per row of each sweep): one problem's solve is that chain, 20 ms for the belief MPC.  On a
// single 64-lane wave (executors with kBqpWave) the band is processed in blocks of kBqpNB
// columns: lane r holds row k0 + r of the block's kBqpNB + bw rows in registers, the block's
// own column chain runs on wave broadcasts (readlane, no barrier), and the rest of the block's
// work is one LDS pass.  Every entry receives the same updates in the same order as in the
// column-at-a-time kernels (host build), so the factor and the solutions are the same numbers.
constexpr int kBqpNB = BMPC_BQP_NB;
template <class X, class = void>
struct BqpWave : std::false_type {};
template <class X>
struct BqpWave<X, std::void_t<decltype(X::kBqpWave)>> : std::integral_constant<bool, X::kBqpWave> {};

template <class X>
BMPC_HD bool bqp_use_blk(const X&, const BandQPDesc& d) {
  if constexpr (BqpWave<X>::value) return d.lb_lds && d.bw + kBqpNB <= 64;
  else return false;
}

// LDS areas of the in-LDS layout: L (nk*W) after the multipliers (W) and the solve vector (nk),
// then the row signs (nk), then the panel multipliers Pl and their pivot products Pw (64 x NB each)
template <class X>
BMPC_HD auto bqp_lds_sg(const X& ex, const BandQPDesc& d) { return ex.lds + d.W + d.nk + (size_t)d.nk * d.W; }

template <class X, class LP>
BMPC_HD void bqp_factor_blk(const X& ex, const BandQPDesc& d, const double* Kb, const double* fdg, LP* L) {
  constexpr int NB = kBqpNB;
  const int nk = d.nk, W = d.W, bw = d.bw, r = ex.lane;
  const auto* sg = bqp_lds_sg(ex, d);
  auto* Pl = bqp_lds_sg(ex, d) + nk;
  auto* Pw = Pl + 64 * NB;
  // the band in, loads batched 16 per lane (a load per loop trip would be a round trip each),
  // then the regularised diagonal over it
  lane_batch<16>(ex, 0, nk * W, [&](int t) { return Kb[t]; }, [&](int t, double v) { L[t] = v; });
  ex.sync();
  lane_batch<16>(ex, 0, nk, [&](int i) { return fdg[i]; }, [&](int i, double v) { L[(size_t)i * W] = v; });
  ex.sync();
  for (int k0 = 0; k0 < nk; k0 += NB) {
    const int nb = nk - k0 < NB ? nk - k0 : NB;
    const int nrow = nk - k0 < NB + bw ? nk - k0 : NB + bw;
    const bool act = r < nrow;
    const size_t rowW = (size_t)(act ? k0 + r : k0) * W;
    // this lane's panel row: entry (k0 + r, k0 + j) at offset r - j (band and lower part only)
    double a[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int off = r - j;
      const bool in = act && j < nb && off >= 0 && off <= bw;
      const double v = L[rowW + (in ? off : 0)];   // unconditional load, masked by arithmetic
      a[j] = in ? v : 0.0;
    }
    const double sgr = act ? (double)sg[k0 + r] : 1.0;
    BQP_TIC(tp);
    double dj_[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (j < nb) {   // wave-uniform
        double dj = ex.rlane(a[j], j);
        const double sj = ex.rlane(sgr, j);
        if (!(sj * dj >= 1e-13)) dj = sj * 2e-7;
        dj_[j] = dj;
        const double l = r > j ? a[j] / dj : 0.0;
        a[j] = r > j ? l : (r == j ? dj : a[j]);
        // rows above jj update an upper-triangle slot of column jj that is never read or
        // written back, and columns past nb are never written back: no lane condition
#pragma unroll
        for (int jj = j + 1; jj < NB; ++jj) {
          const double ljj = ex.rlane(l, jj);
          a[jj] -= l * dj * ljj;
        }
      } else {
        dj_[j] = 0.0;
      }
    }
    // panel back to the band; rows past the block keep copies for the trailing update
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int off = r - j;
      if (act && j < nb && off >= 0 && off <= bw) L[rowW + off] = a[j];
      const bool below = act && r >= NB && j < nb && off <= bw;
      Pl[j * 64 + r] = below ? a[j] : 0.0;   // column-major: lanes of consecutive rows hit consecutive banks
      Pw[j * 64 + r] = below ? a[j] * dj_[j] : 0.0;
    }
    ex.sync();
    BQP_TOC(4, tp);
    BQP_TIC(tt);
    // trailing update of rows / columns k0+NB .. k0+nrow-1 (all inside the band):
    // entry (p, c) -= sum_j (l_pj d_j) l_cj, j in column order
    bqp_tri_for(ex, nrow > NB ? nrow - NB : 0, [&](int pp, int cc) {
      const int p = NB + pp, c = NB + cc;
      LP* e = L + (size_t)(k0 + p) * W + (p - c);
      double v = *e;
#pragma unroll
      for (int j = 0; j < NB; ++j) v -= Pw[j * 64 + p] * Pl[j * 64 + c];
      *e = v;
    });
    ex.sync();
    BQP_TOC(5, tt);
  }
}

// out = (L D L')^{-1} b with the factor in LDS: both sweeps in blocks of kBqpNB rows
template <class X, class LP>
BMPC_HD void bqp_ldl_solve_blk(const X& ex, const BandQPDesc& d, const LP* L, const double* b, double* out) {
  constexpr int NB = kBqpNB;
  const int nk = d.nk, W = d.W, bw = d.bw, r = ex.lane;
  auto* y = ex.lds + W;
  lane_batch<16>(ex, 0, nk, [&](int i) { return b[i]; }, [&](int i, double v) { y[i] = v; });
  ex.sync();
  BQP_TIC(tf);
  for (int k0 = 0; k0 < nk; k0 += NB) {   // L y = b
    const int nb = nk - k0 < NB ? nk - k0 : NB;
    const int nrow = nk - k0 < NB + bw ? nk - k0 : NB + bw;
    const bool act = r < nrow;
    const int row = act ? k0 + r : k0;
    double acc = y[row];
    double lr[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int off = r - j;
      const bool in = act && j < nb && off > 0 && off <= bw;
      const double v = L[(size_t)row * W + (in ? off : 0)];
      lr[j] = in ? v : 0.0;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) acc -= lr[j] * ex.rlane(acc, j);   // lr = 0 off the band / above row j
    if (act) y[row] = acc;
    ex.sync();
  }
  BQP_TOC(6, tf);
  for (int i = r; i < nk; i += 64) y[i] /= L[(size_t)i * W];
  ex.sync();
  BQP_TIC(tb);
  for (int k1 = nk - 1; k1 > 0; k1 -= NB) {   // L' x = y, rows k1, k1 - 1, ... of the block
    const int nb = k1 + 1 < NB ? k1 + 1 : NB;
    const int nrow = k1 + 1 < NB + bw ? k1 + 1 : NB + bw;
    const bool act = r < nrow;
    const int row = act ? k1 - r : k1;
    double acc = y[row];
    double lr[NB];   // L[k1 - j][offset r - j]: the entry of row k1 - j in column k1 - r
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int off = r - j;
      const bool in = act && j < nb && off > 0 && off <= bw;
      const double v = L[(size_t)(in ? k1 - j : k1) * W + (in ? off : 0)];
      lr[j] = in ? v : 0.0;
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) acc -= lr[j] * ex.rlane(acc, j);
    if (act) y[row] = acc;
    ex.sync();
  }
  BQP_TOC(7, tb);
  lane_batch<16>(ex, 0, nk, [&](int i) { return (double)y[i]; }, [&](int i, double v) { out[i] = v; });
  ex.sync();
}

template <class X, class LP>
BMPC_HD void bqp_ldl_solve_any(const X& ex, const BandQPDesc& d, const LP* Lb, const double* b, double* out) {
  BQP_TIC(t0);
  if constexpr (BqpWave<X>::value) {
    if (bqp_use_blk(ex, d)) bqp_ldl_solve_blk(ex, d, Lb, b, out);
    else bqp_ldl_solve(ex, d, Lb, b, out);
  } else {
    bqp_ldl_solve(ex, d, Lb, b, out);
  }
  BQP_TOC(1, t0);
}

template <bool InLds, class X, class LP>
BMPC_HD void bqp_factor_any(const X& ex, const BandQPDesc& d, const double* Kb, const double* fdg, LP* Lb) {
  BQP_TIC(t0);
  if constexpr (InLds) {
    if constexpr (BqpWave<X>::value) {
      if (bqp_use_blk(ex, d)) bqp_factor_blk(ex, d, Kb, fdg, Lb);
      else bqp_factor_lds(ex, d, Kb, fdg, Lb);
    } else {
      bqp_factor_lds(ex, d, Kb, fdg, Lb);
    }
  } else {
    bqp_factor(ex, d, Kb, fdg, Lb);
  }
  BQP_TOC(0, t0);
}

template <bool InLds, class X, class LP>
BMPC_HD int bandqp_solve_t(const X& ex, const BandQPDesc& d, const double* vals, const double* cvals, double* ws,
                           LP* Lb, double* x, double* y, int* iters) {
  const int nk = d.nk, nl = ex.nlanes, lane = ex.lane;
  const BandQPWs v = bandqp_ws(d, ws);
  const double rs = 1e-8;   // static regularisation (ECOS's STATIC_REG)
  BQP_TIC(t_all);
  if (bqp_use_blk(ex, d)) {   // row signs of the pivot rule, for the blocked factorisation
    auto* sg = bqp_lds_sg(ex, d);
    for (int i = lane; i < nk; i += nl) sg[i] = d.kind[i] == QPK_X ? 1.0 : -1.0;
  }
  // ---- assemble the band and the right-hand-side constants c (q | e | g by row kind)
  for (size_t t = lane; t < (size_t)nk * d.W; t += nl) v.Kb[t] = 0.0;
  for (int i = lane; i < nk; i += nl) v.c[i] = 0.0;
  ex.sync();
  for (int t = lane; t < d.nscat; t += nl) v.Kb[d.scat[3 * t + 1]] = d.scat[3 * t + 2] * vals[d.scat[3 * t]];
  for (int t = lane; t < d.ncscat; t += nl) v.c[d.cscat[3 * t + 1]] = d.cscat[3 * t + 2] * cvals[d.cscat[3 * t]];
  ex.sync();
  double nq = 0.0, ne = 0.0, ng = 0.0;
  for (int i = lane; i < nk; i += nl) {
    const int kd = d.kind[i];
    const double a = fabs(v.c[i]);
    if (kd == QPK_X) nq = fmax(nq, a); else if (kd == QPK_EQ) ne = fmax(ne, a); else ng = fmax(ng, a);
  }
  nq = fmax(1.0, ex.max(nq));
  ne = fmax(1.0, ex.max(ne));
  ng = fmax(1.0, ex.max(ng));

  // ---- initial point: solve with S/Z = I, then shift s into the interior (oracle/qp_ipm.py:51-56)
  for (int i = lane; i < nk; i += nl) {
    const int kd = d.kind[i];
    const double pd = kd == QPK_X ? v.Kb[(size_t)i * d.W] : 0.0;
    v.tdg[i] = kd == QPK_X ? pd : (kd == QPK_EQ ? 0.0 : -1.0);
    v.fdg[i] = kd == QPK_X ? pd + rs : v.tdg[i] - rs;
    v.rhs[i] = kd == QPK_X ? -v.c[i] : v.c[i];
  }
  ex.sync();
  bqp_factor_any<InLds>(ex, d, v.Kb, v.fdg, Lb);
  bqp_solve_refined(ex, d, v, Lb, v.rhs, v.w);
  for (int i = lane; i < nk; i += nl) {
    v.t2[i] = d.kind[i] == QPK_X ? v.w[i] : 0.0;
    v.fdg[i] = d.kind[i] == QPK_X ? v.Kb[(size_t)i * d.W] : 0.0;   // diagonal of [P E' G'; E 0 0; G 0 0]
  }
  ex.sync();
  bqp_matvec(ex, d, v.Kb, v.fdg, v.t2, v.r);   // z rows: G x
  double smin = 1e300;
  for (int i = lane; i < nk; i += nl)
    if (d.kind[i] == QPK_IN) {
      v.s[i] = v.c[i] - v.r[i];
      smin = fmin(smin, v.s[i]);
    } else {
      v.s[i] = 0.0;
    }
  smin = ex.min(smin);
  const double shift = (d.n_in > 0 ? fmax(0.0, -smin) : 0.0) + 1.0;
  for (int i = lane; i < nk; i += nl)
    if (d.kind[i] == QPK_IN) {
      v.s[i] += shift;
      v.w[i] = fmax(fabs(v.w[i]), 1.0);
    }
  ex.sync();

  int status = QP_MAX_ITER, it = 0;
  const double inv_m = d.n_in > 0 ? 1.0 / d.n_in : 0.0;
  for (it = 0; it < d.max_iter; ++it) {
    // ---- residuals: rd = Px + q + E'y + G'z, re = Ex - e, rg = Gx + s - g, mu
    for (int i = lane; i < nk; i += nl) v.fdg[i] = d.kind[i] == QPK_X ? v.Kb[(size_t)i * d.W] : 0.0;
    ex.sync();
    bqp_matvec(ex, d, v.Kb, v.fdg, v.w, v.r);
    double rd = 0.0, re = 0.0, rg = 0.0, sz = 0.0;
    for (int i = lane; i < nk; i += nl) {
      const int kd = d.kind[i];
      if (kd == QPK_X) {
        v.r[i] += v.c[i];
        rd = fmax(rd, fabs(v.r[i]));
      } else if (kd == QPK_EQ) {
        v.r[i] -= v.c[i];
        re = fmax(re, fabs(v.r[i]));
      } else {
        v.r[i] += v.s[i] - v.c[i];
        rg = fmax(rg, fabs(v.r[i]));
        sz += v.s[i] * v.w[i];
      }
    }
    rd = ex.max(rd);
    re = ex.max(re);
    rg = ex.max(rg);
    const double mu = ex.sum(sz) * inv_m;
    ex.sync();
    if (!(rd == rd) || !(mu == mu) || !(rg == rg) || !(re == re)) {
      status = QP_NUMERICS;
      break;
    }
    double sn = 0.0;   // |s|: the inequality residual's scale, as in oracle/qp_ipm.py
    for (int i = lane; i < nk; i += nl)
      if (d.kind[i] == QPK_IN) sn = fmax(sn, fabs(v.s[i]));
    sn = ex.max(sn);
    if (rd < d.eps * nq && re < d.eps * ne && rg < d.eps * fmax(ng, sn) && mu < d.eps) {
      status = QP_SOLVED;
      break;
    }
    // ---- factor the Newton matrix (diagonal -S/Z on the inequality rows)
    for (int i = lane; i < nk; i += nl) {
      const int kd = d.kind[i];
      const double pd = kd == QPK_X ? v.Kb[(size_t)i * d.W] : 0.0;
      v.tdg[i] = kd == QPK_X ? pd : (kd == QPK_EQ ? 0.0 : -v.s[i] / v.w[i]);
      v.fdg[i] = kd == QPK_X ? pd + rs : v.tdg[i] - rs;
      v.rhs[i] = kd == QPK_IN ? -v.r[i] + v.s[i] : -v.r[i];
    }
    ex.sync();
    bqp_factor_any<InLds>(ex, d, v.Kb, v.fdg, Lb);
    // ---- predictor (affine) step
    bqp_solve_refined(ex, d, v, Lb, v.rhs, v.dw);
    for (int i = lane; i < nk; i += nl)
      v.ds[i] = d.kind[i] == QPK_IN ? -v.s[i] - v.s[i] / v.w[i] * v.dw[i] : 0.0;
    ex.sync();
    const double aa = bqp_step(ex, d, v);
    double sa = 0.0;
    for (int i = lane; i < nk; i += nl)
      if (d.kind[i] == QPK_IN) sa += (v.s[i] + aa * v.ds[i]) * (v.w[i] + aa * v.dw[i]);
    const double mua = ex.sum(sa) * inv_m;
    const double sig = mu > 0 ? (mua / mu) * (mua / mu) * (mua / mu) : 0.0;
    // ---- corrector: rhs of the inequality rows gains (ds dz - sig mu) / z; t2 keeps that term
    for (int i = lane; i < nk; i += nl)
      if (d.kind[i] == QPK_IN) {
        const double corr = (v.ds[i] * v.dw[i] - sig * mu) / v.w[i];
        v.t2[i] = corr;
        v.rhs[i] += corr;
      }
    ex.sync();
    // t2 is the refinement scratch: stash corr in ds first
    for (int i = lane; i < nk; i += nl) v.ds[i] = d.kind[i] == QPK_IN ? v.t2[i] : 0.0;
    ex.sync();
    bqp_solve_refined(ex, d, v, Lb, v.rhs, v.dw);
    for (int i = lane; i < nk; i += nl)
      if (d.kind[i] == QPK_IN) v.ds[i] = -v.s[i] - v.s[i] / v.w[i] * v.dw[i] - v.ds[i];
    ex.sync();
    const double a = 0.99 * bqp_step(ex, d, v);
    for (int i = lane; i < nk; i += nl) {
      v.w[i] += a * v.dw[i];
      if (d.kind[i] == QPK_IN) v.s[i] += a * v.ds[i];
    }
    ex.sync();
  }
  for (int j = lane; j < d.n; j += nl) x[j] = v.w[d.xmap[j]];
  for (int r = lane; r < d.m; r += nl) {
    const int32_t* ym = d.ymap + 4 * r;
    double yr = 0.0;
    if (ym[0] >= 0) yr += ym[1] * v.w[ym[0]];
    if (ym[2] >= 0) yr += ym[3] * v.w[ym[2]];
    y[r] = yr;
  }
  if (iters && lane == 0) *iters = it;
  ex.sync();
  BQP_TOC(3, t_all);
#if defined(BMPC_BQP_PROF) && defined(__HIP_DEVICE_COMPILE__)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    printf("bqp prof (cycles): factor %llu (panel %llu trailing %llu)  ldl_solve %llu (fwd %llu bwd %llu)  matvec %llu  "
           "total %llu  iters %d\n", g_bqp_prof[0], g_bqp_prof[4], g_bqp_prof[5], g_bqp_prof[1], g_bqp_prof[6],
           g_bqp_prof[7], g_bqp_prof[2], g_bqp_prof[3], it);
    for (int i = 0; i < 8; ++i) g_bqp_prof[i] = 0;
  }
#endif
  return status;
}

// One problem.  vals = [Px; Ax], cvals = [q; l; u] (the CSC value arrays of the shared
// pattern); x [n], y [m] (OSQP's dual: P x + q + A'y = 0); returns the QP_* status.
template <class X>
BMPC_HD int bandqp_solve(const X& ex, const BandQPDesc& d, const double* vals, const double* cvals, double* ws,
                         double* x, double* y, int* iters) {
  if (d.lb_lds) return bandqp_solve_t<true>(ex, d, vals, cvals, ws, ex.lds + d.W + d.nk, x, y, iters);
  return bandqp_solve_t<false>(ex, d, vals, cvals, ws, bandqp_ws(d, ws).Lb, x, y, iters);
}

}  // namespace bmpc
