// mb_riccati.hip -- microbenchmark of the tree Riccati factorisation plus one backward sweep
// for 4096 headline egos (highway N=20, NB=1, m=3: a root node and three child branches of 20
// input nodes, T = 64 state / U = 61 input nodes, n = 4, d = 2), three ways (round-4 verdict
// item 5).  Tools-only: not part of libbmpc.so.
//
//   aos   : the shipped mapping -- one wave per ego over an ego-major slab, one DPP quad per
//           branch (lane = state row), node rows gathered by quad broadcasts
//           (bmpc_ipm.h kkt_factor / bw_node);
//   soa   : 16 egos interleaved per wave (structure of arrays in blocks of 16 egos, so one
//           wave-wide load reads whole 128-B lines of 16 egos), one quad per ego running its
//           three child branches in turn, the same per-node VALU arithmetic;
//   mfma  : the soa layout with the 4x4 and 4x2 block products on v_mfma_f64_4x4x4f64 (four
//           4x4x4 blocks per instruction = four egos; one wave = four groups of four egos).
//   *_pf  : the same with the next node's data loaded before the current node's arithmetic
//           (the addresses do not depend on the recursion).
//
// Per node (FP64): Riccati  M = Pb A, P = Hx + A'M, Qux = B'M, Quu = Hu + B'Pb B, Quu^-1,
// K = -Quu^-1 Qux, P += Qux'K, symmetrise; sweep  ru = r + B'g, kf = -Quu^-1 ru,
// l = q + A'g + K'ru.  Branch ends merge the children's first-node P / l (MPC_branch.py:1766-1787
// is the dynamics these recursions factor).  Every variant's root P / l are checked against the
// aos variant's.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_riccati tools/mb_riccati.hip
// run:   tools/mb_riccati [variant|all] [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int NX = 4, NU = 2, NCH = 3, NLEN = 20;
constexpr int T = 1 + NCH * (NLEN + 1), U = 1 + NCH * NLEN;   // 64, 61
constexpr int EGOS = 4096, BLK = 16;
// per-ego arrays (doubles): inputs, then outputs
constexpr int O_HX = 0, O_HU = O_HX + T * 16, O_A = O_HU + U * 4, O_B = O_A + U * 16, O_Q = O_B + U * 8,
              O_R = O_Q + T * 4, O_P = O_R + U * 2, O_K = O_P + T * 16, O_QI = O_K + U * 8, O_L = O_QI + U * 4,
              O_KF = O_L + T * 4, STRIDE = O_KF + U * 2;
// node numbering: x node 0 / u node 0 = root; child c, step j: u node 1 + c*NLEN + j,
// x node 1 + c*(NLEN+1) + j (x node j+1 of the branch is u node j's successor; j = NLEN terminal)
__host__ __device__ inline int xnode(int c, int j) { return 1 + c * (NLEN + 1) + j; }
__host__ __device__ inline int unode(int c, int j) { return 1 + c * NLEN + j; }

// address of entry `off` of ego e
struct AoS {
  __device__ size_t operator()(int e, int off) const { return (size_t)e * STRIDE + off; }
};
struct SoA {
  __device__ size_t operator()(int e, int off) const {
    return (size_t)(e / BLK) * STRIDE * BLK + (size_t)off * BLK + (e % BLK);
  }
};

__host__ __device__ inline double hval(unsigned a, unsigned b) {
  unsigned x = a * 2654435761u ^ (b + 0x9e3779b9u + (a << 6) + (a >> 2));
  x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
  return (x & 0xffffff) / double(0x1000000);   // [0, 1)
}

template <class AD>
__global__ void k_init(double* w, AD ad) {
  const int e = blockIdx.x;
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) {
        const double v = i == j ? 1.0 + hval(e, t * 97 + i) : 0.05 * (hval(e, t * 131 + i + j) - 0.5);
        w[ad(e, O_HX + t * 16 + i * 4 + j)] = v;   // symmetric (hash of i + j), diagonally dominant
      }
    for (int i = 0; i < NX; ++i) w[ad(e, O_Q + t * 4 + i)] = hval(e, t * 53 + i + 7) - 0.5;
  }
  for (int u = threadIdx.x; u < U; u += blockDim.x) {
    w[ad(e, O_HU + u * 4 + 0)] = 2.0 + hval(e, u * 11);
    w[ad(e, O_HU + u * 4 + 1)] = w[ad(e, O_HU + u * 4 + 2)] = 0.1 * (hval(e, u * 13) - 0.5);
    w[ad(e, O_HU + u * 4 + 3)] = 2.0 + hval(e, u * 17);
    for (int i = 0; i < NX; ++i)
      for (int j = 0; j < NX; ++j) w[ad(e, O_A + u * 16 + i * 4 + j)] = (i == j) + 0.1 * (hval(e, u * 19 + i * 4 + j) - 0.5);
    for (int i = 0; i < NX; ++i)
      for (int m = 0; m < NU; ++m) w[ad(e, O_B + u * 8 + i * 2 + m)] = 0.1 * hval(e, u * 23 + i * 2 + m);
    for (int m = 0; m < NU; ++m) w[ad(e, O_R + u * 2 + m)] = hval(e, u * 29 + m) - 0.5;
  }
}

// ---------------------------------------------------------------------------------------
// quad (VALU) versions: lane gl of a DPP quad owns row gl of the node matrices
// ---------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int S>
__device__ __forceinline__ double qget(double v) { return dpp_d<S | (S << 2) | (S << 4) | (S << 6)>(v); }
__device__ __forceinline__ double qsum(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  return v;
}
__device__ __forceinline__ void qgather(const double (&mine)[NX], double (&full)[NX][NX]) {
#pragma unroll
  for (int c = 0; c < NX; ++c) {
    full[0][c] = qget<0>(mine[c]);
    full[1][c] = qget<1>(mine[c]);
    full[2][c] = qget<2>(mine[c]);
    full[3][c] = qget<3>(mine[c]);
  }
}

struct NodeRic {   // this lane's part of a Riccati node's inputs
  double hx[NX], ar[NX], ac[NX], br[NU], hu[4];
};
template <class AD>
__device__ __forceinline__ void load_ric(const double* w, const AD& ad, int e, int gl, int xk, int u, NodeRic& d) {
#pragma unroll
  for (int j = 0; j < NX; ++j) d.hx[j] = w[ad(e, O_HX + xk * 16 + gl * 4 + j)];
#pragma unroll
  for (int j = 0; j < NX; ++j) d.ar[j] = w[ad(e, O_A + u * 16 + gl * 4 + j)];
#pragma unroll
  for (int j = 0; j < NX; ++j) d.ac[j] = w[ad(e, O_A + u * 16 + j * 4 + gl)];
#pragma unroll
  for (int m = 0; m < NU; ++m) d.br[m] = w[ad(e, O_B + u * 8 + gl * 2 + m)];
#pragma unroll
  for (int m = 0; m < 4; ++m) d.hu[m] = w[ad(e, O_HU + u * 4 + m)];
}

// one Riccati node: Pb (own row) -> P (own row), stores P, K, Quu^-1
template <class AD>
__device__ __forceinline__ void quad_ric(double* w, const AD& ad, int e, int gl, int xk, int u, const NodeRic& d,
                                         const double (&Pb)[NX], double (&Pn)[NX]) {
  double Af[NX][NX], Bf[NX][NX], Mf[NX][NX], PBf[NX][NX];
  qgather(d.ar, Af);
  double bpad[NX] = {d.br[0], d.br[1], 0.0, 0.0};
  qgather(bpad, Bf);
  double Mr[NX];
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < NX; ++r) v += Pb[r] * Af[r][j];
    Mr[j] = v;
  }
  qgather(Mr, Mf);
  double Pk[NX];
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < NX; ++r) v += d.ac[r] * Mf[r][j];
    Pk[j] = d.hx[j] + v;
  }
  double Qux[NU][NX];
#pragma unroll
  for (int m = 0; m < NU; ++m)
#pragma unroll
    for (int j = 0; j < NX; ++j) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < NX; ++r) v += Bf[r][m] * Mf[r][j];
      Qux[m][j] = v;
    }
  double PBr[NX] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int m = 0; m < NU; ++m) {
    double v = 0.0;
#pragma unroll
    for (int c = 0; c < NX; ++c) v += Pb[c] * Bf[c][m];
    PBr[m] = v;
  }
  qgather(PBr, PBf);
  double Quu[NU][NU];
#pragma unroll
  for (int a = 0; a < NU; ++a)
#pragma unroll
    for (int b = 0; b < NU; ++b) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < NX; ++r) v += Bf[r][a] * PBf[r][b];
      Quu[a][b] = d.hu[a * 2 + b] + v;
    }
  // Quu^-1 of the 2x2 (Cholesky form as the IPM's riccati_step)
  const double l00 = sqrt(Quu[0][0]), l10 = Quu[1][0] / l00, l11 = sqrt(Quu[1][1] - l10 * l10);
  const double i00 = 1.0 / l00, i11 = 1.0 / l11, i10 = -l10 * i00 * i11;
  double Qi[NU][NU];
  Qi[0][0] = i00 * i00 + i10 * i10;
  Qi[0][1] = Qi[1][0] = i10 * i11;
  Qi[1][1] = i11 * i11;
  double K[NU][NX];
#pragma unroll
  for (int m = 0; m < NU; ++m)
#pragma unroll
    for (int j = 0; j < NX; ++j) K[m][j] = -(Qi[m][0] * Qux[0][j] + Qi[m][1] * Qux[1][j]);
  double qc[NU], kc[NU];   // column gl of Qux and of K (selects, no runtime register index)
#pragma unroll
  for (int m = 0; m < NU; ++m) {
    qc[m] = Qux[m][0];
    kc[m] = K[m][0];
#pragma unroll
    for (int j = 1; j < NX; ++j) {
      qc[m] = gl == j ? Qux[m][j] : qc[m];
      kc[m] = gl == j ? K[m][j] : kc[m];
    }
  }
#pragma unroll
  for (int j = 0; j < NX; ++j) Pk[j] += qc[0] * K[0][j] + qc[1] * K[1][j];
  double Pf[NX][NX];
  qgather(Pk, Pf);
#pragma unroll
  for (int j = 0; j < NX; ++j) {
    double pji = Pf[j][0];
#pragma unroll
    for (int c = 1; c < NX; ++c) pji = gl == c ? Pf[j][c] : pji;
    Pn[j] = gl == j ? Pk[j] : gl < j ? 0.5 * (Pk[j] + pji) : 0.5 * (pji + Pk[j]);
  }
#pragma unroll
  for (int j = 0; j < NX; ++j) w[ad(e, O_P + xk * 16 + gl * 4 + j)] = Pn[j];
#pragma unroll
  for (int m = 0; m < NU; ++m) w[ad(e, O_K + u * 8 + m * 4 + gl)] = kc[m];
  if (gl == 0)
#pragma unroll
    for (int m = 0; m < 4; ++m) w[ad(e, O_QI + u * 4 + m)] = Qi[m / 2][m % 2];
}

struct NodeSw {
  double q, ac[NX], br[NU], kc[NU], qi[4], r[NU];
};
template <class AD>
__device__ __forceinline__ void load_sw(const double* w, const AD& ad, int e, int gl, int xk, int u, NodeSw& d) {
  d.q = w[ad(e, O_Q + xk * 4 + gl)];
#pragma unroll
  for (int j = 0; j < NX; ++j) d.ac[j] = w[ad(e, O_A + u * 16 + j * 4 + gl)];
#pragma unroll
  for (int m = 0; m < NU; ++m) d.br[m] = w[ad(e, O_B + u * 8 + gl * 2 + m)];
#pragma unroll
  for (int m = 0; m < NU; ++m) d.kc[m] = w[ad(e, O_K + u * 8 + m * 4 + gl)];
#pragma unroll
  for (int m = 0; m < 4; ++m) d.qi[m] = w[ad(e, O_QI + u * 4 + m)];
#pragma unroll
  for (int m = 0; m < NU; ++m) d.r[m] = w[ad(e, O_R + u * 2 + m)];
}
// one sweep node: g (own element of the successor's l) -> l (own element), stores l, kf
template <class AD>
__device__ __forceinline__ double quad_sw(double* w, const AD& ad, int e, int gl, int xk, int u, const NodeSw& d,
                                          double g) {
  const double gf[NX] = {qget<0>(g), qget<1>(g), qget<2>(g), qget<3>(g)};
  double ru[NU];
#pragma unroll
  for (int m = 0; m < NU; ++m) ru[m] = d.r[m] + qsum(d.br[m] * g);
  const double kf0 = -(d.qi[0] * ru[0] + d.qi[1] * ru[1]), kf1 = -(d.qi[2] * ru[0] + d.qi[3] * ru[1]);
  double l = d.q;
#pragma unroll
  for (int j = 0; j < NX; ++j) l += d.ac[j] * gf[j];
  l += d.kc[0] * ru[0] + d.kc[1] * ru[1];
  w[ad(e, O_L + xk * 4 + gl)] = l;
  if (gl == 0) {
    w[ad(e, O_KF + u * 2 + 0)] = kf0;
    w[ad(e, O_KF + u * 2 + 1)] = kf1;
  }
  return l;
}

// a child branch's Riccati recursion (terminal node, then NLEN input nodes) and its sweep
template <bool PF, class AD>
__device__ __forceinline__ void quad_branch_ric(double* w, const AD& ad, int e, int gl, int c, double (&Pn)[NX]) {
  const int xt = xnode(c, NLEN);
#pragma unroll
  for (int j = 0; j < NX; ++j) Pn[j] = w[ad(e, O_HX + xt * 16 + gl * 4 + j)];
#pragma unroll
  for (int j = 0; j < NX; ++j) w[ad(e, O_P + xt * 16 + gl * 4 + j)] = Pn[j];
  NodeRic d;
  load_ric(w, ad, e, gl, xnode(c, NLEN - 1), unode(c, NLEN - 1), d);
  for (int jn = NLEN - 1; jn >= 0; --jn) {
    NodeRic nx;
    if (PF && jn > 0) load_ric(w, ad, e, gl, xnode(c, jn - 1), unode(c, jn - 1), nx);
    double Pb[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) Pb[j] = Pn[j];
    quad_ric(w, ad, e, gl, xnode(c, jn), unode(c, jn), d, Pb, Pn);
    if (jn > 0) {
      if (PF) d = nx;
      else load_ric(w, ad, e, gl, xnode(c, jn - 1), unode(c, jn - 1), d);
    }
  }
}
template <bool PF, class AD>
__device__ __forceinline__ double quad_branch_sw(double* w, const AD& ad, int e, int gl, int c) {
  const int xt = xnode(c, NLEN);
  double g = w[ad(e, O_Q + xt * 4 + gl)];
  w[ad(e, O_L + xt * 4 + gl)] = g;
  NodeSw d;
  load_sw(w, ad, e, gl, xnode(c, NLEN - 1), unode(c, NLEN - 1), d);
  for (int jn = NLEN - 1; jn >= 0; --jn) {
    NodeSw nx;
    if (PF && jn > 0) load_sw(w, ad, e, gl, xnode(c, jn - 1), unode(c, jn - 1), nx);
    g = quad_sw(w, ad, e, gl, xnode(c, jn), unode(c, jn), d, g);
    if (jn > 0) {
      if (PF) d = nx;
      else load_sw(w, ad, e, gl, xnode(c, jn - 1), unode(c, jn - 1), d);
    }
  }
  return g;
}

// (i) shipped mapping: one wave per ego, quads 0..2 on the three child branches, then quad 0 on
// the root (children's first-node P / l summed (c0 + c1) + c2 from the slab)
template <bool PF>
__global__ __launch_bounds__(64) void k_aos(double* w, int egos) {
  const int e = blockIdx.x;
  if (e >= egos) return;
  const AoS ad;
  const int gl = threadIdx.x & 3, grp = threadIdx.x >> 2;
  if (grp < NCH) {
    double Pn[NX];
    quad_branch_ric<PF>(w, ad, e, gl, grp, Pn);
  }
  __syncthreads();
  if (grp == 0) {
    double Pb[NX], Pn[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j)
      Pb[j] = (w[ad(e, O_P + xnode(0, 0) * 16 + gl * 4 + j)] + w[ad(e, O_P + xnode(1, 0) * 16 + gl * 4 + j)]) +
              w[ad(e, O_P + xnode(2, 0) * 16 + gl * 4 + j)];
    NodeRic d;
    load_ric(w, ad, e, gl, 0, 0, d);
    quad_ric(w, ad, e, gl, 0, 0, d, Pb, Pn);
  }
  __syncthreads();
  if (grp < NCH) quad_branch_sw<PF>(w, ad, e, gl, grp);
  __syncthreads();
  if (grp == 0) {
    const double g = (w[ad(e, O_L + xnode(0, 0) * 4 + gl)] + w[ad(e, O_L + xnode(1, 0) * 4 + gl)]) +
                     w[ad(e, O_L + xnode(2, 0) * 4 + gl)];
    NodeSw d;
    load_sw(w, ad, e, gl, 0, 0, d);
    quad_sw(w, ad, e, gl, 0, 0, d, g);
  }
}

// (ii) 16 egos per wave (SoA blocks of 16), one quad per ego running its branches in turn
template <bool PF>
__global__ __launch_bounds__(64) void k_soa(double* w, int egos) {
  const int e = blockIdx.x * BLK + (threadIdx.x >> 2);
  if (blockIdx.x * BLK >= egos) return;
  const SoA ad;
  const int gl = threadIdx.x & 3;
  double S[NX];
  for (int c = 0; c < NCH; ++c) {
    double Pn[NX];
    quad_branch_ric<PF>(w, ad, e, gl, c, Pn);
#pragma unroll
    for (int j = 0; j < NX; ++j) S[j] = c == 0 ? Pn[j] : S[j] + Pn[j];   // (c0 + c1) + c2
  }
  double Pn[NX];
  NodeRic d;
  load_ric(w, ad, e, gl, 0, 0, d);
  quad_ric(w, ad, e, gl, 0, 0, d, S, Pn);
  double g = 0.0;
  for (int c = 0; c < NCH; ++c) {
    const double l = quad_branch_sw<PF>(w, ad, e, gl, c);
    g = c == 0 ? l : g + l;
  }
  NodeSw s;
  load_sw(w, ad, e, gl, 0, 0, s);
  quad_sw(w, ad, e, gl, 0, 0, s, g);
}

// ---------------------------------------------------------------------------------------
// (iii) MFMA: v_mfma_f64_4x4x4f64 = four 4x4x4 blocks, D = A B + C per block.  Operand layout
// (decoded from k_mfma_probe on gfx950, and checked at run time against the VALU result):
// lane l belongs to block (l >> 2) & 3; with r = l >> 4 and c = l & 3 it holds A[c][r] of the A
// operand, B[r][c] of the B operand and C[r][c] / D[r][c] of the accumulator.  So a D result is
// directly the next product's B operand, and as an A operand it is its own transpose.  One wave
// = 4 groups x 4 blocks = 16 egos (SoA blocks of 16); ego = g*4 + block.  Below, l16 = 4r + c is
// the entry index of a 4x4 row-major matrix.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ double mf(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
// value held by entry s = 4r + c of the lane's block
__device__ __forceinline__ double bget(double v, int s) {
  const int src = ((s >> 2) << 4) | (threadIdx.x & 12) | (s & 3);
  return __hiloint2double(__shfl(__double2hiint(v), src, 64), __shfl(__double2loint(v), src, 64));
}

struct NodeM {   // this lane's operand entries of a node (4 groups)
  double hx[4], at[4], a_b[4], btp[4], bb[4], hu[4];
};
__device__ __forceinline__ void load_m(const double* w, int blk, int l16, int b, int xk, int u, NodeM& d) {
  const SoA ad;
  const int r = l16 >> 2, c = l16 & 3;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int e = blk * BLK + g * 4 + b;
    d.hx[g] = w[ad(e, O_HX + xk * 16 + l16)];              // C operand Hx[r][c]
    d.at[g] = w[ad(e, O_A + u * 16 + l16)];                // A operand of A': A'[c][r] = A[r][c]
    d.a_b[g] = d.at[g];                                    // B operand of A: A[r][c]
    d.btp[g] = c < 2 ? w[ad(e, O_B + u * 8 + r * 2 + c)] : 0.0;   // A operand of B' (rows c < 2): B[r][c]
    d.bb[g] = d.btp[g];                                    // B operand of B (cols c < 2): B[r][c]
    d.hu[g] = (r < 2 && c < 2) ? w[ad(e, O_HU + u * 4 + r * 2 + c)] : 0.0;
  }
}

// one Riccati node for the wave's 16 egos; P[g]: D layout (P[r][c] at lane r*4 + c)
__device__ __forceinline__ void mfma_ric(double* w, int blk, int l16, int b, int xk, int u, const NodeM& d,
                                         double (&P)[4]) {
  const SoA ad;
  const int r = l16 >> 2, c = l16 & 3;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int e = blk * BLK + g * 4 + b;
    // Pb symmetric: its D layout as an A operand is Pb' = Pb
    const double M = mf(P[g], d.a_b[g], 0.0);            // Pb A
    double Pk = mf(d.at[g], M, d.hx[g]);                 // Hx + A'M
    const double Qux = mf(d.btp[g], M, 0.0);             // B'M   (rows 0..1)
    const double PB = mf(P[g], d.bb[g], 0.0);            // Pb B  (cols 0..1)
    const double Quu = mf(d.btp[g], PB, d.hu[g]);        // Hu + B'Pb B (2x2 block)
    const double q00 = bget(Quu, 0), q10 = bget(Quu, 4), q11 = bget(Quu, 5);
    const double l00 = sqrt(q00), l10 = q10 / l00, l11 = sqrt(q11 - l10 * l10);
    const double i00 = 1.0 / l00, i11 = 1.0 / l11, i10 = -l10 * i00 * i11;
    const double Q00 = i00 * i00 + i10 * i10, Q01 = i10 * i11, Q11 = i11 * i11;
    // Qi as an A operand (rows r < 2... A[l & 3][l >> 2] = Qi[c][r])
    const double qa = (c < 2 && r < 2) ? (c == r ? (c == 0 ? Q00 : Q11) : Q01) : 0.0;
    const double K = -mf(qa, Qux, 0.0);                  // -Quu^-1 Qux (rows 0..1)
    Pk = mf(Qux, K, Pk);                                 // Pk + Qux'K  (Qux in D layout = Qux' as A operand)
    const double pt = bget(Pk, c * 4 + r);               // Pk[c][r]
    const double Pn = r == c ? Pk : r < c ? 0.5 * (Pk + pt) : 0.5 * (pt + Pk);
    P[g] = Pn;
    w[ad(e, O_P + xk * 16 + l16)] = Pn;
    if (r < 2) w[ad(e, O_K + u * 8 + l16)] = K;         // K[r][c], rows 0..1
    if (r < 2 && c < 2) w[ad(e, O_QI + u * 4 + r * 2 + c)] = r == c ? (r == 0 ? Q00 : Q11) : Q01;
  }
}

struct NodeMS {
  double at[4], btp[4], kt[4], q[4], r[4], qi[4];
};
__device__ __forceinline__ void load_ms(const double* w, int blk, int l16, int b, int xk, int u, NodeMS& d) {
  const SoA ad;
  const int r = l16 >> 2, c = l16 & 3;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int e = blk * BLK + g * 4 + b;
    d.at[g] = w[ad(e, O_A + u * 16 + l16)];                                  // A' operand
    d.btp[g] = c < 2 ? w[ad(e, O_B + u * 8 + r * 2 + c)] : 0.0;              // B' operand
    d.kt[g] = r < 2 ? w[ad(e, O_K + u * 8 + r * 4 + c)] : 0.0;               // K' operand: A[c][r] = K'[c][r] = K[r][c]
    d.q[g] = c == 0 ? w[ad(e, O_Q + xk * 4 + r)] : 0.0;                      // column vector q (C layout, col 0)
    d.r[g] = (c == 0 && r < 2) ? w[ad(e, O_R + u * 2 + r)] : 0.0;
    d.qi[g] = (c < 2 && r < 2) ? w[ad(e, O_QI + u * 4 + c * 2 + r)] : 0.0;  // Qi operand: A[l&3][l>>2] = Qi[c][r]
  }
}
// one sweep node for 16 egos; G[g]: the successor's l as a column vector (D layout, col 0)
__device__ __forceinline__ void mfma_sw(double* w, int blk, int l16, int b, int xk, int u, const NodeMS& d,
                                        double (&G)[4]) {
  const SoA ad;
  const int r = l16 >> 2, c = l16 & 3;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int e = blk * BLK + g * 4 + b;
    const double ru = mf(d.btp[g], G[g], d.r[g]);        // r + B'g
    const double kf = -mf(d.qi[g], ru, 0.0);             // -Quu^-1 ru
    double l = mf(d.at[g], G[g], d.q[g]);                // q + A'g
    l = mf(d.kt[g], ru, l);                              // + K'ru
    G[g] = l;
    if (c == 0) w[ad(e, O_L + xk * 4 + r)] = l;
    if (c == 0 && r < 2) w[ad(e, O_KF + u * 2 + r)] = kf;
  }
}

template <bool PF>
__global__ __launch_bounds__(64) void k_mfma(double* w, int egos) {
  const int blk = blockIdx.x;
  if (blk * BLK >= egos) return;
  const SoA ad;
  const int l16 = ((threadIdx.x >> 4) << 2) | (threadIdx.x & 3), b = (threadIdx.x >> 2) & 3;
  const int r = l16 >> 2, c = l16 & 3;
  double S[4];
  for (int ch = 0; ch < NCH; ++ch) {
    double P[4];
    const int xt = xnode(ch, NLEN);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int e = blk * BLK + g * 4 + b;
      P[g] = w[ad(e, O_HX + xt * 16 + l16)];
      w[ad(e, O_P + xt * 16 + l16)] = P[g];
    }
    NodeM d;
    load_m(w, blk, l16, b, xnode(ch, NLEN - 1), unode(ch, NLEN - 1), d);
    for (int jn = NLEN - 1; jn >= 0; --jn) {
      NodeM nx;
      if (PF && jn > 0) load_m(w, blk, l16, b, xnode(ch, jn - 1), unode(ch, jn - 1), nx);
      mfma_ric(w, blk, l16, b, xnode(ch, jn), unode(ch, jn), d, P);
      if (jn > 0) {
        if (PF) d = nx;
        else load_m(w, blk, l16, b, xnode(ch, jn - 1), unode(ch, jn - 1), d);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) S[g] = ch == 0 ? P[g] : S[g] + P[g];
  }
  {
    NodeM d;
    load_m(w, blk, l16, b, 0, 0, d);
    mfma_ric(w, blk, l16, b, 0, 0, d, S);
  }
  double Gs[4];
  for (int ch = 0; ch < NCH; ++ch) {
    double G[4];
    const int xt = xnode(ch, NLEN);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int e = blk * BLK + g * 4 + b;
      G[g] = c == 0 ? w[ad(e, O_Q + xt * 4 + r)] : 0.0;
      if (c == 0) w[ad(e, O_L + xt * 4 + r)] = G[g];
    }
    NodeMS d;
    load_ms(w, blk, l16, b, xnode(ch, NLEN - 1), unode(ch, NLEN - 1), d);
    for (int jn = NLEN - 1; jn >= 0; --jn) {
      NodeMS nx;
      if (PF && jn > 0) load_ms(w, blk, l16, b, xnode(ch, jn - 1), unode(ch, jn - 1), nx);
      mfma_sw(w, blk, l16, b, xnode(ch, jn), unode(ch, jn), d, G);
      if (jn > 0) {
        if (PF) d = nx;
        else load_ms(w, blk, l16, b, xnode(ch, jn - 1), unode(ch, jn - 1), d);
      }
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) Gs[g] = ch == 0 ? G[g] : Gs[g] + G[g];
  }
  NodeMS d;
  load_ms(w, blk, l16, b, 0, 0, d);
  mfma_sw(w, blk, l16, b, 0, 0, d, Gs);
}

// layout probe: one block's D for A = (lane + 1), B = 100 * (lane + 1) patterns (host decodes)
__global__ void k_mfma_probe(double* out) {
  const int l = threadIdx.x;
  const double a = (l & 15) + 1, bb = 100.0 * ((l & 15) + 1);
  out[l] = mf(a, bb, 0.0);
}

// ---------------------------------------------------------------------------------------
static void root_outputs(const std::vector<double>& h, bool soa, std::vector<double>& out) {
  out.clear();
  for (int e = 0; e < EGOS; ++e) {
    auto at = [&](int off) { return soa ? h[(size_t)(e / BLK) * STRIDE * BLK + (size_t)off * BLK + e % BLK]
                                        : h[(size_t)e * STRIDE + off]; };
    for (int i = 0; i < 16; ++i) out.push_back(at(O_P + i));          // root P
    for (int i = 0; i < 4; ++i) out.push_back(at(O_L + i));           // root l
    for (int i = 0; i < 8; ++i) out.push_back(at(O_K + i));           // root K
    for (int i = 0; i < 2; ++i) out.push_back(at(O_KF + unode(1, 3) * 2 + i));
  }
}

int main(int argc, char** argv) {
  const char* which = argc > 1 ? argv[1] : "all";
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const size_t n = (size_t)EGOS * STRIDE;
  double* w;
  CK(hipMalloc(&w, n * sizeof(double)));
  {   // MFMA operand layout probe (expected: block (l>>2)&3; A[l&3][l>>4], B[l>>4][l&3], D[l>>4][l&3])
    double* po;
    CK(hipMalloc(&po, 64 * sizeof(double)));
    hipLaunchKernelGGL(k_mfma_probe, dim3(1), dim3(64), 0, 0, po);
    double hp[64];
    CK(hipMemcpy(hp, po, sizeof(hp), hipMemcpyDeviceToHost));
    int bad = 0;
    auto av = [](int l) { return (double)((l & 15) + 1); };
    for (int l = 0; l < 64; ++l) {
      const int b = (l >> 2) & 3, i = l >> 4, j = l & 3;
      double v = 0;
      for (int k = 0; k < 4; ++k) v += av(16 * k + 4 * b + i) * 100.0 * av(16 * k + 4 * b + j);
      if (hp[l] != v) ++bad;
    }
    printf("mfma_f64_4x4x4 layout probe: %s\n", bad ? "MISMATCH" : "as assumed");
    if (bad) {
      for (int l = 0; l < 64; ++l) printf("  lane %2d: %.0f\n", l, hp[l]);
    }
    CK(hipFree(po));
  }
  struct V {
    const char* name;
    bool soa;
    void (*launch)(double*);
  };
  V vars[] = {
      {"aos", false, [](double* p) { hipLaunchKernelGGL(k_aos<false>, dim3(EGOS), dim3(64), 0, 0, p, EGOS); }},
      {"aos_pf", false, [](double* p) { hipLaunchKernelGGL(k_aos<true>, dim3(EGOS), dim3(64), 0, 0, p, EGOS); }},
      {"soa", true, [](double* p) { hipLaunchKernelGGL(k_soa<false>, dim3(EGOS / BLK), dim3(64), 0, 0, p, EGOS); }},
      {"soa_pf", true, [](double* p) { hipLaunchKernelGGL(k_soa<true>, dim3(EGOS / BLK), dim3(64), 0, 0, p, EGOS); }},
      {"mfma", true, [](double* p) { hipLaunchKernelGGL(k_mfma<false>, dim3(EGOS / BLK), dim3(64), 0, 0, p, EGOS); }},
      {"mfma_pf", true, [](double* p) { hipLaunchKernelGGL(k_mfma<true>, dim3(EGOS / BLK), dim3(64), 0, 0, p, EGOS); }},
  };
  std::vector<double> h(n), ref, cur;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes_alg = (double)EGOS * 8.0 *
      ((T * 16 + U * (4 + 16 + 8)) + (T * 16 + U * (8 + 4)) +                 // Riccati: read Hx Hu A B, write P K Qi
       (T * 4 + U * (16 + 8 + 8 + 4 + 2)) + (T * 4 + U * 2));                 // sweep: read q A B K Qi r, write l kf
  for (const V& v : vars) {
    if (strcmp(which, "all") && strcmp(which, v.name)) continue;
    CK(hipMemset(w, 0, n * sizeof(double)));
    if (v.soa) hipLaunchKernelGGL(k_init<SoA>, dim3(EGOS), dim3(64), 0, 0, w, SoA());
    else hipLaunchKernelGGL(k_init<AoS>, dim3(EGOS), dim3(64), 0, 0, w, AoS());
    CK(hipDeviceSynchronize());
    v.launch(w);   // warm
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0.0f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      v.launch(w);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    CK(hipMemcpy(h.data(), w, n * sizeof(double), hipMemcpyDeviceToHost));
    root_outputs(h, v.soa, cur);
    double err = 0.0;
    if (ref.empty()) ref = cur;
    for (size_t i = 0; i < cur.size(); ++i) err = fmax(err, fabs(cur[i] - ref[i]) / fmax(1.0, fabs(ref[i])));
    const bool fin = std::isfinite(cur[0]);
    printf("%-8s  mean %8.4f ms  best %8.4f ms  alg bytes %.1f MB -> %.1f GB/s  max rel diff vs aos %.2e%s\n", v.name,
           sum / reps, best, bytes_alg / 1e6, bytes_alg / (best * 1e-3) / 1e9, err, fin ? "" : "  NON-FINITE");
  }
  CK(hipFree(w));
  return 0;
}
