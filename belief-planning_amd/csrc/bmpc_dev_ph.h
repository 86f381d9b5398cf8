// bmpc_dev_ph.h -- the phase-per-kernel CVaR IPM (bmpc_ipm_ph.h) on the GPU: one kernel per
// phase, one 64-lane wave per ego, every phase function inlined into its kernel (the
// translation units that include this header define BMPC_INLINE_ALL), and the host loop over
// the IPM iterations.
//
// The iterations run in lock-step over the batch: iteration it's eleven kernels, then the next.
// An ego that has exited returns from every later kernel after one load of its state block.
// The host stops launching when an iteration's UPD kernels counted no ego going on (a 4-byte
// read-back every kPhCheck iterations, after the first kPhFirst).
#pragma once

#include "bmpc_dev.h"
#include "bmpc_ipm_ph.h"

#ifndef BMPC_PH_FIRST
#define BMPC_PH_FIRST 8   // iterations launched before the first "anyone left?" read-back
#endif
#ifndef BMPC_PH_CHECK
#define BMPC_PH_CHECK 4   // ... and between read-backs
#endif

namespace bmpc {
namespace dev {

struct PhArgs {
  const Bundle* B;
  double* ws;
  double *upred, *xpred, *bw, *J;
  int32_t *status, *iters;
  int32_t* count;   // [maxit + 1]: egos that completed iteration it's step
  int batch;
};

template <class M, int PH>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BMPC_WPE))) void k_ph(const PhArgs a, int it) {
  const int e = blockIdx.x;
  if (e >= a.batch) return;
  const Plan& P = a.B->P;
  const Layout& L = a.B->L;
  double* ws = a.ws + L.stride * (size_t)e;
  using X = DevExecT<M::kTransform, true>;
  constexpr int NX = M::NX, NU = M::NU;
  // gate on the ego's state before touching anything else (a finished ego costs one load)
  if constexpr (PH == PH_INIT2 || PH == PH_INIT3) {
    if (!__builtin_amdgcn_readfirstlane((int)(ws[L.ist + IS_OK] != 0.0))) return;
  } else if constexpr (PH == PH_RES || PH == PH_UPD) {
    if (!__builtin_amdgcn_readfirstlane((int)(ws[L.ist + IS_ACTIVE] != 0.0))) return;
  } else if constexpr (PH != PH_INIT1 && PH != PH_FIN) {
    const bool go = ws[L.ist + IS_ACTIVE] != 0.0 && ws[L.ist + IS_OK] != 0.0;
    if (!__builtin_amdgcn_readfirstlane((int)go)) return;
    if constexpr (PH == PH_RFP0 || PH == PH_RFP1 || PH == PH_RFC0 || PH == PH_RFC1) {
      constexpr int round = (PH == PH_RFP1 || PH == PH_RFC1) ? 1 : 0;
      if (!__builtin_amdgcn_readfirstlane((int)(ws[L.ist + IS_NREF] > (double)round))) return;
    }
  }
  extern __shared__ double lds_dyn[];
  const X ex = solver_exec<M::kTransform, true>(P, lds_dyn);
  if constexpr (PH == PH_INIT1) ipm_prelude<X, M>(ex, P, L, ws);
  ipm_eco<X, M>(ex, P, L, ws);
  Ctx C;
  C.P = (CPlan*)&P;
  C.L = (CLayout*)&L;
  C.ws = (gdouble*)ws;
  if constexpr (PH == PH_INIT1) ph_init1<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_INIT2) ph_init2<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_INIT3) ph_init3<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_RES) ph_res<X, NX, NU>(ex, C, it);
  else if constexpr (PH == PH_FAC) ph_fac<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_CPL) ph_cpl<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_BKP) ph_bkp<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_RFP0) ph_refine<X, NX, NU, 0>(ex, C, 0);
  else if constexpr (PH == PH_RFP1) ph_refine<X, NX, NU, 0>(ex, C, 1);
  else if constexpr (PH == PH_AFF) ph_aff<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_CMB) ph_cmb<X, NX, NU>(ex, C);
  else if constexpr (PH == PH_RFC0) ph_refine<X, NX, NU, 1>(ex, C, 0);
  else if constexpr (PH == PH_RFC1) ph_refine<X, NX, NU, 1>(ex, C, 1);
  else if constexpr (PH == PH_UPD) {
    if (ph_upd<X, NX, NU>(ex, C, it) && threadIdx.x == 0) atomicAdd(a.count + it, 1);
  } else if constexpr (PH == PH_FIN) {
    const IpmResult r = ph_result(C.ws + L.ist);
    ipm_unpack<X, M>(ex, P, L, ws, r);
    const int lane = threadIdx.x;
    if (a.upred)
      for (int i = lane; i < P.U * P.d; i += 64) a.upred[(size_t)e * P.U * P.d + i] = ws[L.upred + i];
    if (a.xpred)
      for (int i = lane; i < P.T * P.n; i += 64) a.xpred[(size_t)e * P.T * P.n + i] = ws[L.xpred + i];
    if (a.bw)
      for (int i = lane; i < P.nbranch - 1; i += 64) a.bw[(size_t)e * (P.nbranch - 1) + i] = ws[L.w + 1 + i];
    if (lane == 0) {
      if (a.J) a.J[e] = ws[L.sol + P.oJ];
      if (a.status) a.status[e] = r.exit_flag;
      if (a.iters) a.iters[e] = r.iters;
    }
  }
}

template <class M, int PH>
hipError_t launch_ph(const SolveLaunch& s, const PhArgs& a, int it) {
  if (s.lds_bytes > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_ph<M, PH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)s.lds_bytes);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((k_ph<M, PH>), dim3(a.batch), dim3(64), s.lds_bytes, s.stream, a, it);
  return hipGetLastError();
}

// the whole IPM of one solve launch (after k_tree), host-driven over the iterations
template <class M>
hipError_t launch_ipm_phased(const SolveLaunch& s) {
  const PhArgs a{s.bundle, s.ws, s.upred, s.xpred, s.bw, s.J, s.status, s.iters, s.d_count, s.batch};
  hipError_t e;
#define BMPC_PH(ph, it_)                               \
  if ((e = launch_ph<M, ph>(s, a, it_)) != hipSuccess) \
    return e;
  if ((e = hipMemsetAsync(s.d_count, 0, sizeof(int32_t) * (size_t)(s.maxit + 1), s.stream)) != hipSuccess) return e;
  BMPC_PH(PH_INIT1, 0)
  BMPC_PH(PH_INIT2, 0)
  BMPC_PH(PH_INIT3, 0)
  int next_check = BMPC_PH_FIRST;
  for (int it = 0; it <= s.maxit; ++it) {
    BMPC_PH(PH_RES, it)
    if (it == s.maxit) break;   // RES exits every ego at maxit
    BMPC_PH(PH_FAC, it)
    BMPC_PH(PH_CPL, it)
    BMPC_PH(PH_BKP, it)
    BMPC_PH(PH_RFP0, it)
    BMPC_PH(PH_RFP1, it)
    BMPC_PH(PH_AFF, it)
    BMPC_PH(PH_CMB, it)
    BMPC_PH(PH_RFC0, it)
    BMPC_PH(PH_RFC1, it)
    BMPC_PH(PH_UPD, it)
    if (it + 1 >= next_check) {
      next_check += BMPC_PH_CHECK;
      if ((e = hipMemcpyAsync(s.h_count, s.d_count + it, sizeof(int32_t), hipMemcpyDeviceToHost, s.stream)) != hipSuccess)
        return e;
      if ((e = hipStreamSynchronize(s.stream)) != hipSuccess) return e;
      if (*s.h_count == 0) break;   // every ego has exited
    }
  }
  BMPC_PH(PH_FIN, 0)
#undef BMPC_PH
  return hipSuccess;
}

}  // namespace dev
}  // namespace bmpc
