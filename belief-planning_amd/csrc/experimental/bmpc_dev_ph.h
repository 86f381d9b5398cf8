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
  int32_t* count;   // [maxit + 1]: egos of this sub-batch that completed iteration it's step
  int e0;           // first ego of the sub-batch this launch covers
  int batch;        // egos in it
};

template <class M, int PH>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BMPC_WPE))) void k_ph(const PhArgs a, int it) {
  if ((int)blockIdx.x >= a.batch) return;
  const int e = a.e0 + blockIdx.x;
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

// ---- mode 2: one kernel, a handful of out-of-line phase functions per iteration -------------
// Each out-of-line device call costs its callee-saved-register round trip through scratch; the
// monolithic k_ipm makes ~24 per IPM iteration (every operator pass is its own function).  Here
// an iteration makes at most seven -- RES, FAC+CPL+BKP, AFF+CMB, UPD and the refinement rounds
// that run -- each with every operator inlined into it.
template <class X, int NX, int NU, int G>
__device__ __forceinline__ bool ph_group_body(const X ex, const Ctx Cin, int it) {
  // arguments arrive in VGPRs: the plan / layout / slab pointers back to SGPRs (scalar loads of
  // every Plan field instead of vector loads)
  const Ctx C = Cin.uniform();
  it = __builtin_amdgcn_readfirstlane(it);
  const gdouble* st = C.ws + C.L->ist;
  if constexpr (G == 0) {   // initial point
    ph_init1<X, NX, NU>(ex, C);
    if (ph_flag(ex, st, IS_OK)) ph_init2<X, NX, NU>(ex, C);
    if (ph_flag(ex, st, IS_OK)) ph_init3<X, NX, NU>(ex, C);
  } else if constexpr (G == 1) {
    ph_res<X, NX, NU>(ex, C, it);
  } else if constexpr (G == 2) {   // factorisation, the c- and affine directions
    ph_fac<X, NX, NU>(ex, C);
    if (ph_flag(ex, st, IS_OK)) ph_cpl<X, NX, NU>(ex, C);
    if (ph_flag(ex, st, IS_OK)) ph_bkp<X, NX, NU>(ex, C);
  } else if constexpr (G == 3) {
    ph_refine<X, NX, NU, 0>(ex, C, it);   // `it` carries the round
  } else if constexpr (G == 4) {   // affine step, combined direction
    ph_aff<X, NX, NU>(ex, C);
    ph_cmb<X, NX, NU>(ex, C);
  } else if constexpr (G == 5) {
    ph_refine<X, NX, NU, 1>(ex, C, it);
  } else {
    return ph_upd<X, NX, NU>(ex, C, it);
  }
  return true;
}

// mode 2 calls each group out of line; mode 3 (INL) inlines every group into the kernel -- each
// appears at one call site, so the kernel makes no device call at all (no callee-saved-register
// round trips through scratch; only the register allocator's own spills remain)
template <class X, int NX, int NU, int G>
__device__ __attribute__((noinline)) bool ph_group_call(const X ex, const Ctx Cin, int it) {
  return ph_group_body<X, NX, NU, G>(ex, Cin, it);
}
template <class X, int NX, int NU, int G, bool INL>
__device__ __forceinline__ bool ph_group(const X ex, const Ctx Cin, int it) {
  if constexpr (INL) return ph_group_body<X, NX, NU, G>(ex, Cin, it);
  else return ph_group_call<X, NX, NU, G>(ex, Cin, it);
}

template <class M, bool INL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BMPC_WPE))) void k_ipm_g(const PhArgs a) {
  if ((int)blockIdx.x >= a.batch) return;
  const int e = a.e0 + blockIdx.x;
  const Plan& P = a.B->P;
  const Layout& L = a.B->L;
  double* ws = a.ws + L.stride * (size_t)e;
  using X = DevExecT<M::kTransform, true>;
  constexpr int NX = M::NX, NU = M::NU;
  extern __shared__ double lds_dyn[];
  const X ex = solver_exec<M::kTransform, true>(P, lds_dyn);
  ipm_prelude<X, M>(ex, P, L, ws);
  ipm_eco<X, M>(ex, P, L, ws);
  Ctx C;
  C.P = (CPlan*)&P;
  C.L = (CLayout*)&L;
  C.ws = (gdouble*)ws;
  const gdouble* st = C.ws + L.ist;
  ph_group<X, NX, NU, 0, INL>(ex, C, 0);
  const int maxit = P.desc.maxit;
  if (ph_flag(ex, st, IS_ACTIVE))
    for (int it = 0; it <= maxit; ++it) {
      ph_group<X, NX, NU, 1, INL>(ex, C, it);
      if (it == maxit || !ph_flag(ex, st, IS_ACTIVE)) break;
      if (ph_flag(ex, st, IS_OK)) ph_group<X, NX, NU, 2, INL>(ex, C, it);
      const int nref = __builtin_amdgcn_readfirstlane((int)st[IS_NREF]);
      for (int r = 0; r < nref; ++r)
        if (ph_flag(ex, st, IS_OK)) ph_group<X, NX, NU, 3, INL>(ex, C, r);
      if (ph_flag(ex, st, IS_OK)) ph_group<X, NX, NU, 4, INL>(ex, C, it);
      for (int r = 0; r < nref; ++r)
        if (ph_flag(ex, st, IS_OK)) ph_group<X, NX, NU, 5, INL>(ex, C, r);
      if (!__builtin_amdgcn_readfirstlane((int)ph_group<X, NX, NU, 6, INL>(ex, C, it))) break;
    }
  const IpmResult r = ph_result(st);
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

template <class M, int PH>
hipError_t launch_ph(const SolveLaunch& s, const PhArgs& a, int it, hipStream_t st) {
  if (s.lds_bytes > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_ph<M, PH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)s.lds_bytes);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((k_ph<M, PH>), dim3(a.batch), dim3(64), s.lds_bytes, st, a, it);
  return hipGetLastError();
}

// the whole IPM of one solve launch (after k_tree on s.stream), host-driven over the iterations.
// Mode 1 splits the batch into s.nsub sub-batches, each on a stream of its own: a phase kernel
// waits for the slowest ego of its sub-batch, and the other sub-batches' kernels fill the gap
// (the HIP streams map to separate hardware queues).
template <class M>
hipError_t launch_ipm_phased(const SolveLaunch& s) {
  hipError_t e;
  if (s.ph_mode == 2 || s.ph_mode == 3) {   // one kernel: grouped out-of-line phases / everything inlined
    const PhArgs a{s.bundle, s.ws, s.upred, s.xpred, s.bw, s.J, s.status, s.iters, s.d_count, 0, s.batch};
    const void* kf = s.ph_mode == 3 ? (const void*)k_ipm_g<M, true> : (const void*)k_ipm_g<M, false>;
    if (s.lds_bytes > 64 * 1024 &&
        (e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s.lds_bytes)) != hipSuccess)
      return e;
    if (s.ph_mode == 3) hipLaunchKernelGGL((k_ipm_g<M, true>), dim3(a.batch), dim3(64), s.lds_bytes, s.stream, a);
    else hipLaunchKernelGGL((k_ipm_g<M, false>), dim3(a.batch), dim3(64), s.lds_bytes, s.stream, a);
    return hipGetLastError();
  }
  const int ns = s.nsub < 1 ? 1 : s.nsub > kMaxSub ? kMaxSub : s.nsub;
  const int per = (s.batch + ns - 1) / ns;
  PhArgs a[kMaxSub];
  hipStream_t st[kMaxSub];
  bool live[kMaxSub];
  int nsub = 0;
  for (int i = 0; i < ns && i * per < s.batch; ++i, ++nsub) {
    const int lo = i * per, hi = lo + per < s.batch ? lo + per : s.batch;
    a[i] = PhArgs{s.bundle, s.ws, s.upred, s.xpred, s.bw, s.J, s.status, s.iters,
                  s.d_count + (size_t)i * (s.maxit + 1), lo, hi - lo};
    st[i] = ns == 1 ? s.stream : s.sub[i];
    live[i] = true;
  }
#define BMPC_PH(ph, it_, i)                                    \
  if ((e = launch_ph<M, ph>(s, a[i], it_, st[i])) != hipSuccess) \
    return e;
  if ((e = hipMemsetAsync(s.d_count, 0, sizeof(int32_t) * (size_t)nsub * (s.maxit + 1), s.stream)) != hipSuccess)
    return e;
  if (ns > 1) {   // the sub-streams start after k_tree and the counter reset on s.stream
    if ((e = hipEventRecord(s.sub_ev[kMaxSub], s.stream)) != hipSuccess) return e;
    for (int i = 0; i < nsub; ++i)
      if ((e = hipStreamWaitEvent(st[i], s.sub_ev[kMaxSub], 0)) != hipSuccess) return e;
  }
  for (int i = 0; i < nsub; ++i) {
    BMPC_PH(PH_INIT1, 0, i)
    BMPC_PH(PH_INIT2, 0, i)
    BMPC_PH(PH_INIT3, 0, i)
  }
  int next_check = BMPC_PH_FIRST;
  for (int it = 0; it <= s.maxit; ++it) {
    bool any = false;
    for (int i = 0; i < nsub; ++i) {
      if (!live[i]) continue;
      any = true;
      BMPC_PH(PH_RES, it, i)
      if (it == s.maxit) continue;   // RES exits every ego at maxit
      BMPC_PH(PH_FAC, it, i)
      BMPC_PH(PH_CPL, it, i)
      BMPC_PH(PH_BKP, it, i)
      BMPC_PH(PH_RFP0, it, i)
      BMPC_PH(PH_RFP1, it, i)
      BMPC_PH(PH_AFF, it, i)
      BMPC_PH(PH_CMB, it, i)
      BMPC_PH(PH_RFC0, it, i)
      BMPC_PH(PH_RFC1, it, i)
      BMPC_PH(PH_UPD, it, i)
    }
    if (!any || it == s.maxit) break;
    if (it + 1 >= next_check) {
      next_check += BMPC_PH_CHECK;
      for (int i = 0; i < nsub; ++i)
        if (live[i] && (e = hipMemcpyAsync(s.h_count + i, a[i].count + it, sizeof(int32_t), hipMemcpyDeviceToHost,
                                           st[i])) != hipSuccess)
          return e;
      for (int i = 0; i < nsub; ++i) {
        if (!live[i]) continue;
        if ((e = hipStreamSynchronize(st[i])) != hipSuccess) return e;
        if (s.h_count[i] == 0) live[i] = false;   // every ego of the sub-batch has exited
      }
    }
  }
  for (int i = 0; i < nsub; ++i) {
    BMPC_PH(PH_FIN, 0, i)
    if (ns > 1) {   // s.stream resumes after every sub-batch
      if ((e = hipEventRecord(s.sub_ev[i], st[i])) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(s.stream, s.sub_ev[i], 0)) != hipSuccess) return e;
    }
  }
#undef BMPC_PH
  return hipSuccess;
}

}  // namespace dev
}  // namespace bmpc
