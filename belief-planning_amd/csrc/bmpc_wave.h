// bmpc_wave.h -- wave-level butterflies on the VALU's cross-lane paths (HIP builds only): the
// executors' reductions (bmpc_dev.h) and the one-wave steps of bmpc_ipm.h use them.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>

namespace bmpc {
namespace dev {

// A lane's DPP source value (every row and bank enabled).  bound_ctrl: a lane whose source lies
// outside its row (row_shr / row_shl edges) reads 0 -- what the former update_dpp with old = 0
// and bound_ctrl off left there -- so no zeroed destination has to be materialised first (one
// v_mov per 32-bit half less: 128 of the Riccati node's 615 instructions); the same values.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// One butterfly level of a wave reduction: v op (lane ^ O)'s v, in every lane.  The partner value
// comes from the VALU's cross-lane paths instead of the LDS crossbar (ds_bpermute): permlane32 /
// permlane16 swaps (gfx950) for O = 32 / 16, DPP row_ror:8 for 8, DPP row shifts for 4, DPP
// quad_perm for 2 and 1.  The same pairs as the __shfl_xor butterfly, own value first (the swaps
// hand every lane its own and its partner's value; a + b is commutative bit for bit), so a
// reduction gives the same bits as before.
template <int OP>
__device__ __forceinline__ double red_op(double a, double b) {
  return OP == 0 ? a + b : OP == 1 ? fmax(a, b) : fmin(a, b);
}
template <int O, int OP, bool DPP>
__device__ __forceinline__ double xor_level(double v) {
  if constexpr (!DPP) {
    return red_op<OP>(v, __shfl_xor(v, O, 64));
  } else if constexpr (O == 32 || O == 16) {
    const unsigned lo = __double2loint(v), hi = __double2hiint(v);
    const auto a = O == 32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                           : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = O == 32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                           : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    // lanes of the lower half of each 2*O block: (own, partner); upper half: (partner, own)
    const double x = __hiloint2double(b[0], a[0]), y = __hiloint2double(b[1], a[1]);
    const bool low = (__lane_id() & O) == 0;
    return low ? red_op<OP>(x, y) : red_op<OP>(y, x);
  } else if constexpr (O == 8) {
    return red_op<OP>(v, dpp_d<0x128>(v));   // row_ror:8 = lane ^ 8 within a row of 16
  } else if constexpr (O == 4) {
    const double up = dpp_d<0x114>(v), dn = dpp_d<0x104>(v);   // row_shr:4 (lane - 4), row_shl:4 (lane + 4)
    return red_op<OP>(v, (__lane_id() & 4) ? up : dn);
  } else if constexpr (O == 2) {
    return red_op<OP>(v, dpp_d<0x4E>(v));    // quad_perm [2,3,0,1]
  } else {
    return red_op<OP>(v, dpp_d<0xB1>(v));    // quad_perm [1,0,3,2]
  }
}
// the whole-wave butterfly (levels 32 .. 1, the order of the former __shfl_xor loops)
template <int OP, bool DPP>
__device__ __forceinline__ double wave_reduce(double v) {
  v = xor_level<32, OP, DPP>(v);
  v = xor_level<16, OP, DPP>(v);
  v = xor_level<8, OP, DPP>(v);
  v = xor_level<4, OP, DPP>(v);
  v = xor_level<2, OP, DPP>(v);
  return xor_level<1, OP, DPP>(v);
}
// the butterfly over aligned groups of g lanes (g a power of two <= 64): levels g/2 .. 1
template <int OP, bool DPP>
__device__ __forceinline__ double group_reduce(double v, int g) {
  if (g > 32) v = xor_level<32, OP, DPP>(v);
  if (g > 16) v = xor_level<16, OP, DPP>(v);
  if (g > 8) v = xor_level<8, OP, DPP>(v);
  if (g > 4) v = xor_level<4, OP, DPP>(v);
  if (g > 2) v = xor_level<2, OP, DPP>(v);
  if (g > 1) v = xor_level<1, OP, DPP>(v);
  return v;
}
}  // namespace dev
}  // namespace bmpc
#endif
