// Wave-wide fp64 reductions for gfx950 kernels (word2vec and sent2vec): no
// LDS traffic — permlane32/16 swaps across rows, DPP moves inside rows.
// Included by HIP translation units only.
#pragma once
#include <hip/hip_runtime.h>

namespace swps {

// Sum of 8 per-lane values over the wave in 10 exchange steps (not 8 x 6):
// at every halving step each lane keeps half of its values and swaps the
// other half with its partner, so afterwards lanes 8j..8j+7 all hold the
// total of value j.  Bits 5 / 4 go through permlane swaps; the steps inside a
// row of 16 are DPP moves (row_mirror, row_half_mirror and quad permutes pair
// every lane with one of the other half — any bijection will do for a sum).
__device__ __forceinline__ double dpp_f64(double v, int ctrl_sel) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  int l2, h2;
  switch (ctrl_sel) {
    case 0:  // row_mirror: lane i <-> 15-i in each row of 16
      l2 = __builtin_amdgcn_update_dpp(0, lo, 0x140, 0xF, 0xF, false);
      h2 = __builtin_amdgcn_update_dpp(0, hi, 0x140, 0xF, 0xF, false);
      break;
    case 1:  // row_half_mirror: lane i <-> 7-i in each half-row
      l2 = __builtin_amdgcn_update_dpp(0, lo, 0x141, 0xF, 0xF, false);
      h2 = __builtin_amdgcn_update_dpp(0, hi, 0x141, 0xF, 0xF, false);
      break;
    case 2:  // quad_perm [1,0,3,2]
      l2 = __builtin_amdgcn_update_dpp(0, lo, 0xB1, 0xF, 0xF, false);
      h2 = __builtin_amdgcn_update_dpp(0, hi, 0xB1, 0xF, 0xF, false);
      break;
    default:  // quad_perm [2,3,0,1]
      l2 = __builtin_amdgcn_update_dpp(0, lo, 0x4E, 0xF, 0xF, false);
      h2 = __builtin_amdgcn_update_dpp(0, hi, 0x4E, 0xF, 0xF, false);
      break;
  }
  return __hiloint2double(h2, l2);
}

// Full wave sum of one value, every lane ends with the total: gfx950's
// v_permlane32_swap / v_permlane16_swap for the cross-row steps and DPP inside
// rows — no LDS traffic (a __shfl_xor ladder is 6 ds_bpermute rounds; this
// form took the fast-mode forward from 4.38 to 4.06 ms per batch).  After the swap the two results
// hold (lower-half value, upper-half value) in every lane, so both halves add
// the same two numbers in the same order.
__device__ __forceinline__ double wave_sum_pl(double v) {
  {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    v = __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  v += dpp_f64(v, 0);
  v += dpp_f64(v, 1);
  v += dpp_f64(v, 2);
  v += dpp_f64(v, 3);
  return v;
}

// pairwise exchange across rows with gfx950's permlane swaps: lanes of the
// lower half (row pair / half wave) end with x_lower + x_partner, lanes of the
// upper half with y_partner + y_upper — each adds the lower lane's value first
template <int W32>
__device__ __forceinline__ double swap_add(double x, double y) {
  const int xl = __double2loint(x), xh = __double2hiint(x), yl = __double2loint(y), yh = __double2hiint(y);
  if (W32) {
    const auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  const auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}

__device__ __forceinline__ double wave_sum8(double (&v)[8], int lane) {
  const bool b3 = lane & 8;
  double w4[4], w2[2];
#pragma unroll
  for (int k = 0; k < 4; k++) w4[k] = swap_add<1>(v[k], v[4 + k]);    // bit 5: lower half keeps v[k]
#pragma unroll
  for (int k = 0; k < 2; k++) w2[k] = swap_add<0>(w4[k], w4[2 + k]);  // bit 4: even rows keep w4[k]
  // bit 3 (row_mirror pairs lane i with 15-i: opposite bit 3)
  const double mine = b3 ? w2[1] : w2[0], give = b3 ? w2[0] : w2[1];
  double x = mine + dpp_f64(give, 0);
  x += dpp_f64(x, 1);  // sum within each 8-lane group
  x += dpp_f64(x, 2);
  x += dpp_f64(x, 3);
  return x;  // lanes 8j..8j+7: total of v[j]
}

}  // namespace swps
