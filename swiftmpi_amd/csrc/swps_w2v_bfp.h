// Block-floating-point intermediates (swps_w2v_cfg.fp64_intermediates =
// SWPS_INTER_BFP40 / SWPS_INTER_BFP32): fp32 tables whose learn_instance
// intermediates neu1 / neu1e carry 40 (or 32) significant bits relative to
// their row's largest element, at 5 (or 4) bytes per element.
//
// Why: the gradient of a key is a mean of many terms g*neu1[p] / neu1e[p]
// (word2vec_global.h:705,716,122-134) that often cancel, and AdaGrad's first
// step lr*g/sqrt(g^2 + 1e-6) (:176-185) passes an absolute error in a small
// mean g on x700.  neu1 / neu1e rounded to fp32 (fast mode) put the rows
// 5e-6 (D = 300) to 1.4e-5 (D = 100) from the reference after one minibatch,
// 1e-4 after two, 1e-2..1e-1 after two epochs.  What matters is the absolute
// error of each term, and a row's elements share a scale (sums of a few table
// rows): one exponent per row and integer mantissas spend the bits where
// fp32's per-element exponents do not.  Measured on the CPU by emulating each
// rounding inside the reference's arithmetic (scripts/diag_bfp.py), full-array
// max relative distance from the reference's fp32-storage run at D = 300 /
// D = 100:
//                 bytes/el   1 batch         2 batches        2 epochs
//   fp32 (fast)       4     4.7e-6/1.4e-5   8.6e-5/1.3e-4    7.5e-3/1.4e-1
//   BFP32             4     1.2e-7/2.3e-7   1.8e-5/8.4e-6    1.4e-3/9.0e-4
//   fp32 + int16      6     1.2e-7/1.2e-7   1.2e-7/1.2e-7    2.2e-5/7.6e-6
//   BFP40             5     1.2e-7/1.2e-7   1.5e-7/1.2e-7    1.1e-4/4.8e-5
// (1.2e-7 is the fp32 storage of the rows themselves; the two-epoch tails are
// a few elements whose dot products crossed an exp-table bucket edge,
// (int)((f + 6) * 83), word2vec_global.h:259 — chaotic, and ~6e4x rarer at
// 2^-40 than at fp32's 2^-24).
//
// A kept position's neu1 (and neu1e) row, ld = bfp_ld(D, RB) floats, with
// e = the exponent of the row's largest |x| (max|x| < 2^e), u = 2^(e-31-8RB):
//   int32 [0, D)               m = rint(x / (2^(8RB) u)), |m| < 2^31
//   int8  [0, D) at float D    RB = 1 only: r = rint((x - m 2^(8RB) u) / u)
//   float D + RB*D/4           u (a power of two, at least the smallest normal)
//   floats up to ld            zero (whole 128-B lines)
// so x = (m 2^(8RB) + r) u with |error| <= u/2 = 2^-(32+8RB) of 2^e.  Readers
// sum the m parts in fp64 (exact products) and the r parts in fp32 (2^-31 of
// the m parts: fp32 adds nothing measurable), scaled per record, and add the
// two at the end.  Multi-chunk partials, the per-key sums, the mean and the
// sharded push payload are fp64.
//
// Lane layout (any D % 4 == 0, D <= 512): NCH 4-element chunks (elements
// 4*(lane + 64c) .. +3; the last one may be partial when NT = 0) and NT
// scalar tails (element 256*NCH + 64t + lane).  Inactive lanes load a valid
// duplicate and never store or dot it.
//
// Included by swps_w2v.hip inside its anonymous namespace (uses FwdArgs,
// GatherArgs, PushArgs, run_recs, item_recs, uniform4, slot_row, xcd_block,
// kGroup, PHead).
#pragma once

constexpr int kBfpMaxD = 512;
inline int bfp_ld(int D, int RB) { return (D + RB * D / 4 + 1 + 31) / 32 * 32; }  // floats per row

// gfx950 wave max (the permlane / DPP pattern of swps_wave.h: any pairing will do for a max)
__device__ __forceinline__ int wave_max_i32(int v) {
  {
    const auto s = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = max(s[0], s[1]);
  }
  {
    const auto s = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = max(s[0], s[1]);
  }
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));  // row_mirror
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  return v;
}

__device__ __forceinline__ double pow2d(int k) { return __longlong_as_double((long long)(1023 + k) << 52); }

template <int NCH, int NT> struct LaneMap {
  static constexpr int NC = NCH ? NCH : 1, NTT = NT ? NT : 1;
  int ci[NC];   // 4-element chunk index (clamped to a valid one)
  int te[NTT];  // tail element (clamped)
  uint32_t act;  // bit c: chunk c holds live elements; bit NCH + t: tail t does
  __device__ __forceinline__ LaneMap(int lane, int D) {
    const int D4 = D >> 2;
    act = 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const int i = lane + 64 * c;
      act |= (uint32_t)(i < D4) << c;
      ci[c] = min(i, D4 - 1);
    }
#pragma unroll
    for (int t = 0; t < NT; t++) {
      const int e = 256 * NCH + 64 * t + lane;
      act |= (uint32_t)(e < D) << (NCH + t);
      te[t] = min(e, D - 1);
    }
  }
  __device__ __forceinline__ bool ca(int c) const { return (act >> c) & 1; }
  __device__ __forceinline__ bool ta(int t) const { return (act >> (NCH + t)) & 1; }
};

// a lane's elements of an fp32 row (table rows, worker-cache rows)
template <int NCH, int NT> struct GSlice {
  float4 v[LaneMap<NCH, NT>::NC];
  float t[LaneMap<NCH, NT>::NTT];
  __device__ __forceinline__ void ld(const float *row, const LaneMap<NCH, NT> &m) {
#pragma unroll
    for (int c = 0; c < NCH; c++) v[c] = ((const float4 *)row)[m.ci[c]];
#pragma unroll
    for (int k = 0; k < NT; k++) t[k] = row[m.te[k]];
  }
  __device__ __forceinline__ void st(float *row, const LaneMap<NCH, NT> &m) const {
#pragma unroll
    for (int c = 0; c < NCH; c++)
      if (m.ca(c)) ((float4 *)row)[m.ci[c]] = v[c];
#pragma unroll
    for (int k = 0; k < NT; k++)
      if (m.ta(k)) row[m.te[k]] = t[k];
  }
};

__device__ __forceinline__ float byte_i8(uint32_t w, int k) {  // sign-extended byte k of w as float
  return (float)((int32_t)(w << (24 - 8 * k)) >> 24);
}

// a lane's elements of a BFP row (mantissas m, RB = 1: residuals r; the row scale is read separately)
template <int NCH, int NT, int RB> struct BRow {
  int4 m[LaneMap<NCH, NT>::NC];
  uint32_t r[LaneMap<NCH, NT>::NC];
  int32_t mt[LaneMap<NCH, NT>::NTT];
  int32_t rt[LaneMap<NCH, NT>::NTT];
  // stl >= 0: this lane's last tail load fetches element stl instead (the row scale; ScaleLane)
  __device__ __forceinline__ void ld(const float *row, const LaneMap<NCH, NT> &mp, int D, int stl = -1) {
    const int8_t *lo = (const int8_t *)(row + D);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      m[c] = ((const int4 *)row)[mp.ci[c]];
      if (RB) r[c] = ((const uint32_t *)lo)[mp.ci[c]];
    }
#pragma unroll
    for (int k = 0; k < NT; k++) {
      mt[k] = ((const int32_t *)row)[k == NT - 1 && stl >= 0 ? stl : mp.te[k]];
      if (RB) rt[k] = lo[mp.te[k]];
    }
  }
};
template <int RB> __device__ __forceinline__ float bfp_scale(const float *row, int D) { return row[D + RB * D / 4]; }

// bfp32 rows whose last tail leaves lanes free (D = 300: elements 256..299 on lanes 0..43): the
// first free lane loads the row scale (float D) with the tail, and the record's scale is a
// readlane of it — one memory instruction per record less than a separate scale load.
template <int NCH, int NT, int RB> struct ScaleLane {
  int lane = -1;  // wave-uniform: the lane carrying the scale, or -1 (separate load)
  int stl = -1;   // this lane's tail index override
  __device__ __forceinline__ ScaleLane(int l, int D) {
    if (RB == 0 && NT > 0) {
      const int f = D - 256 * NCH - 64 * (NT - 1);
      if (f >= 0 && f < 64) {
        lane = f;
        stl = l == f ? D : -1;
      }
    }
  }
  // at load time: the separate scale load when no lane carries it (issued with the row's loads)
  __device__ __forceinline__ float ld(const float *row, int D) const { return lane >= 0 ? 0.f : bfp_scale<RB>(row, D); }
  // at use time (after the loads, so the readlane does not stall the next rows' loads)
  __device__ __forceinline__ float get(const BRow<NCH, NT, RB> &r, float loaded) const {
    if (NT > 0 && lane >= 0) return __int_as_float(__builtin_amdgcn_readlane(r.mt[NT > 0 ? NT - 1 : 0], lane));
    return loaded;
  }
};

// fp64 row accumulator of the forward (neu1, neu1e), stored as a BFP row
template <int NCH, int NT> struct DAcc {
  double v[LaneMap<NCH, NT>::NC][4];
  double t[LaneMap<NCH, NT>::NTT];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
      for (int k = 0; k < 4; k++) v[c][k] = 0.0;
#pragma unroll
    for (int k = 0; k < NT; k++) t[k] = 0.0;
  }
  __device__ __forceinline__ void add(const GSlice<NCH, NT> &r) {  // neu1 += syn0 (word2vec_global.h:680)
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      v[c][0] += (double)r.v[c].x;
      v[c][1] += (double)r.v[c].y;
      v[c][2] += (double)r.v[c].z;
      v[c][3] += (double)r.v[c].w;
    }
#pragma unroll
    for (int k = 0; k < NT; k++) t[k] += (double)r.t[k];
  }
  __device__ __forceinline__ void axpy(double g, const GSlice<NCH, NT> &r) {  // neu1e += g * syn1neg (:703)
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      v[c][0] = __builtin_fma(g, (double)r.v[c].x, v[c][0]);
      v[c][1] = __builtin_fma(g, (double)r.v[c].y, v[c][1]);
      v[c][2] = __builtin_fma(g, (double)r.v[c].z, v[c][2]);
      v[c][3] = __builtin_fma(g, (double)r.v[c].w, v[c][3]);
    }
#pragma unroll
    for (int k = 0; k < NT; k++) t[k] = __builtin_fma(g, (double)r.t[k], t[k]);
  }
  __device__ __forceinline__ double dot(const GSlice<NCH, NT> &r, const LaneMap<NCH, NT> &m) const {  // :692
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      double p = v[c][0] * (double)r.v[c].x;
      p = __builtin_fma(v[c][1], (double)r.v[c].y, p);
      p = __builtin_fma(v[c][2], (double)r.v[c].z, p);
      p = __builtin_fma(v[c][3], (double)r.v[c].w, p);
      s += m.ca(c) ? p : 0.0;
    }
#pragma unroll
    for (int k = 0; k < NT; k++) s += m.ta(k) ? t[k] * (double)r.t[k] : 0.0;
    return s;
  }
  // the BFP row (layout at the top of this file), whole lines
  template <int RB>
  __device__ __forceinline__ void st_bfp(float *row, const LaneMap<NCH, NT> &m, int D, int ld, int lane) const {
    constexpr int MB = 31 + 8 * RB;  // bits below 2^e kept
    // the largest biased fp64 exponent of this lane's live elements = that of their largest |x|
    double amax = 0.0;
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (m.ca(c)) amax = fmax(amax, fabs(v[c][k]));
#pragma unroll
    for (int k = 0; k < NT; k++)
      if (m.ta(k)) amax = fmax(amax, fabs(t[k]));
    const uint32_t eb = (uint32_t)(__double2hiint(amax) >> 20) & 0x7FFu;
    // max|x| < 2^e with e = biased - 1022; keep the scale a normal fp32 (tiny rows: fewer bits, never wrong)
    const int e = max((int)wave_max_i32((int)eb) - 1022, MB - 126);
    const double im = pow2d(31 - e), ir = pow2d(MB - e), hm = pow2d(e - 31);
    auto mant = [&](double x) { return (int32_t)fmin(fmax(rint(x * im), -2147483647.0), 2147483647.0); };
    auto res = [&](double x, int32_t q) {  // the int8 residual below the mantissa's last bit (exact difference)
      return (uint32_t)(int32_t)fmin(fmax(rint((x - (double)q * hm) * ir), -127.0), 127.0) & 0xFFu;
    };
    int8_t *lo = (int8_t *)(row + D);
#pragma unroll
    for (int c = 0; c < NCH; c++)
      if (m.ca(c)) {
        const int4 q = make_int4(mant(v[c][0]), mant(v[c][1]), mant(v[c][2]), mant(v[c][3]));
        ((int4 *)row)[m.ci[c]] = q;
        if (RB)
          ((uint32_t *)lo)[m.ci[c]] = res(v[c][0], q.x) | res(v[c][1], q.y) << 8 | res(v[c][2], q.z) << 16 |
                                      res(v[c][3], q.w) << 24;
      }
#pragma unroll
    for (int k = 0; k < NT; k++)
      if (m.ta(k)) {
        const int32_t q = mant(t[k]);
        ((int32_t *)row)[m.te[k]] = q;
        if (RB) lo[m.te[k]] = (int8_t)res(t[k], q);
      }
    const int s0 = D + RB * D / 4;
    for (int i = s0 + lane; i < ld; i += 64) row[i] = i == s0 ? __int_as_float((e - MB + 127) << 23) : 0.f;
  }
};

// gradient-sum accumulator: fp64 for the mantissa parts (and fp64 partials), fp32 for the residuals
template <int NCH, int NT, int RB> struct BAcc {
  double h[LaneMap<NCH, NT>::NC][4];
  double ht[LaneMap<NCH, NT>::NTT];
  float l[LaneMap<NCH, NT>::NC][4];
  float lt[LaneMap<NCH, NT>::NTT];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
      for (int k = 0; k < 4; k++) {
        h[c][k] = 0.0;
        l[c][k] = 0.f;
      }
#pragma unroll
    for (int k = 0; k < NT; k++) {
      ht[k] = 0.0;
      lt[k] = 0.f;
    }
  }
  // += a * x for a row x = (m 2^(8RB) + r) u: cm = a 2^(8RB) u (fp64), cr = a u (fp32).  h records:
  // a = g (accu_h(g * neu1), word2vec_global.h:705); v records: a = 1 (accu_v(neu1e), :716).
  __device__ __forceinline__ void axpy(double cm, float cr, const BRow<NCH, NT, RB> &x) {
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      h[c][0] = __builtin_fma(cm, (double)x.m[c].x, h[c][0]);
      h[c][1] = __builtin_fma(cm, (double)x.m[c].y, h[c][1]);
      h[c][2] = __builtin_fma(cm, (double)x.m[c].z, h[c][2]);
      h[c][3] = __builtin_fma(cm, (double)x.m[c].w, h[c][3]);
      if (RB)
#pragma unroll
        for (int k = 0; k < 4; k++) l[c][k] = __builtin_fmaf(cr, byte_i8(x.r[c], k), l[c][k]);
    }
#pragma unroll
    for (int k = 0; k < NT; k++) {
      ht[k] = __builtin_fma(cm, (double)x.mt[k], ht[k]);
      if (RB) lt[k] = __builtin_fmaf(cr, (float)x.rt[k], lt[k]);
    }
  }
  __device__ __forceinline__ double tot(int c, int k) const { return RB ? h[c][k] + (double)l[c][k] : h[c][k]; }
  __device__ __forceinline__ double tott(int k) const { return RB ? ht[k] + (double)lt[k] : ht[k]; }
};

// a lane's elements of an fp64 row in natural order (multi-chunk partials, the push payload)
template <int NCH, int NT> struct DSlice {
  double2 a[LaneMap<NCH, NT>::NC][2];
  double t[LaneMap<NCH, NT>::NTT];
  __device__ __forceinline__ void ld(const double *row, const LaneMap<NCH, NT> &m) {
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      a[c][0] = ((const double2 *)row)[2 * m.ci[c]];
      a[c][1] = ((const double2 *)row)[2 * m.ci[c] + 1];
    }
#pragma unroll
    for (int k = 0; k < NT; k++) t[k] = row[m.te[k]];
  }
  template <int RB> __device__ __forceinline__ void add_to(BAcc<NCH, NT, RB> &s) const {
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      s.h[c][0] += a[c][0].x;
      s.h[c][1] += a[c][0].y;
      s.h[c][2] += a[c][1].x;
      s.h[c][3] += a[c][1].y;
    }
#pragma unroll
    for (int k = 0; k < NT; k++) s.ht[k] += t[k];
  }
};

template <int NCH, int NT, int RB>
__device__ __forceinline__ void st_f64(double *row, const LaneMap<NCH, NT> &m, const BAcc<NCH, NT, RB> &s, double mul) {
#pragma unroll
  for (int c = 0; c < NCH; c++)
    if (m.ca(c)) {
      ((double2 *)row)[2 * m.ci[c]] = make_double2(s.tot(c, 0) * mul, s.tot(c, 1) * mul);
      ((double2 *)row)[2 * m.ci[c] + 1] = make_double2(s.tot(c, 2) * mul, s.tot(c, 3) * mul);
    }
#pragma unroll
  for (int k = 0; k < NT; k++)
    if (m.ta(k)) row[m.te[k]] = s.tott(k) * mul;
}

// ---- forward (learn_instance's position body, word2vec_global.h:663-718) ----
// k_forward_t on LaneMap slices, neu1 / neu1e stored as BFP rows.
template <int NCH, int NT, int RB, int G>
__global__ __launch_bounds__(256) void k_forward_b(FwdArgs<float, float> a) {
  const int lane = threadIdx.x & 63;
  const uint32_t blk = a.xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int p = __builtin_amdgcn_readfirstlane((int)(blk * 4 + (threadIdx.x >> 6)));
  if (p >= a.P) return;
  const int D = a.D, W = a.W, N = a.N;
  const LaneMap<NCH, NT> m(lane, D);
  const int S = 2 * W + N + 1;  // slots: contexts then targets
  const int32_t *r = a.rec + (uint64_t)p * (S + 1);
  DAcc<NCH, NT> acc, ne;
  acc.zero();
  ne.zero();
  float gk = 0.f;
  for (int s0 = 0; s0 < S; s0 += G) {
    GSlice<NCH, NT> rows[G];
    int32_t vid[G];
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int slot = s0 + q;
      vid[q] = __builtin_amdgcn_readfirstlane(slot < S ? r[1 + slot] : -1);
      if (vid[q] >= 0) rows[q].ld(slot_row(a, vid[q], slot < 2 * W), m);
    }
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int slot = s0 + q;
      if (vid[q] < 0) continue;
      if (slot < 2 * W) {
        acc.add(rows[q]);
      } else {
        const int d = slot - 2 * W;
        const double part = wave_sum_pl(acc.dot(rows[q], m));
        float f = 0;
        f += part;
        const int label = d == 0 ? 1 : 0;
        float g;
        if (f > 6)
          g = (label - 1) * a.alpha;
        else if (f < -6)
          g = (label - 0) * a.alpha;
        else
          g = (label - a.exptab[(int)((f + 6) * (1000 / 6 / 2))]) * a.alpha;
        ne.axpy((double)g, rows[q]);
        if (lane == d) gk = g;
      }
    }
  }
  acc.template st_bfp<RB>(a.neu1 + (uint64_t)p * a.ld, m, D, a.ld, lane);
  ne.template st_bfp<RB>(a.neu1e + (uint64_t)p * a.ld, m, D, a.ld, lane);
  if (lane <= N) a.pg[(uint64_t)p * (N + 1) + lane] = gk;
}

// record coefficients of a BFP row with scale u (h records: a = g; v records: a = 1)
template <int RB> __device__ __forceinline__ double coef_m(float a, float u) { return (double)a * (double)u * (RB ? 256.0 : 1.0); }

// ---- multi-chunk gradient sums (k_gather_t's role under the fused push) ----
// One wave per chunk of <= 128 records of one (key, kind), software-pipelined
// across items; the fp64 partial in natural element order.
template <int NCH, int NT, int RB, int UNR>
__global__ __launch_bounds__(256) void k_gather_b(GatherArgs<float> a, double *__restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int D = a.D;
  const LaneMap<NCH, NT> m(lane, D);
  const ScaleLane<NCH, NT, RB> sl(lane, D);
  const uint32_t NI = min(a.multi[0], a.max_items);
  const uint32_t stride = gridDim.x * 4;
  uint32_t qi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= NI) return;
  auto item_at = [&](uint32_t q) { return a.multi[1 + __builtin_amdgcn_readfirstlane(q)]; };
  uint32_t item = __builtin_amdgcn_readfirstlane(item_at(qi));
  uint4 d = uniform4(a.desc[item]);
  ItemRecs ri = item_recs(a, d, lane);
  for (;;) {
    const uint32_t qn = qi + stride;
    const bool more = qn < NI;
    const uint32_t nx = more ? __builtin_amdgcn_readfirstlane(item_at(qn)) : 0;
    const uint4 dn = uniform4(more ? a.desc[nx] : make_uint4(0, 0x80000000u, 0, 0));
    const uint32_t s = d.x, e = d.y & 0x7FFFFFFFu, kind = d.y >> 31, n = e - s;
    const float *base = kind == 0 ? a.neu1 : a.neu1e;
    BAcc<NCH, NT, RB> acc;
    acc.zero();
    ItemRecs rn;
    for (uint32_t r0 = 0; r0 < n; r0 += UNR) {
      BRow<NCH, NT, RB> rv[UNR];
      float gg[UNR], sc[UNR];
#pragma unroll
      for (int q = 0; q < UNR; q++) {
        const uint32_t idx = min(r0 + q, n - 1);
        const uint32_t pr = idx < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)ri.p0, (int)idx)
                                     : (uint32_t)__builtin_amdgcn_readlane((int)ri.p1, (int)(idx - 64));
        gg[q] = __int_as_float(idx < 64 ? __builtin_amdgcn_readlane(__float_as_int(ri.g0), (int)idx)
                                        : __builtin_amdgcn_readlane(__float_as_int(ri.g1), (int)(idx - 64)));
        const float *row = base + (uint64_t)pr * a.ld;
        rv[q].ld(row, m, D, sl.stl);
        sc[q] = sl.ld(row, D);
      }
      if (r0 == 0) rn = item_recs(a, dn, lane);  // next item's record info, behind this item's first rows
#pragma unroll
      for (int q = 0; q < UNR; q++) {
        if (r0 + q < n) {
          const float g = kind == 0 ? gg[q] : 1.f, u = sl.get(rv[q], sc[q]);
          acc.axpy(coef_m<RB>(g, u), g * u, rv[q]);
        }
      }
    }
    if (n == 0) rn = item_recs(a, dn, lane);
    st_f64(partial + (uint64_t)item * D, m, acc, 1.0);
    if (!more) break;
    qi = qn;
    item = nx;
    d = dn;
    ri = rn;
  }
}

// Hot (key, kind) runs with more than kGroup chunks: each group leader sums
// its group's fp64 partials in chunk order into its own slot (k_combine).
__global__ __launch_bounds__(256) void k_combine_b(GatherArgs<float> a, double *__restrict__ partial) {
  const int lane = threadIdx.x & 63;
  const int D = a.D;
  const uint32_t NL = min(a.lead[0], a.max_items / 8 + 1);
  for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < NL; q += gridDim.x * 4) {
    const uint32_t item = a.lead[1 + __builtin_amdgcn_readfirstlane(q)];
    const uint4 d = uniform4(a.desc[item]);
    const uint32_t end = min(item + kGroup, a.ioff[d.z + 1]);
    for (int e2 = lane; 2 * e2 < D; e2 += 64) {
      double2 rv[kGroup];
#pragma unroll
      for (uint32_t q2 = 0; q2 < kGroup; q2++)
        rv[q2] = ((const double2 *)(partial + (uint64_t)min(item + q2, end - 1) * D))[e2];
      double2 s = make_double2(0.0, 0.0);
#pragma unroll
      for (uint32_t q2 = 0; q2 < kGroup; q2++)
        if (item + q2 < end) {
          s.x += rv[q2].x;
          s.y += rv[q2].y;
        }
      ((double2 *)(partial + (uint64_t)item * D))[e2] = s;
    }
  }
}

// ---- fused sums + mean + AdaGrad (k_push_thp on BFP rows) ----
// One wave per (key, half), software-pipelined across items: a single-chunk
// run (<= 128 records) is summed here from the BFP neu1 / neu1e rows, a
// multi-chunk run from k_gather_b's fp64 partials (k_combine_b group leaders
// for hot runs); the mean (word2vec_global.h:122-134) in fp64; AdaGrad
// (:176-185) in fp64 on the fp32 table row, whose pre-update value goes to the
// worker cache.  TO_GRADS (sharded learner): the fp64 mean is the push payload
// [U][h|v] (the reference's wire type), zeros for an empty half; a.gpass as in
// k_push_thp.
// WPE: a minimum of waves per SIMD the register allocation must allow (1 = unconstrained).
template <int NCH, int NT, int RB, int UNR, bool TO_GRADS, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_push_b(
    PushArgs<float, float> a, const double *__restrict__ partial, double *__restrict__ grads) {
  constexpr int PU = 4;
  const int lane = threadIdx.x & 63;
  const int D = a.D;
  const LaneMap<NCH, NT> m(lane, D);
  const ScaleLane<NCH, NT, RB> sl(lane, D);
  const uint64_t n2 = 2ull * a.U;
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  uint64_t uh = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (uh >= n2) return;
  auto head = [&](uint64_t x) {
    const uint64_t u = x >> 1;
    const int half = (int)(x & 1);
    PHead h;
    h.s0 = __builtin_amdgcn_readfirstlane(a.seg[(2 * half) * a.U + u]);
    h.s1 = __builtin_amdgcn_readfirstlane(a.seg[(2 * half + 1) * a.U + u]);
    h.i0 = __builtin_amdgcn_readfirstlane(a.ioff[2 * u + half]);
    h.i1 = __builtin_amdgcn_readfirstlane(a.ioff[2 * u + half + 1]);
    h.vid = __builtin_amdgcn_readfirstlane(a.K[u]);
    h.row = TO_GRADS ? 0u : __builtin_amdgcn_readfirstlane(a.krow[u]);
    return h;
  };
  auto recs_of = [&](const PHead &h, uint64_t x) {
    ItemRecs r{0, 0, 1.f, 1.f};
    if (h.s1 > h.s0 && h.i1 - h.i0 == 1) r = run_recs(a.vals, a.pg, a.SH, a.SV, a.HOFF, h.s0, h.s1 - h.s0, (int)(x & 1), lane);
    return r;
  };
  PHead h = head(uh);
  ItemRecs ri = recs_of(h, uh);
  for (;;) {
    const uint64_t nx = uh + stride;
    const bool more = nx < n2;
    PHead hn{0, 0, 0, 0, 0, 0};
    if (more) hn = head(nx);
    const int half = (int)(uh & 1);
    if (TO_GRADS && a.gpass) {  // the key's owner range: its first ohalf keys go in pass 1
      const uint32_t u = (uint32_t)(uh >> 1);
      uint32_t r = 0;
      while (r + 1 < a.nown && a.obnd[r + 1] <= u) r++;
      const bool first = u - a.obnd[r] < a.ohalf[r];
      if (first != (a.gpass == 1)) {  // the other pass's item
        if (more) ri = recs_of(hn, nx);
        if (!more) break;
        uh = nx;
        h = hn;
        continue;
      }
    }
    if (lane == 0 && half == 0) a.local[h.vid] = -1;
    const uint32_t cnt = h.s1 - h.s0;
    const bool one = h.i1 - h.i0 == 1;
    float *row = TO_GRADS ? nullptr : a.rows + (uint64_t)h.row * 4 * D;
    double *gout = TO_GRADS ? grads + ((uh >> 1) * 2 + half) * (uint64_t)D : nullptr;
    GSlice<NCH, NT> wr, w2r;
    ItemRecs rn{0, 0, 1.f, 1.f};
    bool rn_done = false;
    if (!TO_GRADS) {
      if (cnt || a.cache_h) wr.ld(row + half * D, m);
      if (cnt) w2r.ld(row + (2 + half) * D, m);
    }
    if (!TO_GRADS && a.cache_h) {  // the pre-update value, pad as zeros (whole lines)
      float *crow = (half ? a.cache_v : a.cache_h) + (uint64_t)h.vid * a.cs;
      wr.st(crow, m);
      if (a.full)
        for (int e = D + lane; e < a.cs; e += 64) crow[e] = 0.f;
    }
    BAcc<NCH, NT, RB> acc;
    acc.zero();
    if (cnt && one) {
      const float *base = half == 0 ? a.neu1 : a.neu1e;
      for (uint32_t r0 = 0; r0 < cnt; r0 += UNR) {
        BRow<NCH, NT, RB> rv[UNR];
        float gf[UNR], sc[UNR];
#pragma unroll
        for (int q = 0; q < UNR; q++) {
          const uint32_t idx = min(r0 + q, cnt - 1);
          const uint32_t pr = idx < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)ri.p0, (int)idx)
                                       : (uint32_t)__builtin_amdgcn_readlane((int)ri.p1, (int)(idx - 64));
          gf[q] = __int_as_float(idx < 64 ? __builtin_amdgcn_readlane(__float_as_int(ri.g0), (int)idx)
                                          : __builtin_amdgcn_readlane(__float_as_int(ri.g1), (int)(idx - 64)));
          const float *prow = base + (uint64_t)pr * a.ld;
          rv[q].ld(prow, m, D, sl.stl);
          sc[q] = sl.ld(prow, D);
        }
        if (r0 == 0) {  // the next item's record info, behind this item's first rows
          if (more) rn = recs_of(hn, nx);
          rn_done = true;
        }
#pragma unroll
        for (int q = 0; q < UNR; q++) {
          if (r0 + q < cnt) {
            const float g = half == 0 ? gf[q] : 1.f, u = sl.get(rv[q], sc[q]);
            acc.axpy(coef_m<RB>(g, u), g * u, rv[q]);
          }
        }
      }
    } else if (cnt) {
      if (more) rn = recs_of(hn, nx);
      rn_done = true;
      const uint32_t st = (h.i1 - h.i0) > a.group ? kGroup : 1;
      for (uint32_t it0 = h.i0; it0 < h.i1; it0 += PU * st) {
        DSlice<NCH, NT> pv[PU];
#pragma unroll
        for (int q = 0; q < PU; q++) pv[q].ld(partial + (uint64_t)min(it0 + q * st, h.i1 - 1) * D, m);
#pragma unroll
        for (int q = 0; q < PU; q++)
          if (it0 + q * st < h.i1) pv[q].add_to(acc);
      }
    }
    if (TO_GRADS) {
      st_f64(gout, m, acc, cnt ? 1.0 / (double)cnt : 0.0);
    } else if (cnt) {
      const double inv = (double)cnt;
      float *w = row + half * D, *w2 = row + (2 + half) * D;
      GSlice<NCH, NT> wo, w2o;
      auto upd = [&](double sum, float wv, float w2v, float &o, float &o2) {
        const double g = sum / inv;  // the mean (fp64, the reference's push value)
        const double acc2 = (double)w2v + g * g;
        const double step = (g * a.lr) / sqrt(acc2 + a.fudge);
        o2 = (float)acc2;
        o = (float)((double)wv + step);
      };
#pragma unroll
      for (int c = 0; c < NCH; c++) {
        upd(acc.tot(c, 0), wr.v[c].x, w2r.v[c].x, wo.v[c].x, w2o.v[c].x);
        upd(acc.tot(c, 1), wr.v[c].y, w2r.v[c].y, wo.v[c].y, w2o.v[c].y);
        upd(acc.tot(c, 2), wr.v[c].z, w2r.v[c].z, wo.v[c].z, w2o.v[c].z);
        upd(acc.tot(c, 3), wr.v[c].w, w2r.v[c].w, wo.v[c].w, w2o.v[c].w);
      }
#pragma unroll
      for (int k = 0; k < NT; k++) upd(acc.tott(k), wr.t[k], w2r.t[k], wo.t[k], w2o.t[k]);
      w2o.st(w2, m);
      wo.st(w, m);
    }
    if (!rn_done && more) rn = recs_of(hn, nx);
    if (!more) break;
    uh = nx;
    h = hn;
    ri = rn;
  }
}
