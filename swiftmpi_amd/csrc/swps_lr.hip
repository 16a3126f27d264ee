// Sparse logistic regression on one MI355X: the reference's minibatch loop
// (apps/logistic/lr.cpp:157-238, nthreads = 1 semantics) as HIP kernels.
//
// Per minibatch (B+1 valid rows, lr.cpp:308-354 gather == train window):
//   k_lr_forward   one wave per row: s = sum w_i*x_i (fp32, feature order),
//                  p = 1/(1+exp(-s)), e = y - p stored per row (lr.cpp:358-375)
//   k_lr_reduce_*  per pushed key (a run of the batch's records in their static
//                  key-sorted order, built once at load): the gradient records
//                  e[row]*x_i summed in record order (fp32 chain, exact mode),
//                  mean = sum/count (lr.cpp:32-38), AdaGrad fp32 (lr.cpp:68-75)
//                  on the shard row
//   k_lr_tiles(_fin) fast_sums mode: the same per-key means from fp64 sums over
//                  row tiles (e read from LDS, one partial per block piece)
// The records' (row, x_i) in key-sorted order are static (srow / sval), so the
// forward writes one error per row instead of scattering a record per feature.
// Every weight read in a batch belongs to that batch's key set, which the
// reference pulls at the start of the batch and the server only changes at the
// push: reading the shard rows directly is the same snapshot, so no copy.
#include <hip/hip_ext.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <limits>
#include <string>
#include <unordered_map>
#include <chrono>
#include <thread>
#include <unordered_set>

#include "swps_internal.h"
#include "swps_sort.h"
#include "swps_wave.h"

using namespace swps;

namespace {

// weight of vid: from the shard rows [w | g2] (single GPU) or, vid_row ==
// nullptr, from the worker's pulled cache (sharded mode, param.h:13-68)
__device__ __forceinline__ float weight(const uint32_t *__restrict__ vid_row, const float *__restrict__ w, int32_t v) {
  return vid_row ? w[(uint64_t)vid_row[v] * 2] : w[v];
}
// the training loop's form: fidx = the feature's shard row (single GPU, stride 2: precomputed
// vid_row[vid] per record, one dependent random load less) or its vid (cache, stride 1)
__device__ __forceinline__ float weight_at(const float *__restrict__ w, uint32_t fidx, int stride) {
  return w[(uint64_t)fidx * stride];
}

// Ordered fp32 sum of one value per lane (lanes [0, m)) added to acc in lane
// order — the reference's sequential `sum += ...` (bit-exact), with the loads
// of all lanes issued in parallel.
__device__ __forceinline__ float ordered_add(float acc, float x, int m) {
  for (int k = 0; k < m; k++) acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), k));
  return acc;
}

// One wave per example (LR::learn_instance, lr.cpp:358-375): lane k holds
// feature k of the row (64 at a time), s = sum w_i*x_i in feature order,
// p = 1/(1+exp(-s)), e = y - p; gradient record (vid, e*x_i) per feature in
// (row, feature) order.
__global__ __launch_bounds__(256) void k_lr_forward(const uint64_t *__restrict__ row_off, const uint32_t *__restrict__ fidx,
                             const float *__restrict__ fval, const float *__restrict__ label, uint64_t r0, uint64_t nr,
                             const float *__restrict__ rows, int stride, float *__restrict__ err,
                             float *__restrict__ err2) {
  const uint64_t j = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (j >= nr) return;
  const uint64_t r = r0 + j;
  const uint64_t a = row_off[r], b = row_off[r + 1];
  float sum = 0;
  for (uint64_t c = a; c < b; c += 64) {
    const int m = (int)min<uint64_t>(64, b - c);
    float prod = 0.f;
    if (lane < m) {
      const float w = weight_at(rows, fidx[c + lane], stride);
      prod = w * fval[c + lane];
    }
    sum = ordered_add(sum, prod, m);
  }
  const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
  const float error = label[r] - predict;
  // the gradient records e*x_i are formed by the reduce from the static sorted (row, x_i)
  if (lane == 0) {
    err[r] = error;
    err2[r] = error * error;
  }
}

// k_lr_forward with R rows per wave (rows of at most 2*(64/R) features): L = 64/R lanes per
// row, two features per lane (f and f+L).  The examples are latency-bound chains (offsets ->
// feature indices -> weights -> the ordered sum), so R rows per wave put R times the chains
// in flight per wave slot; the R ordered sums run interleaved.  Same products, same
// feature-order fp32 sums as k_lr_forward: bit-identical.
// SCAT (with LDS_SUM): the forward also writes the batch's gradient records e*x_i into their
// key-sorted slots (spos, static), the job of k_lr_records — same fp32 products, no second pass
template <int R, bool LDS_SUM = false, bool SCAT = false>
__global__ __launch_bounds__(256) void k_lr_forward_r(const uint64_t *__restrict__ row_off,
                                                      const uint32_t *__restrict__ fidx, const float *__restrict__ fval,
                                                      const float *__restrict__ label, uint64_t r0, uint64_t nr,
                                                      const float *__restrict__ rows, int stride,
                                                      float *__restrict__ err, float *__restrict__ err2,
                                                      int diag = 0, const uint32_t *__restrict__ spos = nullptr,
                                                      uint64_t nz0 = 0, float *__restrict__ val = nullptr) {
  constexpr int L = 64 / R;
  const int lane = threadIdx.x & 63;
  const int sub = lane / L, k = lane - sub * L;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wave * R >= nr) return;
  const uint64_t j = wave * R + (uint64_t)sub;
  const bool act = sub < R && j < nr;
  int m = 0;
  float p0 = 0.f, p1 = 0.f, y = 0.f, x0 = 0.f, x1 = 0.f;
  uint32_t q0 = 0, q1 = 0;
  if (act) {
    const uint64_t r = r0 + j;
    const uint64_t a = row_off[r];
    m = (int)(row_off[r + 1] - a);
    y = label[r];
    if (SCAT) {
      if (k < m) {
        x0 = fval[a + k];
        q0 = spos[a + k];
      }
      if (k + L < m) {
        x1 = fval[a + k + L];
        q1 = spos[a + k + L];
      }
    }
    if (diag & 1) {  // SWPS_LR_DIAG timing experiment only: no weight gather (w = x)
      if (k < m) p0 = fval[a + k];
      if (k + L < m) p1 = fval[a + k + L];
    } else {
      if (k < m) p0 = weight_at(rows, fidx[a + k], stride) * fval[a + k];
      if (k + L < m) p1 = weight_at(rows, fidx[a + k + L], stride) * fval[a + k + L];
    }
  }
  if (diag & 2) {  // timing experiment only: no ordered chain (a wave tree sum per row)
    float t = p0 + p1;
    for (int o = 1; o < L; o <<= 1) t += __shfl_xor(t, o);
    if (act && k == 0) {
      const float predict = (float)(1. / (1. + (double)(float)exp((double)(-t))));
      err[r0 + j] = y - predict;
      err2[r0 + j] = (y - predict) * (y - predict);
    }
    return;
  }
  if (LDS_SUM) {
    // the ordered sums through LDS: every lane stores its two products, then one lane per row
    // reads its row's products back in feature order (4 per ds_read) and adds them sequentially
    // — the same fp32 adds in the same order as the readlane chain below, without its
    // per-feature readlane latency
    __shared__ float4 sp[4][R][(2 * L + 3) / 4];
    float *row = (float *)sp[threadIdx.x >> 6][sub < R ? sub : 0];
    if (sub < R) {
      row[k] = p0;
      row[k + L] = p1;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    float error = 0.f;
    if (act && k == 0) {
      float s = 0.f;
      const float4 *r4 = (const float4 *)row;
      for (int f4 = 0; f4 * 4 < m; f4++) {
        const float4 v = r4[f4];
        s += v.x;
        if (f4 * 4 + 1 < m) s += v.y;
        if (f4 * 4 + 2 < m) s += v.z;
        if (f4 * 4 + 3 < m) s += v.w;
      }
      const float predict = (float)(1. / (1. + (double)(float)exp((double)(-s))));
      error = y - predict;
      err[r0 + j] = error;
      err2[r0 + j] = error * error;
    }
    if (SCAT) {  // the row's e to its lanes (lane sub*L holds it), then one record per feature
      const float e = __int_as_float(__builtin_amdgcn_ds_bpermute((sub < R ? sub : 0) * L * 4, __float_as_int(error)));
      if (act && k < m) val[q0 - nz0] = e * x0;
      if (act && k + L < m) val[q1 - nz0] = e * x1;
    }
    return;
  }
  int mq[R];
  int mmax = 0;
#pragma unroll
  for (int q = 0; q < R; q++) {
    mq[q] = __builtin_amdgcn_readlane(m, q * L);  // 0 for rows past the batch
    mmax = max(mmax, mq[q]);
  }
  float sum[R];
#pragma unroll
  for (int q = 0; q < R; q++) sum[q] = 0.f;
  for (int f = 0; f < mmax; f++) {  // feature order, R chains interleaved
    const int src = f < L ? __float_as_int(p0) : __float_as_int(p1);
    const int fl = f < L ? f : f - L;
#pragma unroll
    for (int q = 0; q < R; q++)
      if (f < mq[q]) sum[q] += __int_as_float(__builtin_amdgcn_readlane(src, q * L + fl));
  }
  if (act && k == 0) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < R; q++)
      if (q == sub) s = sum[q];
    const float predict = (float)(1. / (1. + (double)(float)exp((double)(-s))));
    const float error = y - predict;
    err[r0 + j] = error;
    err2[r0 + j] = error * error;
  }
}

// k_lr_forward_r<R, LDS_SUM> with G row groups per wave: every group's loads, then every group's
// weight gathers, then the ordered sums (the groups' chains interleaved) — G times the memory
// chains in flight per wave, a G-th of the waves.  Same products, same feature-order fp32 sums:
// bit-identical (SWPS_LR_FWD_G).
// hrow != nullptr (single GPU): the batch's nhot (<= kLrHot) hottest keys' shard rows; fidx codes a
// record of one of them as kLrHotBit | rank, and the block reads its weight from LDS (loaded once per
// block, kLrHotPT per thread)
constexpr int kLrHot = 1024;
constexpr int kLrHotPT = kLrHot / 256;
constexpr uint32_t kLrHotBit = 0x80000000u;
struct HotW {  // a thread's share of the block's hot weights: loads first, LDS stores later
  float v[kLrHotPT];
  __device__ __forceinline__ void ld(const float *rows, const uint32_t *hrow, uint32_t nhot, int tid) {
#pragma unroll
    for (int j = 0; j < kLrHotPT; j++) {
      const uint32_t q = (uint32_t)tid + 256u * j;
      v[j] = hrow && q < nhot ? rows[(uint64_t)hrow[q] * 2] : 0.f;
    }
  }
  __device__ __forceinline__ void st(float *wh, uint32_t nhot, int tid) const {
#pragma unroll
    for (int j = 0; j < kLrHotPT; j++) {
      const uint32_t q = (uint32_t)tid + 256u * j;
      if (q < nhot) wh[q] = v[j];
    }
  }
};
template <int R, int G>
__global__ __launch_bounds__(256) void k_lr_forward_g(const uint64_t *__restrict__ row_off,
                                                      const uint32_t *__restrict__ fidx, const float *__restrict__ fval,
                                                      const float *__restrict__ label, uint64_t r0, uint64_t nr,
                                                      const float *__restrict__ rows, int stride,
                                                      float *__restrict__ err, float *__restrict__ err2,
                                                      const uint32_t *__restrict__ hrow = nullptr, uint32_t nhot = 0) {
  constexpr int L = 64 / R;
  __shared__ float4 sp[4][G][R][(2 * L + 3) / 4];
  __shared__ float wh[kLrHot];
  // the hot weights' loads go out first; their LDS stores and the block barrier come after this
  // thread's own index loads (every wave reaches the barrier: rows past the batch are inactive)
  HotW hw;
  hw.ld(rows, hrow, nhot, threadIdx.x);
  const int lane = threadIdx.x & 63;
  const int sub = lane / L, k = lane - sub * L;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (!hrow && wave * G * R >= nr) return;
  uint64_t a[G];
  int m[G];
  float y[G];
  bool act[G];
#pragma unroll
  for (int g = 0; g < G; g++) {
    const uint64_t j = (wave * G + g) * R + (uint64_t)sub;
    act[g] = sub < R && j < nr;
    a[g] = 0;
    m[g] = 0;
    y[g] = 0.f;
    if (act[g]) {
      a[g] = row_off[r0 + j];
      m[g] = (int)(row_off[r0 + j + 1] - a[g]);
      y[g] = label[r0 + j];
    }
  }
  uint32_t i0[G], i1[G];
  float x0[G], x1[G];
#pragma unroll
  for (int g = 0; g < G; g++) {
    const bool v0 = act[g] && k < m[g], v1 = act[g] && k + L < m[g];
    i0[g] = v0 ? fidx[a[g] + k] : 0u;
    x0[g] = v0 ? fval[a[g] + k] : 0.f;
    i1[g] = v1 ? fidx[a[g] + k + L] : 0u;
    x1[g] = v1 ? fval[a[g] + k + L] : 0.f;
  }
  if (hrow) {
    hw.st(wh, nhot, threadIdx.x);
    __syncthreads();
  }
  float w0[G], w1[G];
#pragma unroll
  for (int g = 0; g < G; g++) {
    if (hrow) {
      w0[g] = act[g] && k < m[g] ? ((i0[g] & kLrHotBit) ? wh[i0[g] & (kLrHotBit - 1)] : rows[(uint64_t)i0[g] * 2]) : 0.f;
      w1[g] = act[g] && k + L < m[g] ? ((i1[g] & kLrHotBit) ? wh[i1[g] & (kLrHotBit - 1)] : rows[(uint64_t)i1[g] * 2])
                                     : 0.f;
    } else {
      w0[g] = act[g] && k < m[g] ? weight_at(rows, i0[g], stride) : 0.f;
      w1[g] = act[g] && k + L < m[g] ? weight_at(rows, i1[g], stride) : 0.f;
    }
  }
#pragma unroll
  for (int g = 0; g < G; g++) {
    float *row = (float *)sp[threadIdx.x >> 6][g][sub < R ? sub : 0];
    if (sub < R) {
      row[k] = act[g] && k < m[g] ? w0[g] * x0[g] : 0.f;
      row[k + L] = act[g] && k + L < m[g] ? w1[g] * x1[g] : 0.f;
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  if (k != 0 || sub >= R) return;
  float sum[G];
  int mm = 0;
#pragma unroll
  for (int g = 0; g < G; g++) {
    sum[g] = 0.f;
    mm = max(mm, act[g] ? m[g] : 0);
  }
  for (int f4 = 0; f4 * 4 < mm; f4++) {
#pragma unroll
    for (int g = 0; g < G; g++) {
      if (!act[g] || f4 * 4 >= m[g]) continue;
      const float4 v = ((const float4 *)sp[threadIdx.x >> 6][g][sub])[f4];
      sum[g] += v.x;
      if (f4 * 4 + 1 < m[g]) sum[g] += v.y;
      if (f4 * 4 + 2 < m[g]) sum[g] += v.z;
      if (f4 * 4 + 3 < m[g]) sum[g] += v.w;
    }
  }
#pragma unroll
  for (int g = 0; g < G; g++) {
    if (!act[g]) continue;
    const uint64_t j = (wave * G + g) * R + (uint64_t)sub;
    const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum[g]))));
    const float error = y[g] - predict;
    err[r0 + j] = error;
    err2[r0 + j] = error * error;
  }
}

// Record-contiguous forward (SWPS_LR_FWD_C, the default): a block takes a static chunk of whole rows
// holding at most RPT*256 records (built on the host at the first batch), so its threads load the
// chunk's indices and values as contiguous 16-B-aligned runs straight from the chunk's first record —
// no per-row offset load in front of them — while the rows' offsets and labels load beside them.
// Products w*x go to LDS in record order; one thread per row then adds its row's products in
// feature order in fp32 (lr.cpp:358-375, -ffp-contract=off): the same products and the same ordered
// sum as every other forward form, so bit-identical.  Two dependent memory round trips per record
// (index -> weight) instead of three, and RPT*256 records per block: a Criteo batch (2.56M records)
// is ~1,250 blocks of 4 waves, all resident at once.
constexpr int kLrFwdRpt = 8;
template <int RPT>
__global__ __launch_bounds__(256) void k_lr_forward_c(const uint2 *__restrict__ chunks,
                                                      const uint64_t *__restrict__ row_off,
                                                      const uint32_t *__restrict__ fidx, const float *__restrict__ fval,
                                                      const float *__restrict__ label, uint64_t r0,
                                                      const float *__restrict__ rows, int stride,
                                                      float *__restrict__ err, float *__restrict__ err2,
                                                      const uint32_t *__restrict__ hrow, uint32_t nhot) {
  constexpr int CAP = RPT * 256;
  __shared__ float prod[CAP];
  __shared__ float wh[kLrHot];
  const int tid = threadIdx.x;
  HotW hw;
  hw.ld(rows, hrow, nhot, tid);
  const uint2 ch = chunks[blockIdx.x];  // first row (batch-relative), rows
  const uint64_t rf = r0 + ch.x;
  const uint64_t c0 = row_off[rf], c1 = row_off[rf + ch.y];
  const uint32_t n = (uint32_t)(c1 - c0);
  uint32_t f[RPT];
  float x[RPT];
#pragma unroll
  for (int k = 0; k < RPT; k++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)k * 256u;
    f[k] = i < n ? fidx[c0 + i] : 0u;
    x[k] = i < n ? fval[c0 + i] : 0.f;
  }
  // this thread's row (rows beyond 256 per chunk are looped below)
  uint64_t ra = 0, rb = 0;
  float y = 0.f;
  if ((uint32_t)tid < ch.y) {
    ra = row_off[rf + tid];
    rb = row_off[rf + tid + 1];
    y = label[rf + tid];
  }
  if (hrow) {
    hw.st(wh, nhot, tid);
    __syncthreads();
  }
  float w[RPT];
#pragma unroll
  for (int k = 0; k < RPT; k++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)k * 256u;
    if (i >= n)
      w[k] = 0.f;
    else if (hrow)
      w[k] = (f[k] & kLrHotBit) ? wh[f[k] & (kLrHotBit - 1)] : rows[(uint64_t)f[k] * 2];
    else
      w[k] = weight_at(rows, f[k], stride);
  }
#pragma unroll
  for (int k = 0; k < RPT; k++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)k * 256u;
    if (i < n) prod[i] = w[k] * x[k];
  }
  __syncthreads();
  for (uint32_t r = (uint32_t)tid; r < ch.y; r += 256u) {
    if (r >= 256u) {
      ra = row_off[rf + r];
      rb = row_off[rf + r + 1];
      y = label[rf + r];
    }
    float sum = 0.f;
    for (uint32_t c = (uint32_t)(ra - c0); c < (uint32_t)(rb - c0); c++) sum += prod[c];
    const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
    const float error = y - predict;
    err[rf + r] = error;
    err2[rf + r] = error * error;
  }
}

// One lane per example: the lane sums its own row in feature order (lr.cpp:
// 358-375, fp32 products and adds, -ffp-contract=off: bit-identical to the
// cross-lane forms above) — no readlane chain.  Per chunk of CH features the
// lane issues every index and value load, then every weight gather, then the
// ordered adds, so a row of <= CH features is three memory round trips.  The
// index/value loads of a wave touch 64 rows' lines at once; a lane's next
// features hit the same lines in L1.  (Measured by SWPS_LR_DIAG on the
// cross-lane k_lr_forward_r<3>: the ordered readlane chain alone was ~12 of
// its ~34 us per 65,537-row batch.)
template <int CH>
__global__ __launch_bounds__(64) void k_lr_forward_l(const uint64_t *__restrict__ row_off,
                                                     const uint32_t *__restrict__ fidx, const float *__restrict__ fval,
                                                     const float *__restrict__ label, uint64_t r0, uint64_t nr,
                                                     const float *__restrict__ rows, int stride,
                                                     float *__restrict__ err, float *__restrict__ err2) {
  const uint64_t j = (uint64_t)blockIdx.x * 64 + threadIdx.x;
  if (j >= nr) return;
  const uint64_t r = r0 + j;
  const uint64_t a = row_off[r], b = row_off[r + 1];
  float sum = 0.f;
  for (uint64_t c = a; c < b; c += CH) {
    const int m = (int)min<uint64_t>(CH, b - c);
    uint32_t id[CH];
    float x[CH], w[CH];
#pragma unroll
    for (int k = 0; k < CH; k++)
      if (k < m) {
        id[k] = fidx[c + k];
        x[k] = fval[c + k];
      }
#pragma unroll
    for (int k = 0; k < CH; k++)
      if (k < m) w[k] = weight_at(rows, id[k], stride);
#pragma unroll
    for (int k = 0; k < CH; k++)
      if (k < m) {
        const float prod = w[k] * x[k];
        sum += prod;
      }
  }
  const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
  const float error = label[r] - predict;
  err[r] = error;
  err2[r] = error * error;
}

// ---- the static per-batch index (built once at load; lr_index) -------------
// The batch's records are its rows' features in (row, feature) order; their
// stable key-sorted order, the runs (one per pushed key) and the run bounds
// depend only on the data, never on the weights: sorted once for the whole
// corpus with (batch << 32 | vid) keys instead of once per minibatch.
__global__ void k_lr_idx_keys(const uint64_t *__restrict__ row_off, uint64_t nr, uint64_t B1,
                              const int32_t *__restrict__ fvid, uint64_t *__restrict__ key, uint32_t *__restrict__ idx) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  const uint64_t b = r / B1;
  for (uint64_t c = row_off[r]; c < row_off[r + 1]; c++) {
    key[c] = (b << 32) | (uint32_t)fvid[c];
    idx[c] = (uint32_t)c;
  }
}

// row of every record
__global__ void k_lr_rowid(const uint64_t *__restrict__ row_off, uint64_t nr, uint32_t *__restrict__ rid) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  for (uint64_t c = row_off[r]; c < row_off[r + 1]; c++) rid[c] = (uint32_t)r;
}

// the records in sorted order: their row and x_i; run heads
__global__ void k_lr_idx_slots(const uint64_t *__restrict__ ks, const uint32_t *__restrict__ perm, uint64_t n,
                               const uint32_t *__restrict__ rid, const float *__restrict__ fval,
                               uint32_t *__restrict__ srow, float *__restrict__ sval, uint32_t *__restrict__ head,
                               uint32_t *__restrict__ spos) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t c = perm[i];
  srow[i] = rid[c];
  sval[i] = fval[c];
  spos[c] = (uint32_t)i;  // the inverse: feature c's slot in the key-sorted record order
  head[i] = (i == 0 || ks[i] != ks[i - 1]) ? 1u : 0u;
}

// every record's run (global index): the forward's staged weights (SWPS_LR_STAGE)
__global__ void k_lr_idx_frun(const uint32_t *__restrict__ perm, const uint32_t *__restrict__ rid1, uint64_t n,
                              uint32_t *__restrict__ frun) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) frun[perm[i]] = rid1[i] - 1;
}
// the batch's weights, one per run (key), dense: the forward gathers from these 4 B x runs
// (L2-resident) instead of the shard's 8-B rows across the table
__global__ void k_lr_stage(const uint32_t *__restrict__ urow, uint32_t nruns, const float *__restrict__ rows,
                           float *__restrict__ wd) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < nruns) wd[r] = rows[(uint64_t)urow[r] * 2];
}

// single GPU, once the shard rows are known: a record of one of its batch's hot keys is coded
// kLrHotBit | rank (k_lr_forward_g reads it from LDS), any other by its key's shard row; the hot
// keys' shard rows per batch
__global__ void k_lr_hot_codes(const uint32_t *__restrict__ frun, const int32_t *__restrict__ hot_of_run,
                               const uint32_t *__restrict__ frow, uint64_t n, uint32_t *__restrict__ code) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const int32_t h = hot_of_run[frun[c]];
  code[c] = h >= 0 ? (kLrHotBit | (uint32_t)h) : frow[c];
}
__global__ void k_lr_hot_rows(const uint32_t *__restrict__ hgrun, uint64_t n, const uint32_t *__restrict__ urow,
                              uint32_t *__restrict__ hrow) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) hrow[q] = urow[hgrun[q]];
}

// shard row of every record's feature / every run's key (single GPU)
__global__ void k_lr_map_rows(const int32_t *__restrict__ vid, uint64_t n, const uint32_t *__restrict__ vid_row,
                              uint32_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = vid_row[vid[i]];
}

__global__ void k_lr_idx_runs(const uint64_t *__restrict__ ks, const uint32_t *__restrict__ head,
                              const uint32_t *__restrict__ rid1, uint64_t n, const uint64_t *__restrict__ bnz0,
                              uint64_t *__restrict__ rkey, uint32_t *__restrict__ uniq, uint32_t *__restrict__ off) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !head[i]) return;
  const uint32_t r = rid1[i] - 1;
  rkey[r] = ks[i];
  uniq[r] = (uint32_t)ks[i];
  off[r] = (uint32_t)(i - bnz0[ks[i] >> 32]);
}

// run lengths from the starts (a run never crosses its batch: the next run's
// start in the same batch, else the batch's record count)
__global__ void k_lr_idx_cnt(const uint64_t *__restrict__ rkey, const uint32_t *__restrict__ off, uint64_t R,
                             const uint64_t *__restrict__ bnz0, uint32_t *__restrict__ cnt) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint64_t b = rkey[r] >> 32;
  const uint64_t end = (r + 1 < R && (rkey[r + 1] >> 32) == b) ? off[r + 1] : bnz0[b + 1] - bnz0[b];
  cnt[r] = (uint32_t)(end - off[r]);
}

// first run of every batch (lower bound of b << 32), and its run count
__global__ void k_lr_idx_bruns(const uint64_t *__restrict__ rkey, uint64_t R, uint64_t nb, uint64_t *__restrict__ brun,
                               uint32_t *__restrict__ bnruns) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nb) return;
  auto lb = [&](uint64_t v) {
    uint64_t lo = 0, hi = R;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (rkey[mid] < v)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  };
  const uint64_t a = lb(b << 32);
  brun[b] = a;
  if (b < nb) bnruns[b] = (uint32_t)(lb((b + 1) << 32) - a);
}

// Per pushed key (a run of the sorted records): s = sum of e*x_i in record
// order (fp32, sequential like `grads[i].val += ...`), mean = s/count
// (lr.cpp:32-38); then either AdaGrad on the shard row (lr.cpp:68-75) or, in
// sharded mode, the mean into the push request at local[vid].
constexpr uint32_t kLrShort = 32;

struct LrReduce {
  const uint32_t *uniq, *cnt, *off, *nruns;
  const float *val;      // the batch's gradient records e*x_i in key-sorted order (k_lr_records)
  const uint32_t *urow;  // shard row per run (single GPU)
  float *rows;
  float lr, fudge;
  const int32_t *local;
  float *grads;
  uint32_t *nlong, *longs;
  int fast;  // swps_lr_cfg.fast_sums: fp64 sums (tree-reduced for long runs) instead of the fp32 chain
  // inline records (k_lr_reduce_fused<true>): e[srow[i]] * sval[i] formed by the reduce itself
  const uint32_t *srow;  // the batch's sorted (row, x_i), from its first record
  const float *sval, *err;
};

// mean = s / count in fp32 (lr.cpp:32-38); fast mode passes the fp64 sum
__device__ __forceinline__ void lr_apply(const LrReduce &a, uint32_t r, float s, uint32_t c, double s64 = 0.0) {
  const float m = a.fast ? (float)(s64 / (double)c) : float(s / c);
  if (a.grads) {
    a.grads[a.local[a.uniq[r]]] = m;
    return;
  }
  float *row = a.rows + (uint64_t)a.urow[r] * 2;
  const float g2 = row[1] + m * m;
  row[1] = g2;
  const float step = a.lr * m;
  row[0] = row[0] + step / sqrtf(g2 + a.fudge);
}

__device__ __forceinline__ float lr_rec(const LrReduce &a, uint32_t i) { return a.val[i]; }

// A short run's records added in record order (fp64 for fast sums, fp32 for the exact chain),
// their loads issued 8 at a time instead of one per add: the same additions in the same order.
template <typename S> __device__ __forceinline__ S short_sum(const float *__restrict__ val, uint32_t o, uint32_t c) {
  S s = 0;
  for (uint32_t i = 0; i < c; i += 8) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = i + j < c ? val[o + i + j] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (i + j < c) s += (S)v[j];
  }
  return s;
}

// the batch's gradient records in key-sorted order: e[row]*x_i (fp32 product, = the
// reference's error * x) from the static sorted (row, x_i); e is L2-resident (4 B per row)
// Four records per thread with 16-B loads and stores: srow / sval / val are indexed by the
// records' absolute position i (val shifted by nz0 & 3 so that its 16-B groups line up with
// theirs); [i0, i1) is the batch's range.
__global__ void k_lr_records(const uint32_t *__restrict__ srow, const float *__restrict__ sval, uint64_t i0,
                             uint64_t i1, const float *__restrict__ err, float *__restrict__ val, int diag = 0) {
  const uint64_t g = (i0 >> 2) + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 16-B group
  const uint64_t b = g << 2;
  if (b >= i1) return;
  if (b >= i0 && b + 4 <= i1) {
    uint4 r = ((const uint4 *)srow)[g];
    if (diag & 4) {  // SWPS_LR_DIAG timing experiment only: coalesced e reads instead of the gathers
      const uint32_t c = (uint32_t)(b - i0) & 0xFFFCu;
      r = make_uint4(c + (r.x >> 31), c + 1, c + 2, c + 3);  // bench batches (>= 65,536 rows) only
    }
    const float4 x = ((const float4 *)sval)[g];
    ((float4 *)val)[g - (i0 >> 2)] = make_float4(err[r.x] * x.x, err[r.y] * x.y, err[r.z] * x.z, err[r.w] * x.w);
    return;
  }
  for (uint64_t i = max(b, i0); i < min(b + 4, i1); i++) val[i - ((i0 >> 2) << 2)] = err[srow[i]] * sval[i];
}

__global__ __launch_bounds__(256) void k_lr_reduce_short(LrReduce a) {
  const uint32_t R = *a.nruns;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < R; r += gridDim.x * blockDim.x) {
    const uint32_t o = a.off[r], c = a.cnt[r];
    if (c > kLrShort) {
      a.longs[atomicAdd(a.nlong, 1u)] = r;
      continue;
    }
    if (a.fast) {
      lr_apply(a, r, 0.f, c, short_sum<double>(a.val, o, c));
      continue;
    }
    lr_apply(a, r, short_sum<float>(a.val, o, c), c);
  }
}

// Long runs (hot features): the exact sequential fp32 chain is the bound, so
// keep it fed — the wave stages 512 records at a time into LDS with
// coalesced loads (next chunk's loads in flight) and lane 0 runs the add
// chain from LDS.
constexpr uint32_t kLrStage = 512;
__global__ __launch_bounds__(256) void k_lr_reduce_long(LrReduce a) {
  __shared__ float4 stage[4][kLrStage / 4];
  const int lane = threadIdx.x & 63;
  float4 *b4 = stage[threadIdx.x >> 6];
  float *b = (float *)b4;
  const uint32_t NL = *a.nlong;
  for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < NL; q += gridDim.x * 4) {
    const uint32_t r = a.longs[q];
    const uint32_t o = a.off[r], c = a.cnt[r];
    if (a.fast) {  // every lane sums a strided slice in fp64, then one fixed-order wave reduction
      double s4[4] = {0.0, 0.0, 0.0, 0.0};
      uint32_t k = lane;
      for (; k + 192 < c; k += 256) {
        s4[0] += (double)lr_rec(a, o + k);
        s4[1] += (double)lr_rec(a, o + k + 64);
        s4[2] += (double)lr_rec(a, o + k + 128);
        s4[3] += (double)lr_rec(a, o + k + 192);
      }
      for (; k < c; k += 64) s4[0] += (double)lr_rec(a, o + k);
      const double tot = wave_sum_pl((s4[0] + s4[1]) + (s4[2] + s4[3]));
      if (lane == 0) lr_apply(a, r, 0.f, c, tot);
      continue;
    }
    float s = 0;
    float x[kLrStage / 64];
#pragma unroll
    for (uint32_t u = 0; u < kLrStage / 64; u++) {
      const uint32_t k = u * 64 + lane;
      x[u] = k < c ? lr_rec(a, o + k) : 0.f;
    }
    for (uint32_t i = 0; i < c; i += kLrStage) {
      const uint32_t n = min(kLrStage, c - i);
#pragma unroll
      for (uint32_t u = 0; u < kLrStage / 64; u++) b[u * 64 + lane] = x[u];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // prefetch the next chunk while lane 0 sums this one
#pragma unroll
      for (uint32_t u = 0; u < kLrStage / 64; u++) {
        const uint32_t k = i + kLrStage + u * 64 + lane;
        x[u] = k < c ? lr_rec(a, o + k) : 0.f;
      }
      if (lane == 0) {
        uint32_t k = 0;
        for (; k + 16 <= n; k += 16) {
          const float4 v0 = b4[k / 4], v1 = b4[k / 4 + 1], v2 = b4[k / 4 + 2], v3 = b4[k / 4 + 3];
          s += v0.x; s += v0.y; s += v0.z; s += v0.w;
          s += v1.x; s += v1.y; s += v1.z; s += v1.w;
          s += v2.x; s += v2.y; s += v2.z; s += v2.w;
          s += v3.x; s += v3.y; s += v3.z; s += v3.w;
        }
        for (; k < n; k++) s += b[k];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) lr_apply(a, r, s, c);
  }
}

// A thread's fp64 share of a long run: accumulator j gets the thread's elements t + j*256,
// t + 2048 + j*256, ... in that order (then the tail into accumulator 0); 32 loads in flight
// while whole groups of 32 remain, then 8 — the same additions in the same order as 8 at a
// time throughout (bit-identical), with four times the loads in flight on hot runs.
__device__ __forceinline__ double long_share(const float *__restrict__ val, uint32_t o, uint32_t c, int t) {
  double s8[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  uint32_t k = t;
  for (; k + 31 * 256 < c; k += 32 * 256) {
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; j++) v[j] = val[o + k + j * 256];
#pragma unroll
    for (int j = 0; j < 32; j++) s8[j & 7] += (double)v[j];
  }
  for (; k + 7 * 256 < c; k += 8 * 256) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = val[o + k + j * 256];
#pragma unroll
    for (int j = 0; j < 8; j++) s8[j] += (double)v[j];
  }
  for (; k < c; k += 256) s8[0] += (double)val[o + k];
  return ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
}

// The same two sums with the records formed inline (e[srow[i]] * sval[i], the fp32 product
// k_lr_records stores): the (row, x_i) loads of a batch of records first, then their e gathers
// (L2-resident), then the additions in the same order — bit-identical, without k_lr_records'
// write and re-read of every record.
__device__ __forceinline__ double short_sum_inl(const LrReduce &a, uint32_t o, uint32_t c) {
  double s = 0;
  for (uint32_t i = 0; i < c; i += 8) {
    uint32_t rw[8];
    float x[8], v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const bool in = i + j < c;
      rw[j] = in ? a.srow[o + i + j] : 0u;
      x[j] = in ? a.sval[o + i + j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = i + j < c ? a.err[rw[j]] * x[j] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (i + j < c) s += (double)v[j];
  }
  return s;
}
__device__ __forceinline__ double long_share_inl(const LrReduce &a, uint32_t o, uint32_t c, int t) {
  double s8[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  uint32_t k = t;
  for (; k + 31 * 256 < c; k += 32 * 256) {
    uint32_t rw[32];
    float x[32];
#pragma unroll
    for (int j = 0; j < 32; j++) {
      rw[j] = a.srow[o + k + j * 256];
      x[j] = a.sval[o + k + j * 256];
    }
#pragma unroll
    for (int j = 0; j < 32; j++) s8[j & 7] += (double)(a.err[rw[j]] * x[j]);
  }
  for (; k + 7 * 256 < c; k += 8 * 256) {
    uint32_t rw[8];
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; j++) {
      rw[j] = a.srow[o + k + j * 256];
      x[j] = a.sval[o + k + j * 256];
    }
#pragma unroll
    for (int j = 0; j < 8; j++) s8[j] += (double)(a.err[rw[j]] * x[j]);
  }
  for (; k < c; k += 256) s8[0] += (double)(a.err[a.srow[o + k]] * a.sval[o + k]);
  return ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
}

// fast_sums, long runs (hot features: up to one record per row of the batch):
// one 256-thread block per run, 8 loads in flight per thread, fp64 partial per
// thread -> wave sums -> the 4 wave sums added in wave order (fixed order:
// deterministic run to run).
__global__ __launch_bounds__(256) void k_lr_reduce_long_fast(LrReduce a) {
  __shared__ double ws[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t NL = *a.nlong;
  for (uint32_t q = blockIdx.x; q < NL; q += gridDim.x) {
    const uint32_t r = a.longs[q];
    const uint32_t o = a.off[r], c = a.cnt[r];
    const double tot = wave_sum_pl(long_share(a.val, o, c, t));
    if (lane == 0) ws[wv] = tot;
    __syncthreads();
    if (t == 0) lr_apply(a, r, 0.f, c, ((ws[0] + ws[1]) + (ws[2] + ws[3])));
    __syncthreads();
  }
}

// fast_sums in one launch: the batch's long runs (> kLrShort records) come from a static list
// built at load (the run lengths depend only on the data), so the first LB blocks reduce them
// (one block per run, as k_lr_reduce_long_fast) while the other blocks take the short runs (a
// thread per run, as k_lr_reduce_short): no counter reset, no dependency between the two, one
// launch instead of three.  Same sums in the same order: bit-identical.
template <bool INL>
__global__ __launch_bounds__(256) void k_lr_reduce_fused(LrReduce a, const uint32_t *__restrict__ slong,
                                                         uint32_t NL, uint32_t LB) {
  __shared__ double ws[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (blockIdx.x < LB) {
    for (uint32_t q = blockIdx.x; q < NL; q += LB) {
      const uint32_t r = slong[q];
      const uint32_t o = a.off[r], c = a.cnt[r];
      const double tot = wave_sum_pl(INL ? long_share_inl(a, o, c, t) : long_share(a.val, o, c, t));
      if (lane == 0) ws[wv] = tot;
      __syncthreads();
      if (t == 0) lr_apply(a, r, 0.f, c, ((ws[0] + ws[1]) + (ws[2] + ws[3])));
      __syncthreads();
    }
    return;
  }
  const uint32_t R = *a.nruns;
  for (uint32_t r = (blockIdx.x - LB) * blockDim.x + t; r < R; r += (gridDim.x - LB) * blockDim.x) {
    const uint32_t o = a.off[r], c = a.cnt[r];
    if (c > kLrShort) continue;  // a long run: the first LB blocks
    lr_apply(a, r, 0.f, c, INL ? short_sum_inl(a, o, c) : short_sum<double>(a.val, o, c));
  }
}

// ---- fast sums through row tiles (k_lr_tiles + k_lr_tiles_fin) --------------------------
// The record path's cost is its e gathers (e[row] for every record of the batch, rows in
// random order within a key's run): 2.56M divergent 4-B reads per Criteo batch.  Cut the batch
// into tiles of 2^tb rows: the static index orders each batch's records by (tile, key), so a
// block loads its tile's slice of e into LDS once and reads every record's e from LDS.  A block
// takes kTileChunk (1,536) consecutive records of one tile (6 per thread, coalesced) and sums each key's
// records with one block-wide segmented scan; a piece = a key's records inside one block.  A key
// with a single piece is applied by k_lr_tiles itself; the others get one fp64 partial per piece,
// added in (tile, record) order by k_lr_tiles_fin.  Same fp32 products e*x_i as the record path,
// fp64 sums in a fixed order: deterministic, within fp64 rounding of k_lr_reduce_fused.
constexpr int kTileMaxBits = 12;         // LDS slice: 4,096 rows (16 KB)
// records per block (SWPS_LR_TILE_CHUNK: 512 / 1024 / 1280 / 1536 / 1792 / 2048 / 4096; same-box A/B at the
// Criteo batch, round 4: 1024 -> 1536 took the tiles group from 28.0 to 25.1 us — 1,664 blocks of
// 6 records per thread instead of 2,497 of 4, so every block is resident at once)
constexpr uint32_t kTileChunk = 1536;
constexpr uint16_t kTileHead = 0x8000;   // trow bit: the record starts a (tile, key) run

struct LrTiles {
  const uint16_t *trow;   // record's row within its tile | kTileHead
  const float *tval;      // record's x_i
  const uint32_t *chunk;  // per block: tile, first record, end record, first piece, end piece
  const uint32_t *tinfo;  // per piece: run (batch-relative) | 1u << 31 when the run is this one piece
  const uint32_t *tdst;   // per piece: its partial's slot (batch-relative), or for a whole run on a
                          // single GPU its key's shard row
  double *part;
  const float *err;
  uint64_t r0, nrb;
  int tb;
  int diag;  // SWPS_LR_DIAG timing experiments only: 8 no piece ends, 16 no e slice fill
};

// segmented-sum scan element (a head seen, open run's sum, heads, last head's record):
// (fp, vp, cp, hp) precedes (f, v, c, h)
__device__ __forceinline__ void seg_after(bool fp, double vp, int cp, uint32_t hp, bool &f, double &v, int &c,
                                          uint32_t &h) {
  if (!f) v = vp + v;
  f = f || fp;
  c += cp;
  h = max(h, hp);
}

template <int RPT, int BS = 256>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RPT > 8 ? 3 : 8))) void k_lr_tiles(LrReduce a, LrTiles t) {
  constexpr int NW = BS / 64;
  __shared__ float es[1 << kTileMaxBits];
  __shared__ double wv[NW];
  __shared__ int wf[NW], wc[NW];
  __shared__ uint32_t wh[NW];
  const uint32_t *ch = t.chunk + (uint64_t)blockIdx.x * 5;
  const uint32_t tile = ch[0], rec0 = ch[1], rec1 = ch[2], piece0 = ch[3];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t i0 = rec0 + (uint32_t)tid * RPT;
  const int n = i0 < rec1 ? (int)min((uint32_t)RPT, rec1 - i0) : 0;
  uint32_t rw[RPT + 1];
  float x[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    rw[j] = j < n ? t.trow[i0 + j] : 0u;
    x[j] = j < n ? t.tval[i0 + j] : 0.f;
  }
  rw[RPT] = n == RPT && i0 + RPT < rec1 ? t.trow[i0 + RPT] : kTileHead;  // the next record: a head ends this thread's last run
  const uint64_t e0 = (uint64_t)tile << t.tb;
  const uint32_t ne = (uint32_t)min<uint64_t>(1ull << t.tb, t.nrb - e0);
  if (!(t.diag & 16)) {  // the tile's slice of e: 16-B loads from the aligned base below it, all in
    // flight, then the LDS stores (err is allocated with 4 floats of slack past its last row)
    constexpr int KE = ((1 << kTileMaxBits) + 4 + 4 * BS - 1) / (4 * BS);
    const uint64_t g0 = t.r0 + e0, gb = g0 & ~3ull;
    const int sh = (int)(g0 - gb);
    const uint32_t nq = (ne + sh + 3) / 4;
    float4 ev[KE];
#pragma unroll
    for (int k = 0; k < KE; k++) {
      const uint32_t q = tid + k * BS;
      ev[k] = q < nq ? ((const float4 *)(t.err + gb))[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < KE; k++) {
      const int i = (int)(tid + k * BS) * 4 - sh;
      if (i >= 0 && i < (int)ne) es[i] = ev[k].x;
      if (i + 1 >= 0 && i + 1 < (int)ne) es[i + 1] = ev[k].y;
      if (i + 2 >= 0 && i + 2 < (int)ne) es[i + 2] = ev[k].z;
      if (i + 3 >= 0 && i + 3 < (int)ne) es[i + 3] = ev[k].w;
    }
  }
  __syncthreads();
  double pr[RPT];
  bool any = false;
  double pre = 0, cur = 0;
  int nh = 0;
  uint32_t lh = 0;
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    pr[j] = j < n ? (double)(es[rw[j] & (kTileHead - 1)] * x[j]) : 0.0;
    const bool h = j < n && ((rw[j] & kTileHead) || i0 + j == rec0);
    if (h) {
      any = true;
      nh++;
      lh = i0 + j;
      cur = pr[j];
    } else if (j < n) {
      if (any)
        cur += pr[j];
      else
        pre += pr[j];
    }
  }
  // block-wide exclusive segmented scan: the sum of this thread's open run before its first
  // record, the heads before it and the last one's record
  bool f = any;
  double v = any ? cur : pre;
  int c = nh;
  uint32_t hh = lh;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double vp = __shfl_up(v, o);
    const int fp = __shfl_up((int)f, o), cp = __shfl_up(c, o);
    const uint32_t hp = __shfl_up(hh, o);
    if (lane >= o) seg_after(fp != 0, vp, cp, hp, f, v, c, hh);
  }
  if (lane == 63) {
    wv[w] = v;
    wf[w] = f;
    wc[w] = c;
    wh[w] = hh;
  }
  double ve = __shfl_up(v, 1);
  int fe = __shfl_up((int)f, 1), ce = __shfl_up(c, 1);
  uint32_t he = __shfl_up(hh, 1);
  if (lane == 0) {
    ve = 0;
    fe = 0;
    ce = 0;
    he = 0;
  }
  __syncthreads();
  bool fw = false;
  double vw = 0;
  int cw = 0;
  uint32_t hw = 0;
  for (int k = 0; k < w; k++) {
    bool fk = wf[k] != 0;
    double vk = wv[k];
    int ck = wc[k];
    uint32_t hk = wh[k];
    seg_after(fw, vw, cw, hw, fk, vk, ck, hk);
    fw = fk;
    vw = vk;
    cw = ck;
    hw = hk;
  }
  bool fx = fe != 0;
  double run = ve;
  int cx = ce;
  uint32_t hs = he;
  seg_after(fw, vw, cw, hw, fx, run, cx, hs);
  // this thread's pieces that end here, in record order: (piece, sum, record count)
  uint32_t p = (uint32_t)cx - 1;  // block-local index of the piece open before this thread's first record
  uint32_t pj[RPT], cj[RPT];
  double sj[RPT];
  bool ej[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    const bool h = (rw[j] & kTileHead) || i0 + j == rec0;
    if (h) {
      p++;
      hs = i0 + j;
      run = pr[j];
    } else {
      run = run + pr[j];
    }
    ej[j] = j < n && (j + 1 < n ? (rw[j + 1] & kTileHead) != 0 : (n < RPT || (rw[RPT] & kTileHead) != 0));
    pj[j] = p;
    cj[j] = i0 + j - hs + 1;
    sj[j] = run;
  }
  if (t.diag & 8) {
    if (sj[0] == 12345.678) t.part[0] = sj[1];  // keeps the sums live
    return;
  }
  // a piece that is its key's whole run: the mean and AdaGrad; else its partial.  Every stage's
  // loads in flight together (a piece end at a time would chain the round trips: vmcnt orders
  // them behind the stores)
  uint32_t info[RPT], dst[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    info[j] = ej[j] ? t.tinfo[piece0 + pj[j]] : 0u;
    dst[j] = ej[j] ? t.tdst[piece0 + pj[j]] : 0u;
  }
  if (a.grads) {  // sharded: the mean into the push request at local[vid]
    uint32_t u[RPT];
#pragma unroll
    for (int j = 0; j < RPT; j++) u[j] = ej[j] && (info[j] >> 31) ? a.uniq[info[j] & 0x7FFFFFFFu] : 0u;
    int32_t lo[RPT];
#pragma unroll
    for (int j = 0; j < RPT; j++) lo[j] = ej[j] && (info[j] >> 31) ? a.local[u[j]] : 0;
#pragma unroll
    for (int j = 0; j < RPT; j++) {
      if (!ej[j]) continue;
      if (info[j] >> 31)
        a.grads[lo[j]] = (float)(sj[j] / (double)cj[j]);
      else
        t.part[dst[j]] = sj[j];
    }
    return;
  }
  float w0[RPT], g0[RPT];
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    const bool one = ej[j] && (info[j] >> 31);
    w0[j] = one ? a.rows[(uint64_t)dst[j] * 2] : 0.f;
    g0[j] = one ? a.rows[(uint64_t)dst[j] * 2 + 1] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < RPT; j++) {
    if (!ej[j]) continue;
    if (info[j] >> 31) {  // lr_apply's AdaGrad step (lr.cpp:68-75) on the shard row
      const float m = (float)(sj[j] / (double)cj[j]);
      const float g2 = g0[j] + m * m;
      const float step = a.lr * m;
      float *row = a.rows + (uint64_t)dst[j] * 2;
      row[1] = g2;
      row[0] = w0[j] + step / sqrtf(g2 + a.fudge);
    } else {
      t.part[dst[j]] = sj[j];
    }
  }
}

// keys with several partials, from static per-key records {first slot, partials, records,
// run (global)} (+ the run's shard row on a single GPU, so the row loads go out with the partial
// loads): the first LB blocks take the keys with more than kTileFinShort partials (a wave each:
// lane-strided fp64 adds, then the fixed-order wave sum), the rest a thread per key (its
// partials added in slot order); then the mean and AdaGrad
constexpr uint32_t kTileFinShort = 16;
__device__ __forceinline__ void fin_apply(const LrReduce &a, uint4 rc, uint32_t row, float w, float g, double s,
                                          uint64_t q0) {
  const float m = (float)(s / (double)rc.z);
  if (a.grads) {
    a.grads[a.local[a.uniq[rc.w - q0]]] = m;
    return;
  }
  const float g2 = g + m * m;
  const float step = a.lr * m;
  float *r = a.rows + (uint64_t)row * 2;
  r[1] = g2;
  r[0] = w + step / sqrtf(g2 + a.fudge);
}
// cnt != nullptr (the per-step plan): ns = cnt[0], nl = cnt[1] from the device, the grid an upper bound
__global__ __launch_bounds__(256) void k_lr_tiles_fin(LrReduce a, const uint4 *__restrict__ ms,
                                                      const uint32_t *__restrict__ msrow, uint32_t ns,
                                                      const uint4 *__restrict__ ml, const uint32_t *__restrict__ mlrow,
                                                      uint32_t nl, uint32_t LB, const double *__restrict__ part,
                                                      uint64_t q0, const uint32_t *__restrict__ cnt = nullptr) {
  const int lane = threadIdx.x & 63;
  if (cnt) {
    ns = cnt[0];
    nl = cnt[1];
  }
  if (blockIdx.x < LB) {
    for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < nl; q += LB * 4) {
      const uint4 rc = ml[q];
      const uint32_t row = a.grads ? 0u : mlrow[q];
      double s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      uint32_t k = lane;
      for (; k + 7 * 64 < rc.y; k += 8 * 64) {
        double v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = part[rc.x + k + j * 64];
#pragma unroll
        for (int j = 0; j < 8; j++) s8[j] += v[j];
      }
      for (; k < rc.y; k += 64) s8[0] += part[rc.x + k];
      const double tot = wave_sum_pl(((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7])));
      if (lane == 0)
        fin_apply(a, rc, row, a.grads ? 0.f : a.rows[(uint64_t)row * 2], a.grads ? 0.f : a.rows[(uint64_t)row * 2 + 1],
                  tot, q0);
    }
    return;
  }
  for (uint32_t q = (blockIdx.x - LB) * blockDim.x + threadIdx.x; q < ns; q += (gridDim.x - LB) * blockDim.x) {
    const uint4 rc = ms[q];
    const uint32_t row = a.grads ? 0u : msrow[q];
    double v[kTileFinShort];
#pragma unroll
    for (int j = 0; j < (int)kTileFinShort; j++) v[j] = (uint32_t)j < rc.y ? part[rc.x + j] : 0.0;
    const float w = a.grads ? 0.f : a.rows[(uint64_t)row * 2], g = a.grads ? 0.f : a.rows[(uint64_t)row * 2 + 1];
    double s = 0;
#pragma unroll
    for (int j = 0; j < (int)kTileFinShort; j++)
      if ((uint32_t)j < rc.y) s += v[j];
    fin_apply(a, rc, row, w, g, s, q0);
  }
}

// ---- the tile index (built at load with the record index; fast sums) ----
__global__ void k_lr_tile_keys(const uint64_t *__restrict__ row_off, uint64_t nr, uint64_t B1, int tb, int tbits,
                               const int32_t *__restrict__ fvid, uint64_t *__restrict__ key, uint32_t *__restrict__ idx) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  const uint64_t b = r / B1, tile = (r - b * B1) >> tb;
  for (uint64_t c = row_off[r]; c < row_off[r + 1]; c++) {
    key[c] = (b << (32 + tbits)) | (tile << 32) | (uint32_t)fvid[c];
    idx[c] = (uint32_t)c;
  }
}

// records in (batch, tile, key) order: row within the tile (+ the run-head bit), x_i, piece heads
__global__ void k_lr_tile_slots(const uint64_t *__restrict__ ks, const uint32_t *__restrict__ perm, uint64_t n,
                                const uint32_t *__restrict__ rid, uint64_t B1, int tb, const float *__restrict__ fval,
                                uint16_t *__restrict__ trow, float *__restrict__ tval, uint32_t *__restrict__ head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t c = perm[i];
  const bool h = i == 0 || ks[i] != ks[i - 1];
  trow[i] = (uint16_t)(((rid[c] % B1) & ((1u << tb) - 1)) | (h ? kTileHead : 0));
  tval[i] = fval[c];
  head[i] = h ? 1u : 0u;
}
__global__ void k_lr_tile_cuts(const uint32_t *__restrict__ cut, uint64_t nc, uint32_t *__restrict__ head) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nc) head[cut[q]] = 1u;
}
// pieces: first record and (batch, key); chunk -> its first piece
__global__ void k_lr_tile_pieces(const uint64_t *__restrict__ ks, const uint32_t *__restrict__ head,
                                 const uint32_t *__restrict__ pidr, uint64_t n, int tbits,
                                 uint64_t *__restrict__ tkey2, uint32_t *__restrict__ pid) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !head[i]) return;
  const uint32_t q = pidr[i] - 1;
  const uint64_t k = ks[i];
  tkey2[q] = ((k >> (32 + tbits)) << 32) | (uint32_t)k;  // (batch, key): pieces in record order after a stable sort
  pid[q] = q;
}
__global__ void k_lr_tile_first(const uint32_t *__restrict__ cut, uint64_t nc, const uint32_t *__restrict__ pidr,
                                uint32_t *__restrict__ piece0) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nc) piece0[q] = pidr[cut[q]] - 1;
}
__global__ void k_lr_tile_heads(const uint64_t *__restrict__ k2s, uint64_t S2, uint32_t *__restrict__ head) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < S2) head[j] = (j == 0 || k2s[j] != k2s[j - 1]) ? 1u : 0u;
}
// piece -> its slot (position in (batch, key, record) order, batch-relative); run -> first slot
__global__ void k_lr_tile_link(const uint64_t *__restrict__ k2s, const uint32_t *__restrict__ perm2,
                               const uint32_t *__restrict__ head, const uint32_t *__restrict__ gid, uint64_t S2,
                               const uint64_t *__restrict__ bsub, uint32_t *__restrict__ tslot,
                               uint32_t *__restrict__ pfirst) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= S2) return;
  tslot[perm2[j]] = (uint32_t)(j - bsub[k2s[j] >> 32]);
  if (head[j]) pfirst[gid[j] - 1] = (uint32_t)j;
}
__global__ void k_lr_tile_np(const uint32_t *__restrict__ pfirst, uint64_t R, uint64_t S2,
                             const uint64_t *__restrict__ rkey, const uint64_t *__restrict__ bsub,
                             uint32_t *__restrict__ np, uint32_t *__restrict__ pst) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= R) return;
  np[g] = (g + 1 < R ? pfirst[g + 1] : (uint32_t)S2) - pfirst[g];
  pst[g] = (uint32_t)(pfirst[g] - bsub[rkey[g] >> 32]);
}
__global__ void k_lr_tile_info(const uint64_t *__restrict__ k2s, const uint32_t *__restrict__ perm2,
                               const uint32_t *__restrict__ gid, uint64_t S2, const uint64_t *__restrict__ brun,
                               const uint32_t *__restrict__ np, uint32_t *__restrict__ tinfo,
                               uint32_t *__restrict__ tgrun) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= S2) return;
  const uint64_t g = gid[j] - 1;
  tinfo[perm2[j]] = (uint32_t)(g - brun[k2s[j] >> 32]) | (np[g] == 1 ? 0x80000000u : 0u);
  tgrun[perm2[j]] = (uint32_t)g;
}
__global__ void k_lr_tile_mrow(const uint4 *__restrict__ m, uint64_t n, const uint32_t *__restrict__ urow,
                               uint32_t *__restrict__ row) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) row[q] = urow[m[q].w];
}
// single GPU, once the runs' shard rows are known: a whole-run piece's destination is its row
__global__ void k_lr_tile_dst(const uint32_t *__restrict__ tinfo, const uint32_t *__restrict__ tslot,
                              const uint32_t *__restrict__ tgrun, uint64_t S2, const uint32_t *__restrict__ urow,
                              uint32_t *__restrict__ tdst) {
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < S2) tdst[p] = (tinfo[p] >> 31) ? urow[tgrun[p]] : tslot[p];
}

// ---- the per-step plan (swps_lr_cfg.plan = SWPS_LR_PLAN_STEP, the default) -------------------
// What the static index (lr_index + lr_tile_index) builds for every batch at load, built for one
// batch on a plan stream while the previous batch trains: lr.cpp:215-227 gathers, dedups and pulls
// each minibatch's keys inside its training loop, and so does this path — on the GPU, with no host
// round trip.  Two orders of the batch's records:
//   K order — stable by vid: one run per pushed key, a key's records in row order;
//   T order — K order stable by row tile: the (tile, key) order the row tiles (k_lr_tiles) walk.
// A piece (a key's records inside one kTileChunk block of a tile) starts at a (tile, key) head or
// at a block cut in T order.  In K order a key's pieces appear in T order, so one scan of the
// piece heads in K order numbers the partial slots in (key, piece) order: the static index's
// slots.  Same records, pieces, partial slots and sums as the static index: bit-identical.
constexpr uint32_t kPlanHotBins = 80;  // record counts >= 8 in quarter-octave bins
__device__ __forceinline__ uint32_t plan_hot_bin(uint32_t recs) {
  const uint32_t lg = 31u - (uint32_t)__clz(recs);  // recs >= 8: lg >= 3
  return min(4u * lg + ((recs >> (lg - 2)) & 3u), kPlanHotBins - 1);
}
// one block: zero the plan's counters, the hot histogram and hot rows; each tile's first block
// (the exclusive scan of its kTileChunk-record block counts, from the CSR)
__global__ __launch_bounds__(1024) void k_plan_reset(const uint64_t *__restrict__ row_off, uint64_t r0, uint64_t nrb,
                                                     int tb, uint32_t chunk, uint64_t ntile,
                                                     uint32_t *__restrict__ tfirst, uint32_t *__restrict__ cnt,
                                                     uint32_t *__restrict__ hist, uint32_t *__restrict__ hrow,
                                                     uint32_t nhrow) {
  __shared__ uint32_t part[1024];
  const uint32_t tid = threadIdx.x;
  if (tid < 4) cnt[tid] = 0;
  if (tid < kPlanHotBins) hist[tid] = 0;
  for (uint32_t q = tid; q < nhrow; q += 1024) hrow[q] = 0;  // unused slots read row 0 (never referenced)
  const uint64_t per = (ntile + 1023) / 1024, t0 = tid * per, t1 = min(ntile, t0 + per);
  auto nchunks = [&](uint64_t tl) {
    const uint64_t rs = r0 + (tl << tb), re = r0 + min(nrb, (tl + 1) << tb);
    return (uint32_t)((row_off[re] - row_off[rs] + chunk - 1) / chunk);
  };
  uint32_t s = 0;
  for (uint64_t tl = t0; tl < t1; tl++) s += nchunks(tl);
  part[tid] = s;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive scan over the threads' sums
    const uint32_t v = tid >= o ? part[tid - o] : 0u;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = part[tid] - s;
  for (uint64_t tl = t0; tl < t1; tl++) {
    tfirst[tl] = run;
    run += nchunks(tl);
  }
}
// K order: each record's row (batch-relative) and tile, and whether it starts its key's records in
// its tile — a (tile, key) run head in T order — carried into the tile sort's values
__global__ void k_plan_tile(const uint32_t *__restrict__ permK, const uint32_t *__restrict__ ks1,
                            const uint32_t *__restrict__ rid, uint64_t z0, uint64_t r0, uint64_t n, int tb,
                            uint32_t *__restrict__ tkey, uint32_t *__restrict__ val2, uint32_t *__restrict__ rowK) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t r = rid[z0 + permK[j]] - (uint32_t)r0, tile = r >> tb;
  bool head = j == 0;
  if (!head) head = ks1[j] != ks1[j - 1] || ((rid[z0 + permK[j - 1]] - (uint32_t)r0) >> tb) != tile;
  tkey[j] = tile;
  rowK[j] = r;
  val2[j] = (uint32_t)j | (head ? 0x80000000u : 0u);
}
// T order: the records' (row in tile | run head, x_i), piece heads (run head or block cut), and
// every K position's T position
__global__ void k_plan_torder(const uint32_t *__restrict__ v2s, const uint32_t *__restrict__ tks,
                              const uint32_t *__restrict__ rowK, const uint32_t *__restrict__ permK,
                              const float *__restrict__ fval, const uint64_t *__restrict__ row_off, uint64_t r0,
                              uint64_t z0, uint64_t n, int tb, uint32_t chunk, uint16_t *__restrict__ trow,
                              float *__restrict__ tval, uint32_t *__restrict__ ph, uint32_t *__restrict__ invT) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const uint32_t v = v2s[t], j = v & 0x7FFFFFFFu, tile = tks[t];
  const bool head = (v >> 31) != 0;
  trow[t] = (uint16_t)((rowK[j] & ((1u << tb) - 1)) | (head ? kTileHead : 0));
  tval[t] = fval[z0 + permK[j]];
  const uint64_t ts = row_off[r0 + ((uint64_t)tile << tb)] - z0;  // the tile's first record (T = CSR at tiles)
  ph[t] = (head || (t - ts) % chunk == 0) ? 1u : 0u;
  invT[j] = (uint32_t)t;
}
// K order: (piece head << 32 | key head), scanned together
__global__ void k_plan_kflags(const uint32_t *__restrict__ ks1, const uint32_t *__restrict__ invT,
                              const uint32_t *__restrict__ ph, uint64_t n, uint64_t *__restrict__ packed) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  packed[j] = ((uint64_t)ph[invT[j]] << 32) | ((j == 0 || ks1[j] != ks1[j - 1]) ? 1u : 0u);
}
__global__ void k_plan_kstart(const uint64_t *__restrict__ pk, uint64_t n, uint32_t *__restrict__ kstart) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t k = (uint32_t)pk[j];
  if (j == 0 || (uint32_t)pk[j - 1] != k) kstart[k - 1] = (uint32_t)j;
}
// a wave's lanes with `take` get consecutive slots of *ctr (one atomic per wave)
__device__ __forceinline__ uint32_t wave_claim(bool take, uint32_t *ctr) {
  const uint64_t m = __ballot(take);
  if (!m) return 0;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  return base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
}
// per key (grid-stride over the batch's U keys, U on the device): its partial slots, records and
// shard row; the keys with several pieces into the finisher's lists (any order: each key's
// partials are summed in slot order whatever its list position); the hot-key histogram (per block
// in LDS, then one atomic per bin)
__global__ __launch_bounds__(256) void k_plan_kinfo(const uint32_t *__restrict__ kstart, const uint64_t *__restrict__ pk,
                                                    uint64_t n, const uint32_t *__restrict__ ks1,
                                                    const uint32_t *__restrict__ vid_row, uint32_t *__restrict__ kwhole,
                                                    uint32_t *__restrict__ krow, uint4 *__restrict__ ms,
                                                    uint32_t *__restrict__ msrow, uint4 *__restrict__ ml,
                                                    uint32_t *__restrict__ mlrow, uint32_t *__restrict__ cnt,
                                                    uint32_t *__restrict__ hist) {
  __shared__ uint32_t lh[kPlanHotBins];
  for (uint32_t b = threadIdx.x; b < kPlanHotBins; b += blockDim.x) lh[b] = 0;
  __syncthreads();
  const uint32_t U = (uint32_t)pk[n - 1];
  const uint32_t stride = gridDim.x * blockDim.x;
  // every lane runs the same number of iterations (the wave-wide claims need whole waves)
  for (uint32_t k0 = blockIdx.x * blockDim.x; k0 < U; k0 += stride) {
    const uint32_t k = k0 + threadIdx.x;
    const bool on = k < U;
    uint32_t slot0 = 0, np = 0, recs = 0, row = 0;
    if (on) {
      const uint32_t s = kstart[k], e = k + 1 < U ? kstart[k + 1] : (uint32_t)n;
      slot0 = (uint32_t)(pk[s] >> 32) - 1;
      np = (uint32_t)(pk[e - 1] >> 32) - slot0;
      recs = e - s;
      row = vid_row[ks1[s]];
      kwhole[k] = np == 1 ? 1u : 0u;
      krow[k] = row;
    }
    const bool shrt = on && np > 1 && np <= kTileFinShort, lng = on && np > kTileFinShort;
    const uint32_t qs = wave_claim(shrt, &cnt[0]), ql = wave_claim(lng, &cnt[1]);
    if (shrt) {
      ms[qs] = make_uint4(slot0, np, recs, k);
      msrow[qs] = row;
    }
    if (lng) {
      ml[ql] = make_uint4(slot0, np, recs, k);
      mlrow[ql] = row;
    }
    if (hist && on && recs >= 8) atomicAdd(&lh[plan_hot_bin(recs)], 1u);
  }
  if (!hist) return;
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kPlanHotBins; b += blockDim.x)
    if (lh[b]) atomicAdd(&hist[b], lh[b]);
}
// the hot keys: every key in a bin above the threshold bin, then keys of that bin while slots
// remain (which of those get in changes nothing but the LDS they are read from)
__global__ void k_plan_hot_thresh(const uint32_t *__restrict__ hist, uint32_t nhot, uint32_t *__restrict__ thr) {
  if (threadIdx.x != 0) return;
  uint32_t above = 0;
  int T = -1;
  for (int b = (int)kPlanHotBins - 1; b >= 0; b--) {
    if (above + hist[b] >= nhot) {
      T = b;
      break;
    }
    above += hist[b];
  }
  thr[0] = T < 0 ? 0u : (uint32_t)T;  // fewer candidates than slots: all of them (above = their count)
  thr[1] = 0;                         // next slot for keys above the threshold bin
  thr[2] = T < 0 ? nhot : above;      // next slot for keys of the threshold bin
  thr[3] = T < 0 ? 1u : 0u;
}
__global__ void k_plan_hot_assign(const uint32_t *__restrict__ kstart, const uint64_t *__restrict__ pk, uint64_t n,
                                  const uint32_t *__restrict__ krow, uint32_t nhot, uint32_t *__restrict__ thr,
                                  int32_t *__restrict__ khot, uint32_t *__restrict__ hrow) {
  const uint32_t U = (uint32_t)pk[n - 1];
  const uint32_t T = thr[0];
  const bool all = thr[3] != 0;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < U; k += gridDim.x * blockDim.x) {
    const uint32_t e = k + 1 < U ? kstart[k + 1] : (uint32_t)n;
    const uint32_t recs = e - kstart[k];
    int32_t h = -1;
    if (recs >= 8) {
      const uint32_t b = plan_hot_bin(recs);
      if (all || b > T) {
        h = (int32_t)atomicAdd(&thr[1], 1u);
      } else if (b == T) {
        const uint32_t q = atomicAdd(&thr[2], 1u);
        if (q < nhot) h = (int32_t)q;
      }
    }
    khot[k] = h;
    if (h >= 0) hrow[h] = krow[k];
  }
}
// every record (K order): its forward code (hot rank or shard row) at its CSR position; every
// piece head: its destination (a whole run's shard row, else its partial slot) and whole-run flag
__global__ void k_plan_records(const uint64_t *__restrict__ pk, const uint32_t *__restrict__ permK,
                               const uint32_t *__restrict__ invT, const uint32_t *__restrict__ pidT, uint64_t n,
                               const uint32_t *__restrict__ kwhole, const uint32_t *__restrict__ krow,
                               const int32_t *__restrict__ khot, uint32_t *__restrict__ fcode,
                               uint32_t *__restrict__ tinfo, uint32_t *__restrict__ tdst) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t v = pk[j];
  const uint32_t k = (uint32_t)v - 1, row = krow[k];
  const int32_t h = khot ? khot[k] : -1;
  fcode[permK[j]] = h >= 0 ? (kLrHotBit | (uint32_t)h) : row;
  if (j == 0 || (pk[j - 1] >> 32) != (v >> 32)) {
    const uint32_t q = pidT[invT[j]] - 1, whole = kwhole[k];
    tinfo[q] = whole ? 0x80000000u : 0u;
    tdst[q] = whole ? row : (uint32_t)(v >> 32) - 1;
  }
}
// the tiles' blocks, a thread per block: {tile, first / end record, first / end piece}
__global__ void k_plan_chunks(const uint64_t *__restrict__ row_off, uint64_t r0, uint64_t nrb, uint64_t z0, int tb,
                              uint32_t chunk, uint64_t ntile, const uint32_t *__restrict__ tfirst,
                              const uint32_t *__restrict__ pidT, uint64_t n, uint64_t nch, uint32_t *__restrict__ out) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nch) return;
  uint64_t lo = 0, hi = ntile;  // the last tile whose first block <= q (empty tiles own no block)
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (tfirst[mid] <= q)
      lo = mid;
    else
      hi = mid;
  }
  uint64_t tl = lo;
  while (tl + 1 < ntile && tfirst[tl + 1] <= q) tl++;
  const uint64_t rs = r0 + (tl << tb), re = r0 + min(nrb, (tl + 1) << tb);
  const uint64_t b = row_off[re] - z0;
  const uint64_t c0 = row_off[rs] - z0 + (q - tfirst[tl]) * chunk, c1 = min(b, c0 + chunk);
  uint32_t *e = out + q * 5;
  e[0] = (uint32_t)tl;
  e[1] = (uint32_t)c0;
  e[2] = (uint32_t)c1;
  e[3] = pidT[c0] - 1;
  e[4] = c1 < n ? pidT[c1] - 1 : pidT[n - 1];
}

// ---- the fixed-point step (swps_lr_cfg.plan = SWPS_LR_PLAN_NONE): no index at all ------------
// lr.cpp's minibatch as the reference runs it — gather the batch's keys, pull, learn, push the
// per-key mean — with the per-key gradient sums made order-free instead of sorted: every record's
// e*x_i (the reference's fp32 `grad`, lr.cpp:368) is added as a 64-bit fixed-point integer
// (scale 2^s chosen at load so that no sum can overflow: |sum| < 2^62), so the sums are exact
// integers whatever order the atomics land in — deterministic run to run, and each key's mean
// float(sum / count) is within a few 2^-s of the fp64 sum's (fast mode's definition).  A block
// takes a chunk of whole rows (k_lr_forward_c's forward: same products, same ordered fp32 row
// sums, the same e), then adds its records' terms: the hot keys' (the corpus's most frequent,
// fixed at load) into LDS, flushed with one global atomic per key per block; the rest straight to
// the key's accumulator.  The first add to a key (its count was 0) appends its shard row to the
// batch's pushed-key list; k_lr_fx_apply then applies the mean and AdaGrad to every listed row
// (lr.cpp:68-75) and clears its accumulator.  Keys are found per record from a per-key code
// (shard row, or hot rank | kLrHotBit) — the pull's lookup — with no per-batch index.
template <int RPT>
__global__ __launch_bounds__(256) void k_lr_fx_step(const uint2 *__restrict__ chunks,
                                                    const uint64_t *__restrict__ row_off,
                                                    const int32_t *__restrict__ fvid,
                                                    const uint32_t *__restrict__ vcode,
                                                    const float *__restrict__ fval, const float *__restrict__ label,
                                                    uint64_t r0, const float *__restrict__ rows,
                                                    const uint32_t *__restrict__ hrow, uint32_t nhot,
                                                    float *__restrict__ err, float *__restrict__ err2,
                                                    unsigned long long *__restrict__ acc_sum,
                                                    uint32_t *__restrict__ acc_cnt, uint32_t *__restrict__ list,
                                                    uint32_t *__restrict__ list_n, double scale,
                                                    uint32_t *__restrict__ stamp, uint32_t tag) {
  constexpr int CAP = RPT * 256;
  __shared__ float prod[CAP];
  __shared__ uint16_t rl[CAP];   // each record's row within the chunk
  __shared__ float es[CAP];      // each row's error
  __shared__ float wh[kLrHot];
  __shared__ unsigned long long hs[kLrHot];
  __shared__ uint32_t hc[kLrHot];
  __shared__ uint32_t bn, bbase;  // the block's first-touched rows (listed in prod's LDS once the sums are done)
  const int tid = threadIdx.x;
  HotW hw;
  hw.ld(rows, hrow, nhot, tid);
  for (uint32_t q = (uint32_t)tid; q < nhot; q += 256u) {
    hs[q] = 0ull;
    hc[q] = 0u;
  }
  if (tid == 0) bn = 0u;
  const uint2 ch = chunks[blockIdx.x];  // first row (batch-relative), rows
  const uint64_t rf = r0 + ch.x;
  const uint64_t c0 = row_off[rf], c1 = row_off[rf + ch.y];
  const uint32_t n = (uint32_t)(c1 - c0);
  int32_t f[RPT];
  float x[RPT];
#pragma unroll
  for (int k = 0; k < RPT; k++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)k * 256u;
    f[k] = i < n ? fvid[c0 + i] : 0;
    x[k] = i < n ? fval[c0 + i] : 0.f;
  }
  uint32_t code[RPT];
#pragma unroll
  for (int k = 0; k < RPT; k++) code[k] = ((uint32_t)tid + (uint32_t)k * 256u) < n ? vcode[f[k]] : 0u;
  uint64_t ra = 0, rb = 0;
  float y = 0.f;
  if ((uint32_t)tid < ch.y) {
    ra = row_off[rf + tid];
    rb = row_off[rf + tid + 1];
    y = label[rf + tid];
  }
  if (hrow) hw.st(wh, nhot, tid);
  __syncthreads();
  float w[RPT];
#pragma unroll
  for (int k = 0; k < RPT; k++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)k * 256u;
    w[k] = i >= n ? 0.f : (code[k] & kLrHotBit) ? wh[code[k] & (kLrHotBit - 1)] : rows[(uint64_t)code[k] * 2];
  }
#pragma unroll
  for (int k = 0; k < RPT; k++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)k * 256u;
    if (i < n) prod[i] = w[k] * x[k];
  }
  for (uint32_t r = (uint32_t)tid; r < ch.y; r += 256u) {  // each record's row
    const uint64_t a = r < 256u ? ra : row_off[rf + r], b = r < 256u ? rb : row_off[rf + r + 1];
    for (uint64_t c = a; c < b; c++) rl[c - c0] = (uint16_t)r;
  }
  __syncthreads();
  for (uint32_t r = (uint32_t)tid; r < ch.y; r += 256u) {  // lr.cpp:358-367, in feature order
    if (r >= 256u) {
      ra = row_off[rf + r];
      rb = row_off[rf + r + 1];
      y = label[rf + r];
    }
    float sum = 0.f;
    for (uint32_t c = (uint32_t)(ra - c0); c < (uint32_t)(rb - c0); c++) sum += prod[c];
    const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
    const float error = y - predict;
    err[rf + r] = error;
    err2[rf + r] = error * error;
    es[r] = error;
  }
  __syncthreads();
  uint32_t *blist = reinterpret_cast<uint32_t *>(prod);  // free now: CAP >= the block's records + hot keys
  // every record's term grad = error * x_i (lr.cpp:368) in fixed point
#pragma unroll
  for (int k = 0; k < RPT; k++) {
    const uint32_t i = (uint32_t)tid + (uint32_t)k * 256u;
    if (i < n) {
      const float g = es[rl[i]] * x[k];
      const unsigned long long q = (unsigned long long)__double2ll_rn((double)g * scale);
      if (code[k] & kLrHotBit) {
        const uint32_t h = code[k] & (kLrHotBit - 1);
        atomicAdd(&hs[h], q);
        atomicAdd(&hc[h], 1u);
      } else {
        const uint32_t row = code[k];
        atomicAdd(&acc_sum[row], q);  // no return value wanted: fire and forget
        atomicAdd(&acc_cnt[row], 1u);
        // the batch's first touch of the key lists it: a plain read filters the repeats (the tag is
        // written only by the exchange, so reading it means the key is listed already)
        if (stamp[row] != tag && atomicExch(&stamp[row], tag) != tag) blist[atomicAdd(&bn, 1u)] = row;
      }
    }
  }
  if (hrow) {
    __syncthreads();
    for (uint32_t q = (uint32_t)tid; q < nhot; q += 256u) {  // the hot keys: one global add per key per block
      const uint32_t c = hc[q];
      if (c) {
        const uint32_t row = hrow[q];
        atomicAdd(&acc_sum[row], hs[q]);
        atomicAdd(&acc_cnt[row], c);
        if (stamp[row] != tag && atomicExch(&stamp[row], tag) != tag) blist[atomicAdd(&bn, 1u)] = row;
      }
    }
  }
  __syncthreads();
  if (tid == 0) bbase = bn ? atomicAdd(list_n, bn) : 0u;  // one reservation per block
  __syncthreads();
  for (uint32_t q = (uint32_t)tid; q < bn; q += 256u) list[bbase + q] = blist[q];
}

// the batch's pushed keys: mean = float(sum / count) and AdaGrad on the shard row (lr.cpp:32-38,
// 68-75), the accumulator cleared for the next batch; zeroes the next batch's list counter
__global__ __launch_bounds__(256) void k_lr_fx_apply(const uint32_t *__restrict__ list,
                                                     const uint32_t *__restrict__ list_n,
                                                     uint32_t *__restrict__ next_n,
                                                     unsigned long long *__restrict__ acc_sum,
                                                     uint32_t *__restrict__ acc_cnt, float *__restrict__ rows, float lr,
                                                     float fudge, double inv_scale) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *next_n = 0u;
  const uint32_t n = *list_n;
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
    const uint32_t row = list[q];
    const long long s = (long long)acc_sum[row];
    const uint32_t c = acc_cnt[row];
    float *r = rows + (uint64_t)row * 2;
    const float w = r[0], g2 = r[1];
    acc_sum[row] = 0ull;
    acc_cnt[row] = 0u;
    const float m = (float)(((double)s * inv_scale) / (double)c);
    const float ng2 = g2 + m * m;
    const float step = lr * m;
    r[1] = ng2;
    r[0] = w + step / sqrtf(ng2 + fudge);
  }
}
// ---- the fixed-point step, bucketed (the default form of SWPS_LR_PLAN_NONE) ------------------
// The same integer sums as k_lr_fx_step, with no global atomic per record.  The vocabulary is cut
// into buckets of 2^kLrFxVB consecutive vids (a bucket's accumulators fit one block's LDS).
// k_lr_fxb_step: a block walks chunks of whole rows (forward as k_lr_fx_step); per chunk it sorts
//   its non-hot records by bucket in LDS (a counting sort: the order within a bucket is whatever
//   the LDS atomics give — the sums below do not depend on it) and writes them, (key, e*x_i as
//   fp32), into the chunk's own span of `rec` with the chunk's bucket offsets (boff[bucket]
//   [chunk], u16: one bucket's offsets contiguous for its reader); hot
//   keys' terms stay in the block's LDS over all its chunks and go out once, as one row of the
//   [block][hot] partial matrix (no atomics: every entry written).
// k_lr_fxb_push: block b < nbk owns bucket b: it adds every chunk's records of the bucket into LDS
//   (the fixed point of each term computed exactly as k_lr_fx_step does), then applies the mean
//   and AdaGrad to each touched key's shard row; the blocks after them each reduce 16 hot keys'
//   columns of the partial matrix and apply theirs.  Integer sums: the result is the atomic form's,
//   bit for bit, whatever the order.
constexpr int kLrFxVB = 12;
// the fill counters are packed [group][bucket]: one wave's reservations (consecutive buckets) are
// 64 consecutive words — a few 128-B requests at the memory side, not 64 (scattered returning
// atomics run ~17x slower per byte: MI355X_MICROARCH.md, Global float atomics)
constexpr uint32_t kLrFxMaxGBits = 4;      // at most 16 chunk groups per bucket region
constexpr uint32_t kLrFxMaxBk = 4096;  // buckets (V <= 2^24); beyond it the atomic form runs
template <int RPT, int NT, bool AFF, int HC, bool RES>
__global__ __launch_bounds__(NT) void k_lr_fxb_step(const uint2 *__restrict__ chunks, uint32_t nchunks,
                                                     const uint64_t *__restrict__ row_off,
                                                     const int32_t *__restrict__ fvid,
                                                     const uint32_t *__restrict__ vcode,
                                                     const float *__restrict__ fval, const float *__restrict__ label,
                                                     uint64_t r0, const float *__restrict__ rows,
                                                     const uint32_t *__restrict__ hrow, uint32_t nhot,
                                                     float *__restrict__ err, float *__restrict__ err2, double scale,
                                                     uint32_t nbk, uint2 *__restrict__ rec, uint16_t *__restrict__ boff,
                                                     uint32_t bstride,
                                                     unsigned long long *__restrict__ hsum,
                                                     uint32_t *__restrict__ hcnt, uint32_t row_base,
                                                     uint32_t *__restrict__ fill, const uint32_t *__restrict__ rbase,
                                                     uint32_t gbits, uint32_t diag) {
  constexpr int CAP = RPT * NT;
  // RES (the bucket regions): bucket q's records of the whole batch go to 2^gbits sub-regions of
  // rec, one per chunk group g = chunk % 2^gbits: [rbase[q << gbits | g], rbase[(q << gbits | g) + 1])
  // (sized at load for any batch), each chunk reserving its span there with one returning atomic on
  // fill[g * nbk + q] — issued as soon as the chunk's bucket counts are known,
  // waited for only at the record writes (the forward hides it), and spread over the groups' words
  // (a word takes about 88 returning atomics per us).  The records of a bucket land in an order that
  // varies run to run; their sums are exact integers, so the results do not (k_lr_fxb_push reads
  // the sub-regions as contiguous runs).
  __shared__ float prod[CAP];
  __shared__ uint16_t rl[CAP];
  __shared__ float es[CAP];
  __shared__ float wh[HC];
  __shared__ unsigned long long hs[HC];
  __shared__ uint32_t hc[HC];
  extern __shared__ uint32_t bc[];  // [nbk]: dynamic
  const int tid = threadIdx.x;
  constexpr int HPT = (HC + NT - 1) / NT;  // the block's hot weights: loads first, LDS stores later
  float hv[HPT];
#pragma unroll
  for (int j = 0; j < HPT; j++) {
    const uint32_t q = (uint32_t)tid + (uint32_t)(NT * j);
    hv[j] = hrow && q < nhot ? rows[(uint64_t)(AFF ? row_base + q : hrow[q]) * 2] : 0.f;
  }
  for (uint32_t q = (uint32_t)tid; q < nhot; q += (uint32_t)NT) {
    hs[q] = 0ull;
    hc[q] = 0u;
  }
#pragma unroll
  for (int j = 0; j < HPT; j++) {
    const uint32_t q = (uint32_t)tid + (uint32_t)(NT * j);
    if (hrow && q < nhot) wh[q] = hv[j];
  }
  const uint64_t z0 = row_off[r0];
  for (uint32_t cix = blockIdx.x; cix < nchunks; cix += gridDim.x) {
    const uint2 ch = chunks[cix];
    const uint64_t rf = r0 + ch.x;
    const uint64_t c0 = row_off[rf], c1 = row_off[rf + ch.y];
    const uint32_t n = (uint32_t)(c1 - c0);
    int32_t f[RPT];
    float x[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = (uint32_t)tid + (uint32_t)k * (uint32_t)NT;
      f[k] = i < n ? fvid[c0 + i] : 0;
      x[k] = i < n ? fval[c0 + i] : 0.f;
    }
    uint32_t code[RPT];  // AFF: f is the key's fid (hot keys first) and its shard row row_base + fid
#pragma unroll
    for (int k = 0; k < RPT; k++)
      code[k] = ((uint32_t)tid + (uint32_t)k * (uint32_t)NT) >= n ? 0u
                : AFF ? ((uint32_t)f[k] < nhot ? (kLrHotBit | (uint32_t)f[k]) : row_base + (uint32_t)f[k])
                      : vcode[f[k]];
    uint64_t ra = 0, rb = 0;
    float y = 0.f;
    if ((uint32_t)tid < ch.y) {
      ra = row_off[rf + tid];
      rb = row_off[rf + tid + 1];
      y = label[rf + tid];
    }
    for (uint32_t q = (uint32_t)tid; q < nbk; q += (uint32_t)NT) bc[q] = 0u;
    __syncthreads();  // wh stored (first chunk); the previous chunk's LDS reads done
    float w[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = (uint32_t)tid + (uint32_t)k * (uint32_t)NT;
      w[k] = i >= n ? 0.f : (code[k] & kLrHotBit) ? wh[code[k] & (kLrHotBit - 1)] : rows[(uint64_t)code[k] * 2];
    }
    uint32_t rk[RES ? RPT : 1];  // RES: each non-hot record's rank inside its bucket in this chunk
    if constexpr (RES) {
#pragma unroll
      for (int k = 0; k < RPT; k++) {
        const uint32_t i = (uint32_t)tid + (uint32_t)k * (uint32_t)NT;
        const bool hot = AFF ? (uint32_t)f[k] < nhot : (code[k] & kLrHotBit) != 0;
        rk[k] = (i < n && !hot) ? atomicAdd(&bc[(uint32_t)f[k] >> kLrFxVB], 1u) : 0u;
      }
    }
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = (uint32_t)tid + (uint32_t)k * (uint32_t)NT;
      if (i < n) prod[i] = w[k] * x[k];
    }
    for (uint32_t r = (uint32_t)tid; r < ch.y; r += (uint32_t)NT) {
      const uint64_t a = r < (uint32_t)NT ? ra : row_off[rf + r], b = r < (uint32_t)NT ? rb : row_off[rf + r + 1];
      for (uint64_t c = a; c < b; c++) rl[c - c0] = (uint16_t)r;
    }
    __syncthreads();
    constexpr int RQ = RES ? 2 : 1;  // RES: the chunk's span in each bucket's region (the atomics'
    uint32_t res[RQ], rbq[RQ];       // results wait in registers until the record writes)
    if constexpr (RES) {
      const uint32_t g = cix & ((1u << gbits) - 1u);
#pragma unroll
      for (int j = 0; j < RQ; j++) {
        const uint32_t q = (uint32_t)tid + (uint32_t)(j * NT), qg = (q << gbits) | g;
        const uint32_t c = q < nbk ? bc[q] : 0u;
        rbq[j] = q < nbk ? rbase[qg] : 0u;
        res[j] = c && !(diag & 256u) ? atomicAdd(&fill[(uint64_t)g * nbk + q], c) : 0u;
      }
      for (uint32_t q = (uint32_t)tid + (uint32_t)(RQ * NT); q < nbk; q += (uint32_t)NT) {  // beyond 2 per thread
        const uint32_t c = bc[q], qg = (q << gbits) | g;
        bc[q] = rbase[qg] + (c ? atomicAdd(&fill[(uint64_t)g * nbk + q], c) : 0u);
      }
    }
    for (uint32_t r = (uint32_t)tid; r < ch.y; r += (uint32_t)NT) {  // lr.cpp:358-367, in feature order
      if (r >= (uint32_t)NT) {
        ra = row_off[rf + r];
        rb = row_off[rf + r + 1];
        y = label[rf + r];
      }
      // the products added one by one in feature order (the reference's fp32 `sum += w*x`); their LDS
      // loads go out 8 at a time so the chain waits on the adds, not on one load per feature
      float sum = 0.f;
      uint32_t c = (uint32_t)(ra - c0);
      const uint32_t ce = (uint32_t)(rb - c0);
      for (; c + 8 <= ce; c += 8) {
        float pv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) pv[u] = prod[c + u];
#pragma unroll
        for (int u = 0; u < 8; u++) sum += pv[u];
      }
      for (; c < ce; c++) sum += prod[c];
      const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
      const float error = y - predict;
      err[rf + r] = error;
      err2[rf + r] = error * error;
      es[r] = error;
    }
    __syncthreads();
    // every record's term g = e * x_i (lr.cpp:368): a hot key's into its LDS sum, the others into
    // prod (free since the row sums) with their rank inside their bucket in rl (free after g) —
    // nothing but f (and, without AFF, the codes) stays in registers across the scan below
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = (uint32_t)tid + (uint32_t)k * (uint32_t)NT;
      if (i < n) {
        const float g = es[rl[i]] * x[k];
        const bool hot = AFF ? (uint32_t)f[k] < nhot : (code[k] & kLrHotBit) != 0;
        if (hot) {
          const uint32_t h = AFF ? (uint32_t)f[k] : code[k] & (kLrHotBit - 1);
          if (!(diag & 64u)) {
            atomicAdd(&hs[h], (unsigned long long)__double2ll_rn((double)g * scale));
            atomicAdd(&hc[h], 1u);
          }
        } else {
          prod[i] = g;
          if constexpr (!RES)
            rl[i] = (diag & 128u) ? (uint16_t)0 : (uint16_t)atomicAdd(&bc[(uint32_t)f[k] >> kLrFxVB], 1u);
        }
      }
    }
    if constexpr (RES) {  // each bucket's first slot of this chunk's span
#pragma unroll
      for (int j = 0; j < RQ; j++) {
        const uint32_t q = (uint32_t)tid + (uint32_t)(j * NT);
        if (q < nbk) bc[q] = rbq[j] + res[j];
      }
    }
    __syncthreads();
    if (!RES && tid < 64 && !(diag & 128u)) {  // one wave: exclusive scan of the bucket counts, the chunk's offsets
      const uint32_t per = (nbk + 63u) / 64u, b0 = (uint32_t)tid * per, b1 = min(nbk, b0 + per);
      uint32_t s = 0;
      for (uint32_t q = b0; q < b1; q++) s += bc[q];
      uint32_t inc = s;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (tid >= d) inc += o;
      }
      uint32_t run = inc - s;
      for (uint32_t q = b0; q < b1; q++) {  // boff[bucket][chunk]: a bucket's offsets contiguous
        const uint32_t c = bc[q];
        bc[q] = run;
        boff[(uint64_t)q * bstride + cix] = (uint16_t)run;
        run += c;
      }
      if (tid == 63) boff[(uint64_t)nbk * bstride + cix] = (uint16_t)inc;
    }
    if constexpr (!RES) __syncthreads();
    const uint64_t base = RES ? 0 : c0 - z0;
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = (uint32_t)tid + (uint32_t)k * (uint32_t)NT;
      const bool hot = AFF ? (uint32_t)f[k] < nhot : (code[k] & kLrHotBit) != 0;
      if (i < n && !hot && !(diag & 4u))
        rec[base + bc[(uint32_t)f[k] >> kLrFxVB] + (RES ? rk[k] : (uint32_t)rl[i])] =
            make_uint2((uint32_t)f[k], __float_as_uint(prod[i]));
    }
    __syncthreads();  // bc / es / rl are the next chunk's
  }
  if (nhot && !(diag & 8u)) {
    __syncthreads();
    unsigned long long *hsr = hsum + (uint64_t)blockIdx.x * nhot;
    uint32_t *hcr = hcnt + (uint64_t)blockIdx.x * nhot;
    for (uint32_t q = (uint32_t)tid; q < nhot; q += (uint32_t)NT) {
      hsr[q] = hs[q];
      hcr[q] = hc[q];
    }
  }
}

// k_lr_fxr_step: k_lr_fxb_step's work for the bench's form (rows placed by fid, bucket regions),
// written without per-record branches so every per-record LDS / memory step of a thread goes out
// as one batch.  A record past the chunk's end, and for the bucket count a hot record, is a dummy:
// its LDS updates land in one of 32 spare slots (lane-spread, never read) and its record is not
// written.  Same products, same ordered row sums, same integer terms: bit-identical to
// k_lr_fxb_step (test_lr_fixed_point_step).
constexpr uint32_t kLrFxDummy = 32;
template <int RPT, int NT, int HC>
__global__ __launch_bounds__(NT) void k_lr_fxr_step(const uint2 *__restrict__ chunks, uint32_t nchunks,
                                                     const uint64_t *__restrict__ row_off,
                                                     const int32_t *__restrict__ ffid, const float *__restrict__ fval,
                                                     const float *__restrict__ label, uint64_t r0,
                                                     const float *__restrict__ rows, uint32_t nhot,
                                                     float *__restrict__ err, float *__restrict__ err2, double scale,
                                                     uint32_t nbk, uint2 *__restrict__ rec,
                                                     unsigned long long *__restrict__ hsum,
                                                     uint32_t *__restrict__ hcnt, uint32_t row_base,
                                                     uint32_t *__restrict__ fill, const uint32_t *__restrict__ rbase,
                                                     uint32_t gbits, const float *__restrict__ wmir, uint32_t diag) {
  // wmir (single GPU): the weights as a dense array by fid, kept by k_lr_fxb_push beside the [w | g2]
  // rows — a 128-B line holds 32 of them instead of 16, so the gathers of the non-hot weights touch
  // half the lines (in every XCD's L2 that reads them); null: the rows themselves
  const float *wsrc = wmir ? wmir : rows;
  const uint64_t wst = wmir ? 1 : 2, wb = wmir ? 0 : row_base;
  constexpr int CAP = RPT * NT;
  __shared__ float prod[CAP];
  __shared__ uint16_t rl[CAP];
  __shared__ float es[CAP];
  __shared__ float wh[HC];
  __shared__ unsigned long long hs[HC + kLrFxDummy];
  __shared__ uint32_t hc[HC + kLrFxDummy];
  extern __shared__ uint32_t bc[];  // [nbk + kLrFxDummy]: dynamic
  const uint32_t tid = threadIdx.x, dum = tid & (kLrFxDummy - 1u);
  constexpr int HPT = (HC + NT - 1) / NT;
  float hv[HPT];
#pragma unroll
  for (int j = 0; j < HPT; j++) {
    const uint32_t q = tid + (uint32_t)(NT * j);
    hv[j] = q < nhot ? wsrc[(wb + q) * wst] : 0.f;
  }
  for (uint32_t q = tid; q < (uint32_t)HC + kLrFxDummy; q += (uint32_t)NT) {
    hs[q] = 0ull;
    hc[q] = 0u;
  }
#pragma unroll
  for (int j = 0; j < HPT; j++) {
    const uint32_t q = tid + (uint32_t)(NT * j);
    if (q < (uint32_t)HC) wh[q] = hv[j];
  }
  const uint32_t gmask = (1u << gbits) - 1u;
  for (uint32_t cix = blockIdx.x; cix < nchunks; cix += gridDim.x) {
    const uint2 ch = chunks[cix];
    const uint64_t rf = r0 + ch.x;
    const uint64_t c0 = row_off[rf], c1 = row_off[rf + ch.y];
    const uint32_t n = (uint32_t)(c1 - c0);
    int32_t f[RPT];
    float x[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) {  // past the end: the chunk's last record, x = 0
      const uint32_t i = tid + (uint32_t)k * (uint32_t)NT;
      const uint64_t c = c0 + min(i, n - 1u);
      f[k] = ffid[c];
      x[k] = fval[c];
    }
    uint64_t ra = 0, rb = 0;
    float y = 0.f;
    if (tid < ch.y) {
      ra = row_off[rf + tid];
      rb = row_off[rf + tid + 1];
      y = label[rf + tid];
    }
    for (uint32_t q = tid; q < nbk + kLrFxDummy; q += (uint32_t)NT) bc[q] = 0u;
    __syncthreads();  // bc zeroed, wh stored (first chunk), the previous chunk's LDS reads done
    // the non-hot records' ranks in their buckets (hot records and the dummies: spare slots) and
    // the weights: hot from LDS, the others gathered (a hot / dummy record loads row row_base)
    uint32_t rk[RPT];
    float w[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = tid + (uint32_t)k * (uint32_t)NT;
      const bool cold = i < n && (uint32_t)f[k] >= nhot;
      const uint32_t fk = (uint32_t)f[k];
      rk[k] = atomicAdd(&bc[cold ? (fk >> kLrFxVB) : nbk + dum], 1u);
      const float g = wsrc[(wb + (cold ? fk : 0u)) * wst];
      const float h = wh[fk < nhot ? fk : 0u];
      w[k] = fk < nhot ? h : g;
    }
    __syncthreads();  // the chunk's bucket counts
    // its span in each bucket's region: a returning atomic per bucket, waited for at the record
    // writes (the forward runs meanwhile)
    constexpr int RQ = 2;
    uint32_t res[RQ], rbq[RQ];
    const uint32_t grp = cix & gmask;
#pragma unroll
    for (int j = 0; j < RQ; j++) {
      const uint32_t q = tid + (uint32_t)(j * NT), qg = (q << gbits) | grp;
      const uint32_t c = q < nbk ? bc[q] : 0u;
      rbq[j] = q < nbk ? rbase[qg] : 0u;
      res[j] = c && !(diag & 256u) ? atomicAdd(&fill[(uint64_t)grp * nbk + q], c) : 0u;
    }
    for (uint32_t q = tid + (uint32_t)(RQ * NT); q < nbk; q += (uint32_t)NT) {  // beyond 2 per thread
      const uint32_t c = bc[q], qg = (q << gbits) | grp;
      bc[q] = rbase[qg] + (c ? atomicAdd(&fill[(uint64_t)grp * nbk + q], c) : 0u);
    }
#pragma unroll
    for (int k = 0; k < RPT; k++) prod[tid + (uint32_t)k * (uint32_t)NT] = w[k] * x[k];
    for (uint32_t r = tid; r < ch.y; r += (uint32_t)NT) {
      const uint64_t a = r < (uint32_t)NT ? ra : row_off[rf + r], b = r < (uint32_t)NT ? rb : row_off[rf + r + 1];
      for (uint64_t c = a; c < b; c++) rl[c - c0] = (uint16_t)r;
    }
    __syncthreads();
    for (uint32_t r = tid; r < ch.y; r += (uint32_t)NT) {  // lr.cpp:358-367, in feature order
      if (r >= (uint32_t)NT) {
        ra = row_off[rf + r];
        rb = row_off[rf + r + 1];
        y = label[rf + r];
      }
      float sum = 0.f;
      uint32_t c = (uint32_t)(ra - c0);
      const uint32_t ce = (uint32_t)(rb - c0);
      for (; c + 8 <= ce; c += 8) {
        float pv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) pv[u] = prod[c + u];
#pragma unroll
        for (int u = 0; u < 8; u++) sum += pv[u];
      }
      for (; c < ce; c++) sum += prod[c];
      const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
      const float error = y - predict;
      err[rf + r] = error;
      err2[rf + r] = error * error;
      es[r] = error;
    }
    __syncthreads();
    // every record's term g = e * x_i (lr.cpp:368): a hot key's into its LDS sum, the others into
    // prod (their record); the dummies' (x = 0) and the non-hot records' LDS adds go to spare slots
    uint16_t rr[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) rr[k] = rl[tid + (uint32_t)k * (uint32_t)NT];
    float ev[RPT];
#pragma unroll
    for (int k = 0; k < RPT; k++) ev[k] = es[rr[k] & (CAP - 1)];
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = tid + (uint32_t)k * (uint32_t)NT;
      const float g = ev[k] * x[k];
      const bool hot = i < n && (uint32_t)f[k] < nhot;
      const uint32_t h = hot ? (uint32_t)f[k] : (uint32_t)HC + dum;
      atomicAdd(&hs[h], (unsigned long long)__double2ll_rn((double)g * scale));
      atomicAdd(&hc[h], 1u);
      prod[i] = g;
    }
#pragma unroll
    for (int j = 0; j < RQ; j++) {  // the spans' first slots
      const uint32_t q = tid + (uint32_t)(j * NT);
      if (q < nbk) bc[q] = rbq[j] + res[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RPT; k++) {
      const uint32_t i = tid + (uint32_t)k * (uint32_t)NT;
      if (i < n && (uint32_t)f[k] >= nhot && !(diag & 4u))
        rec[bc[(uint32_t)f[k] >> kLrFxVB] + rk[k]] = make_uint2((uint32_t)f[k], __float_as_uint(prod[i]));
    }
    __syncthreads();  // bc / es / rl are the next chunk's
  }
  if (nhot && !(diag & 8u)) {
    unsigned long long *hsr = hsum + (uint64_t)blockIdx.x * nhot;
    uint32_t *hcr = hcnt + (uint64_t)blockIdx.x * nhot;
    for (uint32_t q = tid; q < nhot; q += (uint32_t)NT) {
      hsr[q] = hs[q];
      hcr[q] = hc[q];
    }
  }
}

__device__ __forceinline__ void lr_fx_adagrad(float *__restrict__ r, long long s, uint32_t c, float lr, float fudge,
                                              double inv_scale) {  // lr.cpp:32-38, 68-75 (k_lr_fx_apply's rule)
  const float w = r[0], g2 = r[1];
  const float m = (float)(((double)s * inv_scale) / (double)c);
  const float ng2 = g2 + m * m;
  const float step = lr * m;
  r[1] = ng2;
  r[0] = w + step / sqrtf(ng2 + fudge);
}

constexpr uint32_t kLrFxbPushT = 1024;  // k_lr_fxb_push's threads: one block per bucket, 16 waves
constexpr uint32_t kLrFxbHotK = 16;     // hot keys per k_lr_fxb_push block (64 row groups each)
// TO_GRADS (the sharded learner, swps_lr_step): no AdaGrad here — each present key's mean goes to
// the push payload, rows[vid_row[fid]] (vid_row = the batch's key positions by fid, rows = the
// payload; hrow[q] = q); the owners apply it (swps_lr_serve_push)
template <bool TO_GRADS, bool RES>
__global__ __launch_bounds__(kLrFxbPushT) void k_lr_fxb_push(const uint2 *__restrict__ rec,
                                                             const uint16_t *__restrict__ boff,
                                                             const uint32_t *__restrict__ chunk_c0, uint32_t nchunks,
                                                             uint32_t nbk, uint32_t bstride,
                                                             const uint32_t *__restrict__ vid_row,
                                                             const unsigned long long *__restrict__ hsum,
                                                             const uint32_t *__restrict__ hcnt, uint32_t hblocks,
                                                             const uint32_t *__restrict__ hrow, uint32_t nhot,
                                                             float *__restrict__ rows, float lr, float fudge,
                                                             double scale, double inv_scale, uint32_t aff,
                                                             uint32_t row_base, uint32_t first_block,
                                                             uint32_t bper, uint32_t *__restrict__ fill,
                                                             const uint32_t *__restrict__ rbase, uint32_t nkeys,
                                                             uint32_t gbits, float *__restrict__ wmir,
                                                             const uint8_t *__restrict__ pfb, uint32_t diag) {
  constexpr uint32_t T = 1u << kLrFxVB, NT = kLrFxbPushT, PER = T / NT;
  __shared__ unsigned long long as[T];
  __shared__ uint32_t ac[T];
  extern __shared__ uint32_t dyn_lds[];  // bucket blocks: 2 * nchunks + 1 words
  const uint32_t tid = threadIdx.x, bid = blockIdx.x + first_block;
  // bper > 0: the bucket blocks dealt XCD-contiguous — blocks are dealt round-robin over the 8 XCDs,
  // so block i (on XCD i % 8) takes bucket (i % 8) * bper + i / 8 and each XCD owns a run of
  // neighbouring buckets: the 128-B lines a chunk's neighbouring bucket segments share are read
  // through one L2 (speed only; any placement gives the same sums)
  const uint32_t nbb = bper ? 8u * bper : nbk;
  if (bid < nbb) {
    const uint32_t b = bper ? (bid & 7u) * bper + (bid >> 3) : bid;
    if (b >= nbk) return;
    if constexpr (RES) {
      // the bucket's records are one contiguous run of rec; its rows one contiguous run of the
      // table (affine form): their loads go out first, beside the count, so the row updates need no
      // further round trip
      constexpr uint32_t GM = 1u << kLrFxMaxGBits;
      __shared__ uint32_t sR[GM], sB[GM];
      const uint32_t G = 1u << gbits;
      if (tid < G) {  // the groups' counts, and the counters' reset for the next step (in order per thread)
        const uint64_t qg = ((uint64_t)b << gbits) | tid;
        const uint32_t r0 = fill[(uint64_t)tid * nbk + b];
        sR[tid] = (diag & 32u) ? 0u : r0;
        sB[tid] = rbase[qg];
        fill[(uint64_t)tid * nbk + b] = 0u;
      }
      // the rows' loads beside the count only for the buckets whose keys most batches touch (pfb,
      // from the corpus counts at load): elsewhere the untouched rows' bytes would outweigh the
      // round trip they save
      const bool aff_rows = !TO_GRADS && aff, pre = aff_rows && (!pfb || pfb[b]);
      float2 wg[PER];
#pragma unroll
      for (uint32_t k = 0; k < PER; k++) {
        const uint32_t v = (b << kLrFxVB) + tid + k * NT;
        wg[k] = pre && v < nkeys ? *reinterpret_cast<const float2 *>(rows + (uint64_t)(row_base + v) * 2)
                                 : make_float2(0.f, 0.f);
      }
      for (uint32_t v = tid; v < T; v += NT) {
        as[v] = 0ull;
        ac[v] = 0u;
      }
      __syncthreads();
      uint32_t gp[GM + 1], gb[GM];  // the groups' runs as one list: prefix of their counts
      gp[0] = 0;
#pragma unroll
      for (uint32_t g = 0; g < GM; g++) {
        gp[g + 1] = gp[g] + (g < G ? sR[g] : 0u);
        gb[g] = g < G ? sB[g] : 0u;
      }
      const uint32_t R = gp[GM];
      for (uint32_t j0 = tid; j0 < R; j0 += 4 * NT) {
        uint2 r[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t j = j0 + (uint32_t)k * NT;
          if (j < R) {
            uint32_t a = gb[0] + j;
#pragma unroll
            for (uint32_t g = 1; g < GM; g++)
              if (j >= gp[g]) a = gb[g] + (j - gp[g]);
            r[k] = rec[a];
          }
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (j0 + (uint32_t)k * NT < R) {
            atomicAdd(&as[r[k].x & (T - 1)], (unsigned long long)__double2ll_rn((double)__uint_as_float(r[k].y) * scale));
            atomicAdd(&ac[r[k].x & (T - 1)], 1u);
          }
      }
      __syncthreads();
      if (diag & 16u) return;
      if (TO_GRADS) {
#pragma unroll
        for (uint32_t k = 0; k < PER; k++) {
          const uint32_t v = tid + k * NT, c = ac[v];
          if (c) rows[vid_row[(b << kLrFxVB) + v]] = (float)(((double)(long long)as[v] * inv_scale) / (double)c);
        }
        return;
      }
      uint32_t c[PER], row[PER];
#pragma unroll
      for (uint32_t k = 0; k < PER; k++) {
        c[k] = ac[tid + k * NT];
        if (c[k] && !pre) {
          row[k] = aff_rows ? row_base + (b << kLrFxVB) + tid + k * NT : vid_row[(b << kLrFxVB) + tid + k * NT];
          if (row[k] == kNoRow) c[k] = 0u;  // world 1 in place: a key the shard lacks
        }
      }
      if (!pre) {
#pragma unroll
        for (uint32_t k = 0; k < PER; k++)
          if (c[k]) wg[k] = *reinterpret_cast<const float2 *>(rows + (uint64_t)row[k] * 2);
      }
#pragma unroll
      for (uint32_t k = 0; k < PER; k++)
        if (c[k]) {  // lr.cpp:32-38, 68-75 (k_lr_fx_apply's rule)
          const float m = (float)(((double)(long long)as[tid + k * NT] * inv_scale) / (double)c[k]);
          const float ng2 = wg[k].y + m * m;
          const float step = lr * m;
          const uint64_t rr = pre ? (uint64_t)row_base + (b << kLrFxVB) + tid + k * NT : row[k];
          const float nw = wg[k].x + step / sqrtf(ng2 + fudge);
          *reinterpret_cast<float2 *>(rows + rr * 2) = make_float2(nw, ng2);
          if (wmir) wmir[(b << kLrFxVB) + tid + k * NT] = nw;  // the step's dense copy (fid order)
        }
      return;
    }
    for (uint32_t v = tid; v < T; v += NT) {
      as[v] = 0ull;
      ac[v] = 0u;
    }
    __syncthreads();
    // the bucket's records as one list over the chunks' segments (prefix in LDS): a lane takes the
    // j-th record of the list, so one wave's lanes read neighbouring records of a few chunks —
    // different keys, few LDS conflicts — and every lane has about the same number
    uint32_t *segoff = dyn_lds;                 // [nchunks + 1]
    uint32_t *segbase = dyn_lds + nchunks + 1;  // [nchunks]: the segment's first record in rec
    __shared__ uint32_t wsum[NT / 64];
    const uint32_t per = (nchunks + NT - 1) / NT, s0 = tid * per, s1 = min(nchunks, s0 + per);
    uint32_t tot = 0;
    for (uint32_t sq = s0; sq < s1; sq++) {
      const uint32_t lo = boff[(uint64_t)b * bstride + sq], hi = boff[(uint64_t)(b + 1) * bstride + sq];
      segbase[sq] = chunk_c0[sq] + lo;
      segoff[sq] = hi - lo;  // length for now
      tot += hi - lo;
    }
    uint32_t inc = tot;  // block-wide exclusive scan of the threads' totals
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = __shfl_up(inc, d, 64);
      if ((tid & 63u) >= (uint32_t)d) inc += o;
    }
    if ((tid & 63u) == 63u) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t wbase = 0;
    for (uint32_t w = 0; w < (tid >> 6); w++) wbase += wsum[w];
    uint32_t run = wbase + inc - tot;
    for (uint32_t sq = s0; sq < s1; sq++) {
      const uint32_t len = segoff[sq];
      segoff[sq] = run;
      run += len;
    }
    if (tid == NT - 1) segoff[nchunks] = run;
    __syncthreads();
    const uint32_t R = (diag & 32u) ? 0u : segoff[nchunks];
    for (uint32_t j0 = tid; j0 < R; j0 += 4 * NT) {
      uint2 r[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t j = j0 + (uint32_t)k * NT;
        if (j < R) {
          uint32_t lo = 0, hi = nchunks;  // the last segment starting at or before j
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (segoff[mid] <= j)
              lo = mid;
            else
              hi = mid;
          }
          r[k] = rec[segbase[lo] + (j - segoff[lo])];
        }
      }
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (j0 + (uint32_t)k * NT < R) {
          atomicAdd(&as[r[k].x & (T - 1)], (unsigned long long)__double2ll_rn((double)__uint_as_float(r[k].y) * scale));
          atomicAdd(&ac[r[k].x & (T - 1)], 1u);
        }
    }
    __syncthreads();
    if (diag & 16u) return;
    if (TO_GRADS) {  // the bucket's key (records carry fids: the affine form with row base 0)
#pragma unroll
      for (uint32_t k = 0; k < PER; k++) {
        const uint32_t v = tid + k * NT, c = ac[v];
        if (c) rows[vid_row[(b << kLrFxVB) + v]] = (float)(((double)(long long)as[v] * inv_scale) / (double)c);
      }
      return;
    }
    uint32_t c[PER], row[PER];  // the thread's PER vids: row loads, then [w | g2] loads, all in flight
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) {
      c[k] = ac[tid + k * NT];
      if (c[k]) {
        row[k] = aff ? row_base + (b << kLrFxVB) + tid + k * NT : vid_row[(b << kLrFxVB) + tid + k * NT];
        if (row[k] == kNoRow) c[k] = 0u;  // world 1 in place: a key the shard lacks
      }
    }
    float2 wg[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++)
      if (c[k]) wg[k] = *reinterpret_cast<const float2 *>(rows + (uint64_t)row[k] * 2);
#pragma unroll
    for (uint32_t k = 0; k < PER; k++)
      if (c[k]) {  // lr.cpp:32-38, 68-75 (k_lr_fx_apply's rule)
        const float m = (float)(((double)(long long)as[tid + k * NT] * inv_scale) / (double)c[k]);
        const float ng2 = wg[k].y + m * m;
        const float step = lr * m;
        *reinterpret_cast<float2 *>(rows + (uint64_t)row[k] * 2) = make_float2(wg[k].x + step / sqrtf(ng2 + fudge), ng2);
      }
    return;
  }
  // kLrFxbHotK hot keys per block: the other threads' row groups sum each key's column of the step's
  // block partials, then the groups' sums are added in LDS
  constexpr uint32_t KPB = kLrFxbHotK, RG = NT / KPB;
  const uint32_t h0 = (bid - nbb) * KPB, kk = tid % KPB, rg = tid / KPB;
  const uint32_t h = h0 + kk;
  unsigned long long s = 0ull;
  uint32_t c = 0u;
  if (h < nhot) {  // up to 16 partial rows per thread in flight at once (768 step blocks / 64 groups = 12)
    for (uint32_t b0 = rg; b0 < hblocks; b0 += 16 * RG) {
      unsigned long long ps[16];
      uint32_t pc[16];
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const uint32_t blk = b0 + (uint32_t)u * RG;
        ps[u] = blk < hblocks ? hsum[(uint64_t)blk * nhot + h] : 0ull;
        pc[u] = blk < hblocks ? hcnt[(uint64_t)blk * nhot + h] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 16; u++) {
        s += ps[u];
        c += pc[u];
      }
    }
  }
  as[tid] = s;
  ac[tid] = c;
  __syncthreads();
  for (uint32_t w = RG / 2; w >= 1; w >>= 1) {  // tree over the row groups
    if (rg < w) {
      as[tid] += as[tid + w * KPB];
      ac[tid] += ac[tid + w * KPB];
    }
    __syncthreads();
  }
  if (rg == 0 && h < nhot && ac[tid]) {
    if (TO_GRADS)
      rows[vid_row[hrow[h]]] = (float)(((double)(long long)as[tid] * inv_scale) / (double)ac[tid]);
    else if (hrow[h] != kNoRow) {
      lr_fx_adagrad(rows + (uint64_t)hrow[h] * 2, (long long)as[tid], ac[tid], lr, fudge, inv_scale);
      if (wmir) wmir[h] = rows[(uint64_t)hrow[h] * 2];  // hot key q = fid q (affine form)
    }
  }
}

// the step's dense weight copy: wmir[fid] = the w of shard row row_base + fid
__global__ void k_lr_mirror(const float *__restrict__ rows, uint32_t row_base, uint64_t V, float *__restrict__ wmir) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < V) wmir[q] = rows[((uint64_t)row_base + q) * 2];
}

// every record's fid (the fixed-point step's key numbering)
__global__ void k_lr_fx_fid(const int32_t *__restrict__ fvid, uint64_t n, const uint32_t *__restrict__ fid,
                            int32_t *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)fid[fvid[i]];
}
// the per-key codes of the fixed-point step: hot rank | kLrHotBit, else the key's shard row
__global__ void k_lr_fx_codes(const uint32_t *__restrict__ vid_row, uint64_t V, const int32_t *__restrict__ hot_of_vid,
                              uint32_t *__restrict__ vcode) {
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  const int32_t h = hot_of_vid ? hot_of_vid[v] : -1;
  vcode[v] = h >= 0 ? (kLrHotBit | (uint32_t)h) : vid_row ? vid_row[v] : (uint32_t)v;  // null: the vid
}
__global__ void k_lr_fx_hrow(const uint32_t *__restrict__ hot_vid, uint32_t nhot, const uint32_t *__restrict__ vid_row,
                             uint32_t *__restrict__ hrow) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < nhot) hrow[q] = vid_row ? vid_row[hot_vid[q]] : hot_vid[q];
}

// ---- the corpus vocabulary on the GPU (lr_ingest): vid = rank of the key among the distinct keys
__global__ void k_lr_voc_heads(const uint32_t *__restrict__ ks, uint64_t n, uint32_t *__restrict__ head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) head[i] = (i == 0 || ks[i] != ks[i - 1]) ? 1u : 0u;
}
// every record's vid; per distinct key its key, its first record (the stable sort keeps CSR order)
// and its first position in key order (the next key's minus its own = its record count)
__global__ void k_lr_voc_ids(const uint32_t *__restrict__ ks, const uint32_t *__restrict__ perm,
                             const uint32_t *__restrict__ rank, uint64_t n, int32_t *__restrict__ fvid,
                             uint32_t *__restrict__ ukey, uint32_t *__restrict__ ufirst, uint32_t *__restrict__ ustart) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = rank[i] - 1;
  fvid[perm[i]] = (int32_t)r;
  if (i == 0 || ks[i] != ks[i - 1]) {
    ukey[r] = ks[i];
    ufirst[r] = perm[i];
    ustart[r] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256) void k_lr_predict(const uint64_t *__restrict__ row_off, const int32_t *__restrict__ fvid,
                             const float *__restrict__ fval, uint64_t nr, const uint32_t *__restrict__ vid_row,
                             const float *__restrict__ rows, float *__restrict__ pred) {
  const uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= nr) return;
  const uint64_t a = row_off[r], b = row_off[r + 1];
  float sum = 0;
  for (uint64_t c = a; c < b; c += 64) {
    const int m = (int)min<uint64_t>(64, b - c);
    float prod = 0.f;
    if (lane < m) prod = weight(vid_row, rows, fvid[c + lane]) * fval[c + lane];
    sum = ordered_add(sum, prod, m);
  }
  if (lane == 0) pred[r] = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
}

// pulled weights [U] (request order K) into the worker cache; local[vid] = u
__global__ void k_lr_install(const int32_t *__restrict__ K, uint64_t U, const float *__restrict__ vals,
                             float *__restrict__ wcache, int32_t *__restrict__ local, int stride) {
  uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  wcache[(uint64_t)K[u] * stride] = vals[u];
  if (local) local[K[u]] = (int32_t)u;
}

// the sharded fixed-point step's install: the value of key K[u] at its fid's row of the step's layout
// (wcache2[2 * fid]: the affine form with row base 0, hot keys first), and its position u by fid
// (stride 1: the dense copy the branch-free step gathers from)
__global__ void k_lr_install_fx(const int32_t *__restrict__ K, uint64_t U, const float *__restrict__ vals,
                                const uint32_t *__restrict__ fid, float *__restrict__ wcache2, uint32_t stride,
                                uint32_t *__restrict__ localf) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const uint32_t q = fid[K[u]];
  wcache2[(uint64_t)q * stride] = vals[u];
  if (localf) localf[q] = (uint32_t)u;
}
// world 1 in place: the weight of key K[u] read from its shard row prow[u] (the slot's lookup), and
// that row by fid — the push applies AdaGrad there (an absent key: weight 0, row kNoRow, skipped)
__global__ void k_lr_install_fx_rows(const int32_t *__restrict__ K, uint64_t U, const uint32_t *__restrict__ prow,
                                     const float *__restrict__ rows, const uint32_t *__restrict__ fid,
                                     float *__restrict__ wcache2, uint32_t stride, uint32_t *__restrict__ localf) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= U) return;
  const uint32_t q = fid[K[u]], r = prow[u];
  wcache2[(uint64_t)q * stride] = r == kNoRow ? 0.f : rows[(uint64_t)r * 2];
  localf[q] = r;
}

__global__ void k_lr_keys(const int32_t *__restrict__ K, uint64_t n, const uint64_t *__restrict__ vkeys,
                          uint64_t *__restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = vkeys[K[i]];
}

inline unsigned nblk(uint64_t n, unsigned bs = 256) { return (unsigned)std::max<uint64_t>(1, (n + bs - 1) / bs); }

struct LTimer {
  bool on = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;  // k >= 16: timer k - 16, not counted
  double ms[4] = {0};
  uint64_t cnt[4] = {0};
  hipEvent_t begin(hipStream_t s) {
    if (!on) return nullptr;
    hipEvent_t e;
    (void)hipEventCreate(&e);
    (void)hipEventRecord(e, s);
    return e;
  }
  void end(int k, hipEvent_t b, hipStream_t s) {
    if (!b) return;
    hipEvent_t e;
    (void)hipEventCreate(&e);
    (void)hipEventRecord(e, s);
    pending.push_back({k, {b, e}});
  }
  // events for hipExtLaunchKernelGGL: stamped by the GPU at the kernel's own start / end, so a
  // short kernel's time does not include the stream's gaps around it (as rocprof measures it)
  hipEvent_t ext() {
    if (!on) return nullptr;
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  void ext_end(int k, hipEvent_t b, hipEvent_t e) {
    if (b && e) pending.push_back({k, {b, e}});
  }
  // a further kernel of the same launch group: its own stamped time added, the launch not counted
  // again (a group's kernels summed, as rocprof sums them, without the gaps between them)
  void ext_more(int k, hipEvent_t b, hipEvent_t e) {
    if (b && e) pending.push_back({k + 16, {b, e}});
  }
  void resolve() {
    for (auto &q : pending) {
      float t = 0;
      (void)hipEventElapsedTime(&t, q.second.first, q.second.second);
      ms[q.first & 15] += t;
      if (q.first < 16) cnt[q.first]++;
      (void)hipEventDestroy(q.second.first);
      (void)hipEventDestroy(q.second.second);
    }
    pending.clear();
  }
};

}  // namespace

struct swps_lr {
  swps_table *t = nullptr;
  swps_lr_cfg cfg{};
  hipStream_t s = nullptr;
  std::vector<float> label;
  std::vector<uint64_t> row_off;
  std::vector<int32_t> fvid;
  std::vector<float> fval;
  std::vector<uint64_t> vocab_keys;  // vid order = key order (lr_vocab)
  std::vector<uint32_t> vocab_cnt;   // records per key in the corpus
  std::vector<uint32_t> pull_order;  // init_ref: the vids in the first pull's order (lr.cpp:161-166)
  // the table layout of the single-GPU init: vid -> rank of its new row (SWPS_LR_PLACE=1: by
  // (batch, row tile, key) of first appearance, 2: by (batch, key); 0, the default: the insert's own
  // order).  Same-box A/B at the Criteo step, round 4: the forward's L2-miss reads fell 47.3 ->
  // 38.5 MB (13.7 -> 13.3 us) but the row tiles' rose 27.8 -> 30.4 MB and the finisher's 8.3 ->
  // 9.6 MB (push 24.7 -> 25.7 us): 1.645e9 -> 1.63e9 examples/s, so off
  std::vector<uint32_t> vid_place;
  int place = 0;
  // SWPS_LR_XCD=1: the row tiles' blocks by key octile per XCD (lr_xcd_order); off by default — the
  // natural order already deals block j of every tile to XCD j % 8 at the Criteo batch (104 blocks
  // per tile), and the octile order measured 24.7 -> 25.3 us (A/B, round 4)
  int xcd = 0;
  bool loaded = false, inited = false;
  uint64_t cursor = 0, nbatches = 0;
  DevMem d_label, d_row_off, d_fvid, d_fval, d_vid_row, d_err, d_err2, d_val_s, d_tmp, d_pred, d_longs;
  DevMem d_frow, d_urow;  // single GPU: shard row per record's feature / per run (built at the first batch)
  bool rows_mapped = false;
  // the static per-batch index (lr_index): every batch's records in key-sorted order (row, x_i); the runs
  // (pushed keys) of all batches: vid, start and length relative to the batch; first run and run count per batch
  DevMem d_srow, d_sval, d_spos, d_ruk, d_roff, d_rcnt, d_bnruns;
  std::vector<uint64_t> brun;
  std::vector<uint64_t> blong;  // [nb+1] offsets of each batch's long runs in d_slong (k_lr_reduce_fused)
  DevMem d_slong;
  int fused_reduce = 1;         // fast sums: k_lr_reduce_fused (SWPS_LR_FUSED=0: memset + short + long; A/B)
  std::vector<uint32_t> bmaxf;  // longest row (features) per batch: k_lr_forward_r's row packing
  int rows_per_wave = 1;        // SWPS_LR_PACK: 1 = 3 or 2 rows per wave by length, ordered sums through LDS
                                // (the default; longer rows: one per wave); 3 = the same with readlane chains;
                                // 2 = at most 2 (readlane); 4 = a lane per row (k_lr_forward_l); 0 = a row per wave
  int inline_records = 0;       // SWPS_LR_INLINE=1: fast sums form the records inside the reduce (A/B)
  int fwd_records = 0;          // SWPS_LR_FWD_RECORDS=1: the forward scatters the records (A/B: 66.6 vs 53.4 us per step, off)
  // fast sums through row tiles (k_lr_tiles): SWPS_LR_TILES=0 for the record path (A/B, tests);
  // SWPS_LR_TILE_BITS shrinks the tiles (tests: many pieces per key)
  int tiles = 1, tile_bits = kTileMaxBits;
  uint32_t tile_chunk = kTileChunk, tile_threads = 256;
  bool tiles_ready = false;
  DevMem d_trow, d_tval, d_tinfo, d_tslot, d_tgrun, d_tdst, d_tchunk, d_tnp, d_tpst, d_tmulti, d_tmlong, d_tpart;
  DevMem d_tmsrow, d_tmlrow;
  uint64_t tile_npieces = 0;
  // [nb+1] offsets of each batch's blocks (4 u32 each) / runs with several pieces / those with many
  std::vector<uint64_t> bchunk, bmulti, bmlong;  // (blocks: tile, first / end record, first / end piece)
  uint64_t max_bpiece = 0;
  int stage = 0;                // SWPS_LR_STAGE: the forward reads the batch's weights staged densely (k_lr_stage)
  DevMem d_frun, d_wstage;
  int hot = 1;  // SWPS_LR_HOT: the forward reads the batch's hot keys' weights from LDS (k_lr_forward_g)
  // SWPS_LR_NHOT: how many (<= kLrHot).  Same-box A/B at the Criteo step, round 4 (forward µs):
  // 256 13.84, 512 13.53, 768 14.0-14.3, 1024 15.6 — each block loads them all
  uint32_t nhot = 512;
  DevMem d_hot_of_run, d_hgrun, d_hrow, d_fhot;
  std::vector<uint32_t> bnhot;
  uint64_t max_bruns = 0;
  int fwd_groups = 2;            // SWPS_LR_FWD_G: row groups per wave in the forward (1, 2, 4; A/B: 2)
  int fwd_c = 1;                 // SWPS_LR_FWD_C: the record-contiguous forward (k_lr_forward_c; 0 = off)
  int fwd_rpt = 8;               // its records per thread (SWPS_LR_FWD_C = 4 / 16 for A/B; 1 = the default 8)
  DevMem d_fchunk;               // its static chunks of whole rows (uint2 {first row in batch, rows})
  std::vector<uint64_t> bfchunk;  // [nb+1] each batch's first chunk
  int fwd_diag = 0;             // SWPS_LR_DIAG: timing experiments (1: forward without weight gather, 2: without ordered chain, 4: records without e gathers)
  uint64_t max_bnnz = 0;
  uint32_t *h_small = nullptr;
  LTimer timer;
  // sharded mode (swps_lr_shard): per-batch key sets ordered by owner rank
  bool sharded = false;
  int32_t rank = 0, world = 1;
  std::vector<int32_t> allK, init_order;  // vids
  std::vector<uint64_t> kofs, bU, bcounts, icounts;
  DevMem d_K, d_vkeys, d_init_order, d_wcache, d_local, d_serve_rows;
  // the sharded learner runs the fixed-point step (plan none, fast sums): the pulled weights at
  // stride 2 (wcache2[2 * vid], the step's row layout) and the mean gradients from its push
  bool fx_sharded = false;
  DevMem d_wcache2, d_fx_fidv, d_localf;  // [2V] weights by fid; fid by vid; batch position by fid
  DevMem d_wdense;  // [V] the same weights dense by fid (the branch-free step's gathers: 32 per line)
  swps::ShardDriver *drv = nullptr;  // swps_lr_shard_comm: the library drives the exchange
  uint64_t serve_n = 0;
  // world 1 in place (AppOps::pull_in_place): serve_pull only looks the slot's rows up, the step's
  // install reads the weights from those shard rows and its push applies AdaGrad to them — the
  // owner's copy, the payload and the owner's apply are gone; serve_push then has nothing to do
  const uint32_t *pull_rows = nullptr;
  bool pushed_in_place = false;
  // world 1, rows placed by fid (the full pull inserts them in fid order): shard row = w1_base + fid,
  // so the in-place step is the single-GPU affine step (dense weight copy kept by the push, no
  // install); -1: not affine (the install reads the rows the slot's lookup names)
  int64_t w1_base = -1;
  DevMem d_w1_hrow;  // the hot keys' shard rows (w1_base + q)
  // the library driver's step slot (AppOps::set_slot): the keys an owner serves at a slot are the
  // same every epoch, so their row lookups and the push's grouping sort are kept per slot
  int64_t slot = -1;
  struct SlotRows {
    DevMem rows, sorted;
    uint64_t n = 0;
    bool sorted_valid = false;
  };
  std::vector<std::unique_ptr<SlotRows>> slot_rows;
  // the static per-batch index (lr_index) exists; the per-step plan builds none at load
  bool index_built = false;
  // per-step plan (cfg.plan == SWPS_LR_PLAN_STEP; single GPU, fast sums through row tiles): the
  // plan stream, its scratch, and two slots of what a step reads (plan(i+1) fills one while step i
  // reads the other)
  bool plan_step = false, plan_ready = false;
  hipStream_t ps = nullptr;
  struct PlanSlot {
    swps::DevMem fcode, hrow, trow, tval, chunk, tinfo, tdst, ms, msrow, ml, mlrow, cnt;
    uint64_t nch = 0;
    hipEvent_t ready = nullptr, used = nullptr;
    bool pending_use = false;
  };
  PlanSlot pslot[2];
  swps::DevMem p_ks1, p_permK, p_tkey, p_tks, p_val2, p_v2s, p_rowK, p_ph, p_pidT, p_invT, p_packed, p_pk, p_kstart,
      p_kwhole, p_krow, p_khot, p_hist, p_thr, p_tfirst, p_tmp;
  swps::DevMem d_rid;  // the row of every record (per-step plan)
  // the fixed-point step (cfg.plan == SWPS_LR_PLAN_NONE): per-key codes, hot keys, accumulators
  bool fx_ready = false;
  int fx_bits = 40;                      // fixed-point scale 2^fx_bits (load: no sum can reach 2^62)
  int fx_floor = 0;                      // the least fx_bits the fixed point runs at (lr_ingest)
  bool fx_fallback = false;              // the fixed point was asked for, fx_bits fell below the floor
  int32_t plan_req = 0;                  // the caller's plan (cfg.plan is the one running)
  std::vector<uint32_t> fx_hot_vids;     // the corpus's most frequent keys (load)
  swps::DevMem d_vcode, d_fx_hot, d_fx_hrow, d_acc_sum, d_acc_cnt, d_fx_list, d_fx_n, d_fx_stamp;
  // the bucketed form (k_lr_fxb_step / k_lr_fxb_push; SWPS_LR_FX_ATOMIC=1 runs the atomic one)
  swps::DevMem d_fchunk_c0;              // each chunk's first record, relative to its batch's first
  swps::DevMem d_fxb_rec, d_fxb_boff, d_fxb_hsum, d_fxb_hcnt;
  swps::DevMem d_fxb_fill, d_fxb_rbase;  // the bucket regions (fxb_res): fill counters, region starts
  bool fxb_res = true;                   // SWPS_LR_FXB_RES=0: the per-chunk bucket segments (round 5)
  bool fxr = true;                       // k_lr_fxr_step (SWPS_LR_FXR=0: k_lr_fxb_step<..., RES>)
  // the step's dense weight copy by fid (single GPU, k_lr_fxr_step + RES): refreshed from the rows at
  // the start of every swps_lr_train_batches call (anything else that writes the table — pulls, pushes,
  // loads — runs between calls), then kept by the push
  swps::DevMem d_wmir, d_pfb;             // weights by fid; per bucket: prefetch its rows in the push
  bool fx_mirror = true, mirror_stale = true;
  // SWPS_LR_FX_PF: 0 no bucket prefetches, 1 dense buckets, 2 all (default: the same PMC traffic, and
  // same box, 2 reps: --app lr 35.5 -> 35.2 us, the line's 10-batch leg 30.8 -> 30.7 us)
  int fx_pf = 2;
  uint32_t fxb_gbits = 0;                // chunk groups per bucket region: 2^fxb_gbits
  uint64_t fxb_region_recs = 0;          // the regions' total capacity (records)
  int fx_atomic = 0;
  uint32_t fxb_grid = 768, fxb_nbk = 0, fxb_diag = 0;
  bool fxb_xcd = true;  // k_lr_fxb_push's bucket blocks XCD-contiguous (SWPS_LR_FXB_XCD=0: in order)
  int fx_nt = 256;  // the fixed-point step's threads per block at 4,096-record chunks (SWPS_LR_FX_NT)
  // fid: the fixed-point step's key numbering — hot keys first (rank), then the rest in row-placement
  // order; swps_lr_init places the rows in fid order, so a key's shard row is fx_row_base + fid
  // (fx_affine, checked after the init) and the step needs no per-key code gather
  std::vector<uint32_t> fx_fid;
  swps::DevMem d_ffid;  // every record's fid
  bool fx_affine = false;
  uint32_t fx_row_base = 0;
  uint64_t max_bchunks = 0;
  uint32_t fx_tag = 0;  // the step's tag in d_fx_stamp (never 0: the stamps start at 0)
  int plan_sort = 1;   // SWPS_LR_PLAN_SORT: tile shape of the plan's radix sorts (sort_pairs_tiled)
  uint64_t plan_next = 0;  // the first step whose plan is not enqueued yet
  int plan_vbits = 1;
  bool plan_sync = true;  // the next plan waits for the compute stream (shard rows just (re)initialised)
  hipEvent_t ev_rows = nullptr;
  int B1() const { return cfg.minibatch + 1; }
};

namespace {

// lr.cpp:161-166: the first gather collects every feature of every valid row
// into `_local_keys` (std::unordered_set<unsigned>); the first pull visits it
// in iteration order, initialising each miss with global_random().gen_float().
template <typename T> int lr_scan_incl(const T *in, T *out, uint64_t n, DevMem &tmp, hipStream_t s) {
  size_t b = 0;
  SWPS_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, b, in, out, (int)n, s));
  SWPS_TRY(tmp.ensure(b));
  b = tmp.bytes;
  SWPS_HIP(hipcub::DeviceScan::InclusiveSum(tmp.p, b, in, out, (int)n, s));
  return SWPS_OK;
}

// XCD-aware block order for the row tiles: the dispatcher deals blocks round-robin over the 8
// XCDs (blocks b and b + 8 share one; MI355X_MICROARCH.md), and a tile's blocks walk its records
// in key order, so the j-th of a tile's n blocks covers about the j/n-th stretch of the key space
// in every tile.  Blocks [q0, q1) of a block table (E u32 each) are reordered so that block slot i
// takes a block of key octile i % 8 (octile = j * 8 / n within its tile) while such blocks remain:
// one XCD then holds the pieces of one stretch of keys from every tile — their partial slots
// (in key order) and their rows (in first-appearance order by key, lr_ingest) stay within one L2
// instead of being split between eight.  Speed only: every block's work is independent of its slot.
template <typename T>
void lr_xcd_order(std::vector<T> &v, int E, uint64_t q0, uint64_t q1, const std::vector<uint32_t> &oct) {
  constexpr int kXcd = 8;
  std::vector<std::vector<uint64_t>> qs(kXcd);
  for (uint64_t q = q0; q < q1; q++) qs[oct[q - q0] % kXcd].push_back(q);
  std::vector<size_t> at(kXcd, 0);
  std::vector<T> out;
  out.reserve((q1 - q0) * E);
  for (uint64_t i = 0; i < q1 - q0; i++) {
    int x = (int)(i % kXcd);
    if (at[x] == qs[x].size()) {  // that octile's blocks are done: the queue with the most left
      for (int y = 0; y < kXcd; y++)
        if (qs[y].size() - at[y] > qs[x].size() - at[x]) x = y;
    }
    const uint64_t q = qs[x][at[x]++];
    out.insert(out.end(), v.begin() + q * E, v.begin() + (q + 1) * E);
  }
  std::copy(out.begin(), out.end(), v.begin() + q0 * E);
}

// The tile index (k_lr_tiles): every batch's records in (tile, key) order; the blocks (kTileChunk
// consecutive records of one tile); the pieces (a key's records inside one block) with their
// run, their partial's slot in (key, record) order, and per run its piece count and first slot;
// per batch the runs with more than one piece.  ks / perm / rid / tmp are lr_index's scratch.
int lr_tile_index(swps_lr *l, DevMem &ks, DevMem &perm, DevMem &rid, DevMem &rkey, DevMem &d_brun, uint64_t R, int bbits,
                  DevMem &tmp) {
  hipStream_t s = l->s;
  const uint64_t nr = l->label.size(), nb = l->nbatches, B1 = (uint64_t)l->B1();
  const uint64_t n = l->row_off[nr];
  const int tb = l->tile_bits;
  const uint64_t ntile = (B1 + (1ULL << tb) - 1) >> tb;
  int tbits = 1;
  while ((1ULL << tbits) < ntile) tbits++;
  if (32 + tbits + bbits > 64) return SWPS_OK;  // the record path
  // blocks, from the CSR: batch b's tile t holds the records of rows [b*B1 + t*2^tb, ...), and
  // the (batch, tile, key) order keeps each (batch, tile) group contiguous
  std::vector<uint32_t> cut, chunks;
  l->bchunk.assign(nb + 1, 0);
  for (uint64_t b = 0; b < nb; b++) {
    l->bchunk[b] = cut.size();
    const uint64_t rb0 = b * B1, rb1 = std::min<uint64_t>(nr, rb0 + B1);
    for (uint64_t tl = 0; rb0 + (tl << tb) < rb1; tl++) {
      const uint64_t rs = rb0 + (tl << tb), re = std::min<uint64_t>(rb1, rs + (1ULL << tb));
      for (uint64_t c0 = l->row_off[rs]; c0 < l->row_off[re]; c0 += l->tile_chunk) {
        const uint64_t c1 = std::min<uint64_t>(l->row_off[re], c0 + l->tile_chunk);
        // record positions in sorted order equal CSR positions at group granularity
        cut.push_back((uint32_t)c0);
        chunks.insert(chunks.end(), {(uint32_t)tl, (uint32_t)c0, (uint32_t)c1, 0u, 0u});
      }
    }
  }
  l->bchunk[nb] = cut.size();
  DevMem key, idx, head, pidr, d_cut, d_p0;
  SWPS_TRY(key.ensure(n * 8));
  SWPS_TRY(idx.ensure(n * 4));
  k_lr_tile_keys<<<nblk(nr), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), nr, B1, tb, tbits, l->d_fvid.as<int32_t>(),
                                           key.as<uint64_t>(), idx.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  size_t sb = 0;
  SWPS_HIP(sort_pairs(nullptr, sb, key.as<uint64_t>(), ks.as<uint64_t>(), idx.as<uint32_t>(), perm.as<uint32_t>(), n,
                      32 + tbits + bbits, s));
  SWPS_TRY(tmp.ensure(sb));
  sb = tmp.bytes;
  SWPS_HIP(sort_pairs(tmp.p, sb, key.as<uint64_t>(), ks.as<uint64_t>(), idx.as<uint32_t>(), perm.as<uint32_t>(), n,
                      32 + tbits + bbits, s));
  key.release();
  idx.release();
  k_lr_rowid<<<nblk(nr), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), nr, rid.as<uint32_t>());
  SWPS_TRY(l->d_trow.ensure(n * 2));
  SWPS_TRY(l->d_tval.ensure(n * 4));
  SWPS_TRY(head.ensure(n * 4));
  SWPS_TRY(pidr.ensure(n * 4));
  k_lr_tile_slots<<<nblk(n), 256, 0, s>>>(ks.as<uint64_t>(), perm.as<uint32_t>(), n, rid.as<uint32_t>(), B1, tb,
                                           l->d_fval.as<float>(), l->d_trow.as<uint16_t>(), l->d_tval.as<float>(),
                                           head.as<uint32_t>());
  SWPS_TRY(upload(d_cut, cut, s));
  k_lr_tile_cuts<<<nblk(cut.size()), 256, 0, s>>>(d_cut.as<uint32_t>(), cut.size(), head.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  SWPS_TRY(lr_scan_incl(head.as<uint32_t>(), pidr.as<uint32_t>(), n, tmp, s));
  uint32_t S2 = 0;
  SWPS_HIP(hipMemcpyAsync(&S2, pidr.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  DevMem tkey2, k2s, pid, perm2, head2, gid, pfirst, d_bsub, d_bcnt;
  SWPS_TRY(tkey2.ensure((uint64_t)S2 * 8));
  SWPS_TRY(k2s.ensure((uint64_t)S2 * 8));
  SWPS_TRY(pid.ensure((uint64_t)S2 * 4));
  SWPS_TRY(perm2.ensure((uint64_t)S2 * 4));
  SWPS_TRY(d_p0.ensure(std::max<uint64_t>(cut.size(), 1) * 4));
  k_lr_tile_pieces<<<nblk(n), 256, 0, s>>>(ks.as<uint64_t>(), head.as<uint32_t>(), pidr.as<uint32_t>(), n, tbits,
                                            tkey2.as<uint64_t>(), pid.as<uint32_t>());
  k_lr_tile_first<<<nblk(cut.size()), 256, 0, s>>>(d_cut.as<uint32_t>(), cut.size(), pidr.as<uint32_t>(),
                                                    d_p0.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  head.release();
  pidr.release();
  sb = 0;  // stable: a key's pieces stay in (tile, record) order
  SWPS_HIP(sort_pairs(nullptr, sb, tkey2.as<uint64_t>(), k2s.as<uint64_t>(), pid.as<uint32_t>(), perm2.as<uint32_t>(),
                      S2, 32 + bbits, s));
  SWPS_TRY(tmp.ensure(sb));
  sb = tmp.bytes;
  SWPS_HIP(sort_pairs(tmp.p, sb, tkey2.as<uint64_t>(), k2s.as<uint64_t>(), pid.as<uint32_t>(), perm2.as<uint32_t>(),
                      S2, 32 + bbits, s));
  SWPS_TRY(head2.ensure((uint64_t)S2 * 4));
  SWPS_TRY(gid.ensure((uint64_t)S2 * 4));
  k_lr_tile_heads<<<nblk(S2), 256, 0, s>>>(k2s.as<uint64_t>(), S2, head2.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  SWPS_TRY(lr_scan_incl(head2.as<uint32_t>(), gid.as<uint32_t>(), S2, tmp, s));
  uint32_t R2 = 0;
  SWPS_HIP(hipMemcpyAsync(&R2, gid.as<uint32_t>() + S2 - 1, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  if (R2 != R) return fail(SWPS_E_STATE, "LR tile index: run count mismatch");
  SWPS_TRY(d_bsub.ensure((nb + 1) * 8));
  SWPS_TRY(d_bcnt.ensure((nb + 1) * 4));
  k_lr_idx_bruns<<<nblk(nb + 1), 256, 0, s>>>(k2s.as<uint64_t>(), S2, nb, d_bsub.as<uint64_t>(), d_bcnt.as<uint32_t>());
  SWPS_TRY(l->d_tslot.ensure((uint64_t)S2 * 4));
  SWPS_TRY(l->d_tinfo.ensure((uint64_t)S2 * 4));
  SWPS_TRY(l->d_tgrun.ensure((uint64_t)S2 * 4));
  SWPS_TRY(l->d_tdst.ensure((uint64_t)S2 * 4));
  l->tile_npieces = S2;
  SWPS_TRY(pfirst.ensure(R * 4));
  SWPS_TRY(l->d_tnp.ensure(R * 4));
  SWPS_TRY(l->d_tpst.ensure(R * 4));
  k_lr_tile_link<<<nblk(S2), 256, 0, s>>>(k2s.as<uint64_t>(), perm2.as<uint32_t>(), head2.as<uint32_t>(),
                                           gid.as<uint32_t>(), S2, d_bsub.as<uint64_t>(), l->d_tslot.as<uint32_t>(),
                                           pfirst.as<uint32_t>());
  k_lr_tile_np<<<nblk(R), 256, 0, s>>>(pfirst.as<uint32_t>(), R, S2, rkey.as<uint64_t>(), d_bsub.as<uint64_t>(),
                                        l->d_tnp.as<uint32_t>(), l->d_tpst.as<uint32_t>());
  k_lr_tile_info<<<nblk(S2), 256, 0, s>>>(k2s.as<uint64_t>(), perm2.as<uint32_t>(), gid.as<uint32_t>(), S2,
                                           d_brun.as<uint64_t>(), l->d_tnp.as<uint32_t>(), l->d_tinfo.as<uint32_t>(),
                                           l->d_tgrun.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  // first piece of every block; the runs with several pieces
  std::vector<uint64_t> bsub(nb + 1);
  std::vector<uint32_t> np(R), p0(cut.size()), pst(R), rcnt(R);
  SWPS_HIP(hipMemcpyAsync(pst.data(), l->d_tpst.p, R * 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipMemcpyAsync(rcnt.data(), l->d_rcnt.p, R * 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipMemcpyAsync(bsub.data(), d_bsub.p, (nb + 1) * 8, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipMemcpyAsync(np.data(), l->d_tnp.p, R * 4, hipMemcpyDeviceToHost, s));
  if (!cut.empty()) SWPS_HIP(hipMemcpyAsync(p0.data(), d_p0.p, cut.size() * 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  std::vector<uint32_t> multi, mlong;
  l->bmulti.assign(nb + 1, 0);
  l->bmlong.assign(nb + 1, 0);
  l->max_bpiece = 0;
  for (uint64_t b = 0; b < nb; b++) {
    l->bmulti[b] = multi.size() / 4;
    l->bmlong[b] = mlong.size() / 4;
    l->max_bpiece = std::max<uint64_t>(l->max_bpiece, bsub[b + 1] - bsub[b]);
    for (uint64_t q = l->bchunk[b]; q < l->bchunk[b + 1]; q++) {  // first and end piece (global)
      chunks[q * 5 + 3] = p0[q];
      chunks[q * 5 + 4] = q + 1 < cut.size() ? p0[q + 1] : S2;
    }
    for (uint64_t g = l->brun[b]; g < l->brun[b + 1]; g++)
      if (np[g] > 1)  // {first slot, partials, records, run}
        (np[g] > kTileFinShort ? mlong : multi).insert((np[g] > kTileFinShort ? mlong : multi).end(),
                                                       {pst[g], np[g], rcnt[g], (uint32_t)g});
  }
  l->bmulti[nb] = multi.size() / 4;
  l->bmlong[nb] = mlong.size() / 4;
  if (l->xcd)
    for (uint64_t b = 0; b < nb; b++) {  // key octile of each block within its tile
      const uint64_t q0 = l->bchunk[b], q1 = l->bchunk[b + 1];
      std::vector<uint32_t> oct(q1 - q0);
      for (uint64_t q = q0; q < q1;) {
        uint64_t e = q;
        while (e < q1 && chunks[e * 5] == chunks[q * 5]) e++;
        for (uint64_t j = q; j < e; j++) oct[j - q0] = (uint32_t)((j - q) * 8 / (e - q));
        q = e;
      }
      lr_xcd_order(chunks, 5, q0, q1, oct);
    }
  if (multi.empty()) multi.assign(4, 0);
  if (mlong.empty()) mlong.assign(4, 0);
  SWPS_TRY(l->d_tmsrow.ensure(multi.size()));  // 4 B per entry: the runs' shard rows (single GPU)
  SWPS_TRY(l->d_tmlrow.ensure(mlong.size()));
  SWPS_TRY(upload(l->d_tmlong, mlong, s));
  if (chunks.empty()) chunks.assign(5, 0);
  SWPS_TRY(upload(l->d_tchunk, chunks, s));
  SWPS_TRY(upload(l->d_tmulti, multi, s));
  SWPS_TRY(l->d_tpart.ensure(std::max<uint64_t>(l->max_bpiece, 1) * 8));
  SWPS_HIP(hipStreamSynchronize(s));
  l->tiles_ready = true;
  return SWPS_OK;
}

// The static per-batch index (see k_lr_idx_*): one (batch << 32 | vid) radix
// sort of every record of the corpus at load time.
int lr_index(swps_lr *l) {
  hipStream_t s = l->s;
  const uint64_t nr = l->label.size(), nb = l->nbatches, B1 = (uint64_t)l->B1();
  const uint64_t n = l->row_off[nr];
  if (n >= (1ULL << 32)) return fail(SWPS_E_UNSUPPORTED, "more than 2^32 features per rank");
  std::vector<uint64_t> bnz0(nb + 1);
  for (uint64_t b = 0; b <= nb; b++) bnz0[b] = l->row_off[std::min<uint64_t>(nr, b * B1)];
  l->index_built = true;
  l->rows_mapped = false;
  DevMem d_bnz0, key, idx, ks, perm, head, rid1, rkey, tmp;
  SWPS_TRY(upload(d_bnz0, bnz0, s));
  SWPS_TRY(l->d_srow.ensure(std::max<uint64_t>(n, 1) * 4));
  SWPS_TRY(l->d_spos.ensure(std::max<uint64_t>(n, 1) * 4));
  SWPS_TRY(l->d_sval.ensure(std::max<uint64_t>(n, 1) * 4));
  SWPS_TRY(l->d_bnruns.ensure(std::max<uint64_t>(nb, 1) * 4));
  l->brun.assign(nb + 1, 0);
  if (n == 0) return SWPS_OK;
  SWPS_TRY(key.ensure(n * 8));
  SWPS_TRY(idx.ensure(n * 4));
  SWPS_TRY(ks.ensure(n * 8));
  SWPS_TRY(perm.ensure(n * 4));
  k_lr_idx_keys<<<nblk(nr), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), nr, B1, l->d_fvid.as<int32_t>(),
                                          key.as<uint64_t>(), idx.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  int vbits = 1;
  while ((1ULL << vbits) <= l->vocab_keys.size()) vbits++;
  int bbits = 1;
  while ((1ULL << bbits) <= nb) bbits++;
  // stable on (batch, vid): the batch's records stay in (row, feature) order inside a key,
  // the order the per-minibatch sort produced (lr.cpp:358-375's accumulation order)
  size_t sb = 0;
  SWPS_HIP(sort_pairs(nullptr, sb, key.as<uint64_t>(), ks.as<uint64_t>(), idx.as<uint32_t>(), perm.as<uint32_t>(), n,
                      32 + bbits, s));
  SWPS_TRY(tmp.ensure(sb));
  sb = tmp.bytes;
  SWPS_HIP(sort_pairs(tmp.p, sb, key.as<uint64_t>(), ks.as<uint64_t>(), idx.as<uint32_t>(), perm.as<uint32_t>(), n,
                      32 + bbits, s));
  (void)vbits;
  key.release();
  idx.release();
  SWPS_TRY(head.ensure(n * 4));
  SWPS_TRY(rid1.ensure(n * 4));
  k_lr_rowid<<<nblk(nr), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), nr, rid1.as<uint32_t>());
  k_lr_idx_slots<<<nblk(n), 256, 0, s>>>(ks.as<uint64_t>(), perm.as<uint32_t>(), n, rid1.as<uint32_t>(),
                                          l->d_fval.as<float>(), l->d_srow.as<uint32_t>(), l->d_sval.as<float>(),
                                          head.as<uint32_t>(), l->d_spos.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  SWPS_TRY(lr_scan_incl(head.as<uint32_t>(), rid1.as<uint32_t>(), n, tmp, s));
  SWPS_TRY(l->d_frun.ensure(n * 4));
  k_lr_idx_frun<<<nblk(n), 256, 0, s>>>(perm.as<uint32_t>(), rid1.as<uint32_t>(), n, l->d_frun.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  uint32_t R = 0;
  SWPS_HIP(hipMemcpyAsync(&R, rid1.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  SWPS_TRY(rkey.ensure((uint64_t)R * 8));
  SWPS_TRY(l->d_ruk.ensure((uint64_t)R * 4));
  SWPS_TRY(l->d_roff.ensure((uint64_t)R * 4));
  SWPS_TRY(l->d_rcnt.ensure((uint64_t)R * 4));
  k_lr_idx_runs<<<nblk(n), 256, 0, s>>>(ks.as<uint64_t>(), head.as<uint32_t>(), rid1.as<uint32_t>(), n,
                                         d_bnz0.as<uint64_t>(), rkey.as<uint64_t>(), l->d_ruk.as<uint32_t>(),
                                         l->d_roff.as<uint32_t>());
  k_lr_idx_cnt<<<nblk(R), 256, 0, s>>>(rkey.as<uint64_t>(), l->d_roff.as<uint32_t>(), R, d_bnz0.as<uint64_t>(),
                                        l->d_rcnt.as<uint32_t>());
  DevMem d_brun;
  SWPS_TRY(d_brun.ensure((nb + 1) * 8));
  k_lr_idx_bruns<<<nblk(nb + 1), 256, 0, s>>>(rkey.as<uint64_t>(), R, nb, d_brun.as<uint64_t>(),
                                               l->d_bnruns.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  SWPS_HIP(hipMemcpyAsync(l->brun.data(), d_brun.p, (nb + 1) * 8, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  l->max_bruns = 0;
  for (uint64_t b = 0; b < nb; b++) l->max_bruns = std::max<uint64_t>(l->max_bruns, l->brun[b + 1] - l->brun[b]);
  // every batch's long runs (> kLrShort records), relative to its first run: k_lr_reduce_fused
  {
    std::vector<uint32_t> cnt(R);
    if (R) SWPS_HIP(hipMemcpy(cnt.data(), l->d_rcnt.p, (uint64_t)R * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> lst;
    l->blong.assign(nb + 1, 0);
    for (uint64_t b = 0; b < nb; b++) {
      l->blong[b] = lst.size();
      for (uint64_t q = l->brun[b]; q < l->brun[b + 1]; q++)
        if (cnt[q] > kLrShort) lst.push_back((uint32_t)(q - l->brun[b]));
    }
    l->blong[nb] = lst.size();
    if (lst.empty()) lst.push_back(0);
    SWPS_TRY(upload(l->d_slong, lst, s));
    // every batch's kLrHot most frequent keys (runs of at least 8 records): the forward's LDS weights
    std::vector<int32_t> hot_of_run(std::max<uint64_t>(R, 1), -1);
    std::vector<uint32_t> hgrun(std::max<uint64_t>(nb, 1) * kLrHot, 0);
    l->bnhot.assign(nb, 0);
    std::vector<uint32_t> ord;
    for (uint64_t b = 0; b < nb; b++) {
      ord.clear();
      for (uint64_t q = l->brun[b]; q < l->brun[b + 1]; q++)
        if (cnt[q] >= 8) ord.push_back((uint32_t)q);
      const size_t h = std::min<size_t>(ord.size(), (size_t)l->nhot);
      std::partial_sort(ord.begin(), ord.begin() + h, ord.end(), [&](uint32_t x, uint32_t y) {
        return cnt[x] != cnt[y] ? cnt[x] > cnt[y] : x < y;
      });
      for (size_t i = 0; i < h; i++) {
        hot_of_run[ord[i]] = (int32_t)i;
        hgrun[b * kLrHot + i] = ord[i];
      }
      l->bnhot[b] = (uint32_t)h;
    }
    SWPS_TRY(upload(l->d_hot_of_run, hot_of_run, s));
    SWPS_TRY(upload(l->d_hgrun, hgrun, s));
    SWPS_HIP(hipStreamSynchronize(s));
  }
  l->tiles_ready = false;
  if (l->cfg.fast_sums && l->tiles) SWPS_TRY(lr_tile_index(l, ks, perm, rid1, rkey, d_brun, R, bbits, tmp));
  return SWPS_OK;
}

// every record's vid on the host (the sharded schedule, the row placement experiment), once
int lr_fvid_host(swps_lr *l) {
  const uint64_t n = l->row_off.empty() ? 0 : l->row_off.back();
  if (l->fvid.size() == n) return SWPS_OK;
  l->fvid.resize(n);
  if (n) SWPS_HIP(hipMemcpyAsync(l->fvid.data(), l->d_fvid.p, n * 4, hipMemcpyDeviceToHost, l->s));
  SWPS_HIP(hipStreamSynchronize(l->s));
  return SWPS_OK;
}

// The corpus vocabulary on the GPU: a stable radix sort of every record's key gives the distinct
// keys in key order — vid = rank — each key's first record and record count.  The reference's
// first pull visits lr.cpp:161-166's `_local_keys` (std::unordered_set<unsigned>) in iteration
// order, which depends only on the order the keys were first inserted: with init_ref, the V
// distinct keys (not the records) are inserted in first-occurrence order on the host and the
// iteration order kept as the init's pull order.
int lr_vocab(swps_lr *l, const uint32_t *feat, uint64_t n) {
  hipStream_t s = l->s;
  if (n >= (1ULL << 32)) return fail(SWPS_E_UNSUPPORTED, "more than 2^32 features per rank");
  SWPS_TRY(l->d_fvid.ensure(std::max<uint64_t>(n, 1) * 4));
  l->vocab_keys.clear();
  l->pull_order.clear();
  l->vocab_cnt.clear();
  l->fvid.clear();
  if (!n) return SWPS_OK;
  DevMem dfeat, ks, perm, head, rank, ukey, ufirst, ustart, tmp;
  SWPS_TRY(dfeat.ensure(n * 4));
  SWPS_HIP(hipMemcpyAsync(dfeat.p, feat, n * 4, hipMemcpyHostToDevice, s));
  SWPS_TRY(ks.ensure(n * 4));
  SWPS_TRY(perm.ensure(n * 4));
  size_t b = 0;
  SWPS_HIP(sort_pairs_iota(nullptr, b, dfeat.as<uint32_t>(), ks.as<uint32_t>(), perm.as<uint32_t>(), n, 32, s));
  SWPS_TRY(tmp.ensure(b));
  b = tmp.bytes;
  SWPS_HIP(sort_pairs_iota(tmp.p, b, dfeat.as<uint32_t>(), ks.as<uint32_t>(), perm.as<uint32_t>(), n, 32, s));
  dfeat.release();
  SWPS_TRY(head.ensure(n * 4));
  SWPS_TRY(rank.ensure(n * 4));
  k_lr_voc_heads<<<nblk(n), 256, 0, s>>>(ks.as<uint32_t>(), n, head.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  SWPS_TRY(lr_scan_incl(head.as<uint32_t>(), rank.as<uint32_t>(), n, tmp, s));
  uint32_t V = 0;
  SWPS_HIP(hipMemcpyAsync(&V, rank.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  SWPS_TRY(ukey.ensure((uint64_t)V * 4));
  SWPS_TRY(ufirst.ensure((uint64_t)V * 4));
  SWPS_TRY(ustart.ensure((uint64_t)V * 4));
  k_lr_voc_ids<<<nblk(n), 256, 0, s>>>(ks.as<uint32_t>(), perm.as<uint32_t>(), rank.as<uint32_t>(), n,
                                       l->d_fvid.as<int32_t>(), ukey.as<uint32_t>(), ufirst.as<uint32_t>(),
                                       ustart.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  std::vector<uint32_t> uk(V), us(V);
  SWPS_HIP(hipMemcpyAsync(uk.data(), ukey.p, (uint64_t)V * 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipMemcpyAsync(us.data(), ustart.p, (uint64_t)V * 4, hipMemcpyDeviceToHost, s));
  std::vector<uint32_t> order;
  if (l->cfg.init_ref) {  // the distinct keys by first occurrence
    DevMem fs, ord;
    SWPS_TRY(fs.ensure((uint64_t)V * 4));
    SWPS_TRY(ord.ensure((uint64_t)V * 4));
    int fb = 1;
    while ((1ULL << fb) < n) fb++;
    b = 0;
    SWPS_HIP(sort_pairs_iota(nullptr, b, ufirst.as<uint32_t>(), fs.as<uint32_t>(), ord.as<uint32_t>(), V, fb, s));
    SWPS_TRY(tmp.ensure(b));
    b = tmp.bytes;
    SWPS_HIP(sort_pairs_iota(tmp.p, b, ufirst.as<uint32_t>(), fs.as<uint32_t>(), ord.as<uint32_t>(), V, fb, s));
    order.resize(V);
    SWPS_HIP(hipMemcpyAsync(order.data(), ord.p, (uint64_t)V * 4, hipMemcpyDeviceToHost, s));
  }
  SWPS_HIP(hipStreamSynchronize(s));
  l->vocab_keys.assign(uk.begin(), uk.end());
  l->vocab_cnt.resize(V);
  for (uint32_t r = 0; r < V; r++) l->vocab_cnt[r] = (r + 1 < V ? us[r + 1] : (uint32_t)n) - us[r];
  if (l->cfg.init_ref) {
    std::unordered_set<uint32_t> K0;  // default-constructed, grown by inserts: the reference's buckets
    for (uint32_t r : order) K0.insert(uk[r]);
    l->pull_order.reserve(V);
    for (uint32_t k : K0) l->pull_order.push_back((uint32_t)(std::lower_bound(uk.begin(), uk.end(), k) - uk.begin()));
  }
  return SWPS_OK;
}

// SWPS_LR_LOAD_TIMES: the load's phases on stderr
struct LoadTimer {
  bool on = getenv("SWPS_LR_LOAD_TIMES") != nullptr;
  double t = now();
  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void operator()(const char *what) {
    if (!on) return;
    const double u = now();
    fprintf(stderr, "[lr load] %-30s %8.4f s\n", what, u - t);
    t = u;
  }
};

// every label and feature value finite (lr.cpp:103-131 parses "nan" / "inf" with %f and trains on
// them silently; here they are refused at load: they would make every sum they reach — and the
// fixed-point scale, from max |x_i| — undefined).  Threads over slices of the values.
int lr_check_finite(const swps_lr *l) {
  for (uint64_t r = 0; r < l->label.size(); r++)
    if (!std::isfinite(l->label[r])) return fail(SWPS_E_CFG, "non-finite label at row " + std::to_string(r));
  const uint64_t nf = l->fval.size();
  const int nth = (int)std::min<uint64_t>(16, std::max<uint64_t>(1, nf >> 22));
  std::vector<uint64_t> bad(nth, ~0ull);
  std::vector<std::thread> th;
  for (int q = 0; q < nth; q++)
    th.emplace_back([&, q] {
      for (uint64_t i = nf * q / nth; i < nf * (q + 1) / nth; i++)
        if (!std::isfinite(l->fval[i])) {
          bad[q] = i;
          return;
        }
    });
  for (auto &t : th) t.join();
  for (uint64_t b : bad)
    if (b != ~0ull) {
      const uint64_t row = (uint64_t)(std::upper_bound(l->row_off.begin(), l->row_off.end(), b) - l->row_off.begin()) - 1;
      return fail(SWPS_E_CFG, "non-finite feature value at record " + std::to_string(b) + " (row " +
                                  std::to_string(row) + ")");
    }
  return SWPS_OK;
}

// the 1st percentile of |x_i| over the nonzero values (a deterministic sample of at most 2^20 of them)
double lr_small_abs_x(const swps_lr *l) {
  const uint64_t nf = l->fval.size(), step = std::max<uint64_t>(1, nf >> 20);
  std::vector<float> a;
  a.reserve(nf / step + 1);
  for (uint64_t i = 0; i < nf; i += step)
    if (l->fval[i] != 0.f) a.push_back(std::fabs(l->fval[i]));
  if (a.empty()) return 0.0;
  std::nth_element(a.begin(), a.begin() + a.size() / 100, a.end());
  return a[a.size() / 100];
}

// feat: the caller's array of every record's key (read during this call only)
int lr_ingest(swps_lr *l, const uint32_t *feat, uint64_t nfeat) {
  LoadTimer phase;
  SWPS_TRY(lr_check_finite(l));
  l->cfg.plan = l->plan_req;  // a reload decides the fixed point's floor again
  l->fx_fallback = false;
  l->fx_floor = 0;
  SWPS_TRY(lr_vocab(l, feat, nfeat));
  phase("vocabulary (GPU sort)");
  const uint64_t nr = l->label.size();
  l->nbatches = nr ? (nr + l->B1() - 1) / l->B1() : 0;
  // the rows the single-GPU init gives the keys (swps_lr_init): in the order the keys first appear,
  // by (batch, row tile), then by key.  A batch's keys seen for the first time — most of its
  // ~144k keys on Criteo-like data after the first batches — then sit in one dense run of rows that
  // its forward and its row tiles walk in key order, and the keys of the first batches (the
  // frequent ones) in a few MB: the weight gathers and row updates share 128-B lines instead of
  // touching one line per key in a table of millions of rows
  l->vid_place.clear();
  if (l->place) {
    SWPS_TRY(lr_fvid_host(l));
    const uint64_t B1 = l->B1(), V = l->vocab_keys.size();
    const uint64_t ntile = (B1 + (1ULL << l->tile_bits) - 1) >> l->tile_bits;
    std::vector<uint64_t> grp(V, ~0ull);
    for (uint64_t r = 0; r < nr; r++) {
      const uint64_t g = l->place == 2 ? r / B1 : (r / B1) * ntile + ((r % B1) >> l->tile_bits);
      for (uint64_t c = l->row_off[r]; c < l->row_off[r + 1]; c++)
        if (grp[l->fvid[c]] == ~0ull) grp[l->fvid[c]] = g;
    }
    std::vector<std::pair<uint64_t, uint32_t>> ord(V);
    for (uint64_t i = 0; i < V; i++) ord[i] = {(grp[i] << 32) | (uint32_t)l->vocab_keys[i], (uint32_t)i};
    std::sort(ord.begin(), ord.end());
    l->vid_place.resize(V);
    for (uint64_t j = 0; j < V; j++) l->vid_place[ord[j].second] = (uint32_t)j;
  }
  phase("row placement (host)");
  hipStream_t s = l->s;
  SWPS_TRY(upload(l->d_label, l->label, s));
  SWPS_TRY(upload(l->d_row_off, l->row_off, s));
  SWPS_TRY(upload(l->d_fval, l->fval, s));
  SWPS_TRY(l->d_vid_row.ensure(std::max<size_t>(1, l->vocab_keys.size()) * 4));
  SWPS_TRY(l->d_err.ensure((std::max<uint64_t>(1, nr) + 4) * 4));  // + slack: k_lr_tiles' 16-B loads
  SWPS_TRY(l->d_err2.ensure(std::max<uint64_t>(1, nr) * 4));
  // per batch: its longest row and record count
  {
    const uint64_t B1 = l->B1();
    l->max_bnnz = 0;
    l->bmaxf.assign(l->nbatches, 0);
    for (uint64_t r = 0; r < nr; r++)
      l->bmaxf[r / B1] = std::max<uint32_t>(l->bmaxf[r / B1], (uint32_t)(l->row_off[r + 1] - l->row_off[r]));
    for (uint64_t b = 0; b < l->nbatches; b++)
      l->max_bnnz = std::max<uint64_t>(l->max_bnnz,
                                       l->row_off[std::min<uint64_t>(nr, (b + 1) * B1)] - l->row_off[b * B1]);
  }
  // the per-step plan builds each batch's index while the previous batch trains; otherwise (exact
  // sums, the record path, SWPS_LR_PLAN_LOAD) every batch's index is built here, once
  l->index_built = false;
  l->plan_ready = false;
  l->plan_next = 0;
  l->fx_ready = false;
  phase("uploads + batch extents");
  if (l->cfg.plan == SWPS_LR_PLAN_NONE && l->cfg.fast_sums) {
    // the fixed-point step: its scale (every sum below 2^62: |e| <= max|y| + 1, at most the batch's
    // records per key) and the corpus's most frequent keys (their sums go through LDS)
    float mx = 0.f, my = 0.f;
    {  // max |x_i| over the corpus: threads over slices
      const uint64_t nf = l->fval.size();
      const int nth = (int)std::min<uint64_t>(16, std::max<uint64_t>(1, nf >> 22));
      std::vector<float> part(nth, 0.f);
      std::vector<std::thread> th;
      for (int q = 0; q < nth; q++)
        th.emplace_back([&, q] {
          float m = 0.f;
          for (uint64_t i = nf * q / nth; i < nf * (q + 1) / nth; i++) m = std::max(m, std::fabs(l->fval[i]));
          part[q] = m;
        });
      for (auto &t : th) t.join();
      for (float m : part) mx = std::max(mx, m);
    }
    for (float v : l->label) my = std::max(my, std::fabs(v));
    const double bound = std::max(1e-30, ((double)my + 1.0) * (double)mx * (double)std::max<uint64_t>(l->max_bnnz, 1));
    l->fx_bits = (int)std::min(40.0, std::floor(62.0 - std::log2(bound)));
    // the floor: a term e * x_i is rounded to a multiple of 2^-s, so the quantum must stay below
    // 1e-7 of a small term — |e| = 0.5 times the 1st percentile of |x_i| — as fp32's own rounding
    // of such a term (2^-24 relative) would.  Heavy-tailed values (|x_i| from 1e-4 to 1e6) push s
    // down past it (s = 26 against a floor of 38 there; Criteo's shape: 39 against 30); then the
    // step runs the fp64-sum path (plan step) instead, and swps_lr_plan_info says so.
    const double small = lr_small_abs_x(l);
    l->fx_floor = small > 0 ? (int)std::ceil(std::log2(1.0 / (1e-7 * 0.5 * small))) : 0;
    if (getenv("SWPS_LR_FX_FLOOR")) l->fx_floor = atoi(getenv("SWPS_LR_FX_FLOOR"));  // tests: force it
    if (l->fx_bits < l->fx_floor) {
      l->fx_fallback = true;
      l->cfg.plan = SWPS_LR_PLAN_STEP;
    }
  }
  if (l->cfg.plan == SWPS_LR_PLAN_NONE && l->cfg.fast_sums) {
    const std::vector<uint32_t> &cnt = l->vocab_cnt;
    std::vector<uint32_t> ord;
    for (uint32_t v = 0; v < cnt.size(); v++)
      if (cnt[v] >= 8) ord.push_back(v);
    const size_t h = std::min<size_t>(ord.size(), (size_t)l->nhot);
    std::partial_sort(ord.begin(), ord.begin() + h, ord.end(),
                      [&](uint32_t a, uint32_t b) { return cnt[a] != cnt[b] ? cnt[a] > cnt[b] : a < b; });
    l->fx_hot_vids.assign(ord.begin(), ord.begin() + h);
    // fids: the hot keys by rank, then the others in the placement order above (or by vid); the
    // rows are placed in that order
    const uint64_t V = l->vocab_keys.size();
    std::vector<uint32_t> by(V);
    if (l->vid_place.size() == V)
      for (uint64_t v = 0; v < V; v++) by[l->vid_place[v]] = (uint32_t)v;
    else
      for (uint64_t v = 0; v < V; v++) by[v] = (uint32_t)v;
    l->fx_fid.assign(V, ~0u);
    for (size_t q = 0; q < h; q++) l->fx_fid[l->fx_hot_vids[q]] = (uint32_t)q;
    uint32_t next = (uint32_t)h;
    for (uint64_t j = 0; j < V; j++)
      if (l->fx_fid[by[j]] == ~0u) l->fx_fid[by[j]] = next++;
    l->vid_place = l->fx_fid;
    phase("fixed-point scale, hot keys, fids");
  }
  if (!((l->cfg.plan == SWPS_LR_PLAN_STEP || l->cfg.plan == SWPS_LR_PLAN_NONE) && l->cfg.fast_sums && l->tiles))
    SWPS_TRY(lr_index(l));
  l->rows_mapped = false;
  SWPS_HIP(hipStreamSynchronize(s));
  l->loaded = true;
  return SWPS_OK;
}

// the forward's chunks of whole rows of every batch (k_lr_forward_c), once: from the row lengths
// only (rows never span chunks; a row longer than a chunk's capacity turns the form off)
int lr_fwd_chunks(swps_lr *l) {
  if (!(l->fwd_c && l->rows_per_wave == 1 && !l->fwd_diag && !l->stage && l->bfchunk.empty())) return SWPS_OK;
  const uint64_t nr = l->label.size();
  hipStream_t s = l->s;
  std::vector<uint2> ch;
  std::vector<uint32_t> c0;
  l->fwd_rpt = l->fwd_c == 4 || l->fwd_c == 16 ? l->fwd_c : kLrFwdRpt;  // records per thread (A/B: 4, 8, 16)
  if (l->cfg.plan == SWPS_LR_PLAN_NONE && l->cfg.fast_sums && l->fwd_c == 1) {
    // the fixed-point step: chunks of 4,096 records (its push reads each (chunk, bucket) segment:
    // fewer, longer segments); SWPS_LR_FX_RPT = 8 for 2,048
    const char *e = getenv("SWPS_LR_FX_RPT");
    l->fwd_rpt = e && atoi(e) == 8 ? 8 : 16;
  }
  const uint64_t cap = (uint64_t)l->fwd_rpt * 256;
  l->bfchunk.assign(1, 0);
  for (uint64_t b = 0; b < l->nbatches && l->fwd_c; b++) {
    const uint64_t a0 = b * l->B1(), a1 = std::min<uint64_t>(nr, a0 + l->B1());
    uint64_t first = a0;
    for (uint64_t r = a0; r < a1; r++) {
      if (l->row_off[r + 1] - l->row_off[r] > cap) {
        l->fwd_c = 0;
        break;
      }
      if (l->row_off[r + 1] - l->row_off[first] > cap) {
        ch.push_back(make_uint2((uint32_t)(first - a0), (uint32_t)(r - first)));
        c0.push_back((uint32_t)(l->row_off[first] - l->row_off[a0]));
        first = r;
      }
    }
    if (a1 > first) {
      ch.push_back(make_uint2((uint32_t)(first - a0), (uint32_t)(a1 - first)));
      c0.push_back((uint32_t)(l->row_off[first] - l->row_off[a0]));
    }
    l->bfchunk.push_back(ch.size());
    l->max_bchunks = std::max<uint64_t>(l->max_bchunks, l->bfchunk[b + 1] - l->bfchunk[b]);
  }
  if (l->fwd_c) {
    SWPS_TRY(upload(l->d_fchunk, ch, s));
    SWPS_TRY(upload(l->d_fchunk_c0, c0, s));
    SWPS_HIP(hipStreamSynchronize(s));  // `ch` is a local
  }
  return SWPS_OK;
}

// ---- the per-step plan: setup, one batch's plan on the plan stream, the planned step ----------
bool lr_plan_usable(const swps_lr *l) {
  return l->cfg.plan == SWPS_LR_PLAN_STEP && !l->sharded && l->cfg.fast_sums && l->tiles && l->fwd_c &&
         l->rows_per_wave == 1 && !l->fwd_diag && !l->stage && !l->fwd_records && !l->inline_records &&
         l->tile_threads == 256 && l->nbatches > 0;
}

bool lr_fx_usable(const swps_lr *l) {
  return l->cfg.plan == SWPS_LR_PLAN_NONE && !l->sharded && l->cfg.fast_sums && l->fwd_c && l->rows_per_wave == 1 &&
         !l->fwd_diag && !l->stage && l->nbatches > 0 && (l->fwd_rpt == 8 || l->fwd_rpt == 16);
}

// the sharded learner's fixed-point step: the bucketed form only (its LDS bounds), vids as keys
bool lr_fx_sharded_usable(const swps_lr *l) {
  const uint64_t V = l->vocab_keys.size();
  const char *e = getenv("SWPS_LR_FX_SHARDED");
  return l->cfg.plan == SWPS_LR_PLAN_NONE && l->cfg.fast_sums && l->fwd_c && l->rows_per_wave == 1 &&
         !l->fwd_diag && !l->stage && l->nbatches > 0 && (l->fwd_rpt == 8 || l->fwd_rpt == 16) && V > 0 &&
         ((V + (1u << kLrFxVB) - 1) >> kLrFxVB) <= kLrFxMaxBk && (2 * l->max_bchunks + 1) * 4 <= 96 * 1024 &&
         !(getenv("SWPS_LR_FX_ATOMIC") && atoi(getenv("SWPS_LR_FX_ATOMIC")) != 0) && !(e && atoi(e) == 0) &&
         l->fx_fid.size() == V;
}

// one batch of the fixed-point step: k_lr_fxb_step over the batch's chunks of whole rows, then
// k_lr_fxb_push over its buckets and hot keys (the atomic form: k_lr_fx_step, k_lr_fx_apply)
int lr_batch_fx(swps_lr *l, const float *d_vals = nullptr, float *d_grads = nullptr) {
  hipStream_t s = l->s;
  const bool shd = l->fx_sharded;
  const uint64_t V = std::max<uint64_t>(l->vocab_keys.size(), 1), cap = l->t->cfg.capacity;
  if (!l->fx_ready) {  // the per-key codes (shard rows are fixed from swps_lr_init on) and buffers
    const bool hot = l->hot != 0 && !l->fx_hot_vids.empty();
    const uint32_t nh = hot ? (uint32_t)l->fx_hot_vids.size() : 0u;
    SWPS_TRY(l->d_vcode.ensure(V * 4));
    SWPS_TRY(l->d_fx_hrow.ensure(kLrHot * 4));
    std::vector<int32_t> hov;
    if (hot) {
      hov.assign(V, -1);
      for (uint32_t q = 0; q < nh; q++) hov[l->fx_hot_vids[q]] = (int32_t)q;
    }
    DevMem dhov;
    // sharded: a key's "row" is its vid (wcache2[2 * vid]); single GPU: its shard row
    const uint32_t *vr = shd ? nullptr : l->d_vid_row.as<uint32_t>();
    if (hot) {
      SWPS_TRY(upload(dhov, hov, s));
      SWPS_TRY(upload(l->d_fx_hot, l->fx_hot_vids, s));
      k_lr_fx_hrow<<<nblk(nh), 256, 0, s>>>(l->d_fx_hot.as<uint32_t>(), nh, vr, l->d_fx_hrow.as<uint32_t>());
    }
    k_lr_fx_codes<<<nblk(V), 256, 0, s>>>(vr, l->vocab_keys.size(),
                                          hot ? dhov.as<int32_t>() : nullptr, l->d_vcode.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    const char *ea = getenv("SWPS_LR_FX_ATOMIC");  // A/B and tests: the per-record atomic form
    l->fx_atomic = ea && atoi(ea) != 0;
    if (const char *eg = getenv("SWPS_LR_FXB_GRID")) l->fxb_grid = (uint32_t)std::max(1, atoi(eg));
    if (const char *ed = getenv("SWPS_LR_FXB_DIAG")) l->fxb_diag = (uint32_t)atoi(ed);
    if (const char *ex = getenv("SWPS_LR_FXB_XCD")) l->fxb_xcd = atoi(ex) != 0;
    if (const char *en = getenv("SWPS_LR_FX_NT")) l->fx_nt = atoi(en) == 512 ? 512 : 256;
    l->fxb_nbk = (uint32_t)((V + (1u << kLrFxVB) - 1) >> kLrFxVB);
    if (l->fxb_nbk > kLrFxMaxBk || (2 * l->max_bchunks + 1) * 4 > 96 * 1024) l->fx_atomic = 1;  // LDS bounds
    if (shd && l->fx_atomic) return fail(SWPS_E_STATE, "sharded fixed-point step needs the bucketed form");
    l->fx_affine = false;
    if (shd) {  // the affine form over wcache2 (row base 0): records carry fids, hot key q = fid q
      const uint64_t nnz = l->row_off.back();
      SWPS_TRY(l->d_ffid.ensure(std::max<uint64_t>(nnz, 1) * 4));
      k_lr_fx_fid<<<nblk(nnz), 256, 0, s>>>(l->d_fvid.as<int32_t>(), nnz, l->d_fx_fidv.as<uint32_t>(),
                                            l->d_ffid.as<int32_t>());
      std::vector<uint32_t> iota(std::max<uint32_t>(nh, 1));
      for (uint32_t q = 0; q < iota.size(); q++) iota[q] = q;
      SWPS_TRY(upload(l->d_fx_hrow, iota, s));
      SWPS_HIP(hipGetLastError());
      SWPS_HIP(hipStreamSynchronize(s));
      l->fx_affine = true;
      l->fx_row_base = 0;
    }
    if (!shd && !l->fx_atomic && l->fx_fid.size() == V && l->vocab_keys.size() == V &&
        !(getenv("SWPS_LR_FX_AFFINE") && atoi(getenv("SWPS_LR_FX_AFFINE")) == 0)) {
      // rows placed in fid order by swps_lr_init (a table that held some keys before breaks it)
      std::vector<uint32_t> vr(V);
      SWPS_HIP(hipMemcpyAsync(vr.data(), l->d_vid_row.p, V * 4, hipMemcpyDeviceToHost, s));
      SWPS_HIP(hipStreamSynchronize(s));
      const uint32_t base = vr[0] - l->fx_fid[0];
      bool aff = (uint64_t)base + V <= l->t->cfg.capacity;
      for (uint64_t v = 0; v < V && aff; v++) aff = vr[v] == base + l->fx_fid[v];
      if (aff) {
        DevMem dfid;
        SWPS_TRY(upload(dfid, l->fx_fid, s));
        const uint64_t nnz = l->row_off.back();
        SWPS_TRY(l->d_ffid.ensure(std::max<uint64_t>(nnz, 1) * 4));
        k_lr_fx_fid<<<nblk(nnz), 256, 0, s>>>(l->d_fvid.as<int32_t>(), nnz, dfid.as<uint32_t>(), l->d_ffid.as<int32_t>());
        SWPS_HIP(hipGetLastError());
        SWPS_HIP(hipStreamSynchronize(s));
        l->fx_affine = true;
        l->fx_row_base = base;
      }
    }
    if (const char *er = getenv("SWPS_LR_FXB_RES")) l->fxb_res = atoi(er) != 0;
    if (const char *er = getenv("SWPS_LR_FXR")) l->fxr = atoi(er) != 0;
    if (const char *em = getenv("SWPS_LR_FX_MIRROR")) l->fx_mirror = atoi(em) != 0;
    if (!l->fx_atomic && l->fxb_res) {
      // the bucket regions: bucket q's region holds any batch's records of its keys — at most the
      // batch's records, and at most the corpus count of its non-hot keys
      const std::vector<uint32_t> &cnt = l->vocab_cnt;
      std::vector<uint8_t> ishot(V, 0);
      if (hot)
        for (uint32_t q = 0; q < nh; q++) ishot[l->fx_hot_vids[q]] = 1;
      std::vector<uint64_t> bsum(l->fxb_nbk, 0);
      for (uint64_t v = 0; v < l->vocab_keys.size(); v++)
        if (!ishot[v]) {
          const uint64_t key = l->fx_affine ? l->fx_fid[v] : v;
          bsum[key >> kLrFxVB] += cnt[v];
        }
      // 2^gbits chunk groups per bucket (chunk % 2^gbits), each its own sub-region and counter: a
      // group's sub-region also holds at most its chunks' records.  The most groups whose regions
      // stay within 2^31 records and 4 GB (SWPS_LR_FXB_GBITS caps it)
      const uint64_t chunk_rec = (uint64_t)l->fwd_rpt * 256;
      int gmax = 3;  // 8 groups (SWPS_LR_FXB_GBITS: 0 .. kLrFxMaxGBits)
      if (const char *eg = getenv("SWPS_LR_FXB_GBITS")) gmax = std::min(std::max(atoi(eg), 0), (int)kLrFxMaxGBits);
      std::vector<uint32_t> rb;
      uint64_t tot = ~0ull;
      for (int gb = gmax; gb >= 0; gb--) {
        const uint64_t G = 1ull << gb, grp = ((l->max_bchunks + G - 1) / G) * chunk_rec;
        rb.assign(((uint64_t)l->fxb_nbk << gb) + 1, 0);
        tot = 0;
        for (uint64_t qg = 0; qg < ((uint64_t)l->fxb_nbk << gb) && tot < (1ull << 31); qg++) {
          rb[qg] = (uint32_t)tot;
          tot += std::min<uint64_t>(std::min<uint64_t>(bsum[qg >> gb], l->max_bnnz), grp);
        }
        l->fxb_gbits = (uint32_t)gb;
        if (tot < (1ull << 31) && (tot * 8 <= (4ull << 30) || gb == 0)) break;
      }
      if (const char *ep = getenv("SWPS_LR_FX_PF")) l->fx_pf = atoi(ep);
      {  // prefetch a bucket's rows in the push where a batch touches many of its keys: on average
         // at least 1,024 non-hot records per batch (of 4,096 keys)
        std::vector<uint8_t> pf(l->fxb_nbk);
        for (uint32_t q = 0; q < l->fxb_nbk; q++)
          pf[q] = l->fx_pf == 2 || (l->fx_pf == 1 && bsum[q] >= 1024ull * std::max<uint64_t>(l->nbatches, 1));
        SWPS_TRY(upload(l->d_pfb, pf, s));
        SWPS_HIP(hipStreamSynchronize(s));
      }
      if (tot < (1ull << 31)) {
        const uint64_t nqg = (uint64_t)l->fxb_nbk << l->fxb_gbits;
        rb[nqg] = (uint32_t)tot;
        SWPS_TRY(upload(l->d_fxb_rbase, rb, s));
        SWPS_TRY(l->d_fxb_fill.ensure(nqg * 4));
        SWPS_HIP(hipMemsetAsync(l->d_fxb_fill.p, 0, nqg * 4, s));
        SWPS_TRY(l->d_fxb_rec.ensure(std::max<uint64_t>(tot, 1) * 8));
        l->fxb_region_recs = tot;
        SWPS_HIP(hipStreamSynchronize(s));  // rb
      } else {
        l->fxb_res = false;
      }
    } else {
      l->fxb_res = false;
    }
    if (!l->fx_atomic) {
      SWPS_TRY(l->d_fxb_rec.ensure(std::max<uint64_t>(l->max_bnnz, 1) * 8));
      SWPS_TRY(l->d_fxb_boff.ensure(std::max<uint64_t>(l->max_bchunks, 1) * (l->fxb_nbk + 1) * 2));
      SWPS_TRY(l->d_fxb_hsum.ensure((uint64_t)l->fxb_grid * kLrHot * 8));
      SWPS_TRY(l->d_fxb_hcnt.ensure((uint64_t)l->fxb_grid * kLrHot * 4));
    } else if (!l->d_acc_sum.p) {
      SWPS_TRY(l->d_acc_sum.ensure(cap * 8));
      SWPS_TRY(l->d_acc_cnt.ensure(cap * 4));
      SWPS_TRY(l->d_fx_stamp.ensure(cap * 4));
      SWPS_HIP(hipMemsetAsync(l->d_acc_sum.p, 0, cap * 8, s));
      SWPS_HIP(hipMemsetAsync(l->d_acc_cnt.p, 0, cap * 4, s));
      SWPS_HIP(hipMemsetAsync(l->d_fx_stamp.p, 0, cap * 4, s));
      l->fx_tag = 0;
    }
    SWPS_TRY(l->d_fx_list.ensure(std::max<uint64_t>(l->max_bnnz, 1) * 4));
    SWPS_TRY(l->d_fx_n.ensure(16));
    SWPS_HIP(hipMemsetAsync(l->d_fx_n.p, 0, 16, s));
    SWPS_HIP(hipStreamSynchronize(s));  // dhov
    l->fx_ready = true;
  }
  const uint64_t step = l->cursor, nr = l->label.size(), bi = step % l->nbatches;
  const uint64_t r0 = bi * l->B1(), r1 = std::min<uint64_t>(nr, r0 + l->B1());
  l->cursor++;
  if (l->row_off[r1] == l->row_off[r0]) {
    l->pull_rows = nullptr;
    l->pushed_in_place = false;
    return SWPS_OK;
  }
  const bool hot = l->hot != 0 && !l->fx_hot_vids.empty();
  const uint64_t nfc = l->bfchunk[bi + 1] - l->bfchunk[bi];
  // sharded, branch-free step: the pulled weights dense by fid (its gathers read 32 per line)
  const bool shd_dense = shd && !l->fx_atomic && l->fxb_res && l->fx_affine && l->fxr;
  // world 1 in place (serve_pull looked the slot's rows up and copied nothing): the install reads the
  // shard rows, localf holds each key's row, and the push applies AdaGrad there (no payload)
  const uint32_t *prow = shd ? l->pull_rows : nullptr;
  l->pull_rows = nullptr;
  const bool w1aff = prow && shd_dense && l->w1_base >= 0;
  if (w1aff) {  // the single-GPU affine form: the dense copy from the rows once per train call
    SWPS_TRY(l->d_wdense.ensure(V * 4));
    if (l->mirror_stale) {
      k_lr_mirror<<<nblk(V), 256, 0, s>>>(l->t->rows.as<float>(), (uint32_t)l->w1_base, V, l->d_wdense.as<float>());
      SWPS_HIP(hipGetLastError());
      l->mirror_stale = false;
    }
    l->pushed_in_place = true;
  } else if (shd) {  // the owners' pull values at the step's row layout; each key's position for the payload
    const uint64_t U = l->bU[bi];
    if (shd_dense) SWPS_TRY(l->d_wdense.ensure(V * 4));
    float *wc = shd_dense ? l->d_wdense.as<float>() : l->d_wcache2.as<float>();
    const uint32_t ws = shd_dense ? 1u : 2u;
    if (U && prow)
      k_lr_install_fx_rows<<<nblk(U), 256, 0, s>>>(l->d_K.as<int32_t>() + l->kofs[bi], U, prow,
                                                   l->t->rows.as<float>(), l->d_fx_fidv.as<uint32_t>(), wc, ws,
                                                   l->d_localf.as<uint32_t>());
    else if (U)
      k_lr_install_fx<<<nblk(U), 256, 0, s>>>(l->d_K.as<int32_t>() + l->kofs[bi], U, d_vals,
                                              l->d_fx_fidv.as<uint32_t>(), wc, ws, l->d_localf.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    l->pushed_in_place = prow != nullptr;
  }
  if (!l->fx_atomic) {
    const uint32_t nh = hot ? (uint32_t)l->fx_hot_vids.size() : 0u, grid = (uint32_t)std::min<uint64_t>(nfc, l->fxb_grid);
    const double scale = std::ldexp(1.0, l->fx_bits);
    hipEvent_t fb = l->timer.ext(), fe = l->timer.ext();
    const size_t dyn = (size_t)l->fxb_nbk * 4;
    // chunks of 4,096 records: 512 threads x 8 (default) or 256 x 16; of 2,048: 256 x 8
    const bool res = l->fxb_res;
    const int nt = l->fwd_rpt == 16 && l->fx_nt == 512 && !res ? 512 : 256, rpt = nt == 512 ? 8 : l->fwd_rpt;
    auto *kern = res ? (rpt == 16 ? (nh <= 512 ? (l->fx_affine ? k_lr_fxb_step<16, 256, true, 512, true>
                                                               : k_lr_fxb_step<16, 256, false, 512, true>)
                                               : (l->fx_affine ? k_lr_fxb_step<16, 256, true, kLrHot, true>
                                                               : k_lr_fxb_step<16, 256, false, kLrHot, true>))
                                  : (nh <= 512 ? (l->fx_affine ? k_lr_fxb_step<8, 256, true, 512, true>
                                                               : k_lr_fxb_step<8, 256, false, 512, true>)
                                               : (l->fx_affine ? k_lr_fxb_step<8, 256, true, kLrHot, true>
                                                               : k_lr_fxb_step<8, 256, false, kLrHot, true>)))
                 : nt == 512 ? (nh <= 512 ? (l->fx_affine ? k_lr_fxb_step<8, 512, true, 512, false>
                                                          : k_lr_fxb_step<8, 512, false, 512, false>)
                                          : (l->fx_affine ? k_lr_fxb_step<8, 512, true, kLrHot, false>
                                                          : k_lr_fxb_step<8, 512, false, kLrHot, false>))
                 : rpt == 16 ? (nh <= 512 ? (l->fx_affine ? k_lr_fxb_step<16, 256, true, 512, false>
                                                          : k_lr_fxb_step<16, 256, false, 512, false>)
                                          : (l->fx_affine ? k_lr_fxb_step<16, 256, true, kLrHot, false>
                                                          : k_lr_fxb_step<16, 256, false, kLrHot, false>))
                 : (nh <= 512 ? (l->fx_affine ? k_lr_fxb_step<8, 256, true, 512, false>
                                              : k_lr_fxb_step<8, 256, false, 512, false>)
                              : (l->fx_affine ? k_lr_fxb_step<8, 256, true, kLrHot, false>
                                              : k_lr_fxb_step<8, 256, false, kLrHot, false>));
    const bool mir = res && l->fx_affine && l->fxr && l->fx_mirror && !shd;
    if (mir && l->mirror_stale) {  // the dense weight copy from the rows (swps_lr_train_batches' start)
      SWPS_TRY(l->d_wmir.ensure(V * 4));
      k_lr_mirror<<<nblk(V), 256, 0, s>>>(l->t->rows.as<float>(), l->fx_row_base, V, l->d_wmir.as<float>());
      SWPS_HIP(hipGetLastError());
      l->mirror_stale = false;
    }
    if (res && l->fx_affine && l->fxr) {  // the branch-free form (bit-identical)
      // SWPS_LR_FX_NT=512 with 4,096-record chunks: 512 threads x 8 records (A/B)
      const bool w512 = l->fx_nt == 512 && l->fwd_rpt == 16;
      auto *kr = w512 ? (nh <= 512 ? k_lr_fxr_step<8, 512, 512> : k_lr_fxr_step<8, 512, kLrHot>)
                 : rpt == 16 ? (nh <= 512 ? k_lr_fxr_step<16, 256, 512> : k_lr_fxr_step<16, 256, kLrHot>)
                             : (nh <= 512 ? k_lr_fxr_step<8, 256, 512> : k_lr_fxr_step<8, 256, kLrHot>);
      hipExtLaunchKernelGGL(kr, dim3(grid), dim3(w512 ? 512 : 256), (size_t)(l->fxb_nbk + kLrFxDummy) * 4, s, fb, fe, 0,
                            (const uint2 *)l->d_fchunk.as<uint2>() + l->bfchunk[bi], (uint32_t)nfc,
                            (const uint64_t *)l->d_row_off.as<uint64_t>(), (const int32_t *)l->d_ffid.as<int32_t>(),
                            (const float *)l->d_fval.as<float>(), (const float *)l->d_label.as<float>(), r0,
                            (const float *)(shd ? l->d_wcache2.as<float>() : l->t->rows.as<float>()),
                            hot ? nh : 0u, l->d_err.as<float>(), l->d_err2.as<float>(), scale, l->fxb_nbk,
                            l->d_fxb_rec.as<uint2>(), l->d_fxb_hsum.as<unsigned long long>(),
                            l->d_fxb_hcnt.as<uint32_t>(), l->fx_row_base, l->d_fxb_fill.as<uint32_t>(),
                            (const uint32_t *)l->d_fxb_rbase.as<uint32_t>(), l->fxb_gbits,
                            shd_dense ? (const float *)l->d_wdense.as<float>()
                            : mir     ? (const float *)l->d_wmir.as<float>()
                                      : (const float *)nullptr,
                            l->fxb_diag);
    } else
    hipExtLaunchKernelGGL(kern, dim3(grid), dim3(nt), dyn, s, fb, fe, 0,
                          (const uint2 *)l->d_fchunk.as<uint2>() + l->bfchunk[bi], (uint32_t)nfc,
                          (const uint64_t *)l->d_row_off.as<uint64_t>(),
                          (const int32_t *)(l->fx_affine ? l->d_ffid.as<int32_t>() : l->d_fvid.as<int32_t>()),
                          (const uint32_t *)l->d_vcode.as<uint32_t>(), (const float *)l->d_fval.as<float>(),
                          (const float *)l->d_label.as<float>(), r0,
                          (const float *)(shd ? l->d_wcache2.as<float>() : l->t->rows.as<float>()),
                          hot ? (const uint32_t *)l->d_fx_hrow.as<uint32_t>() : (const uint32_t *)nullptr, nh,
                          l->d_err.as<float>(), l->d_err2.as<float>(), scale, l->fxb_nbk, l->d_fxb_rec.as<uint2>(),
                          l->d_fxb_boff.as<uint16_t>(), (uint32_t)l->max_bchunks, l->d_fxb_hsum.as<unsigned long long>(),
                          l->d_fxb_hcnt.as<uint32_t>(), l->fx_row_base, l->d_fxb_fill.as<uint32_t>(),
                          (const uint32_t *)l->d_fxb_rbase.as<uint32_t>(), l->fxb_gbits, l->fxb_diag);
    l->timer.ext_end(0, fb, fe);
    hipEvent_t ab = l->timer.ext(), ae = l->timer.ext();
    // SWPS_LR_FXB_DIAG (timing experiments only; results wrong): 1 buckets only, 2 hot keys only,
    // 4 no record scatter, 8 no hot partials, 16 buckets without the row updates, 32 buckets
    // without their records, 64 no hot-key LDS sums, 128 no bucket sort, 256 no region reservation
    const uint32_t bper = l->fxb_xcd ? (l->fxb_nbk + 7u) / 8u : 0u, nbb = bper ? 8u * bper : l->fxb_nbk;
    const uint32_t pb0 = (l->fxb_diag & 2u) ? nbb : 0u,
                   pb1 = (l->fxb_diag & 1u) ? nbb : nbb + (nh + kLrFxbHotK - 1) / kLrFxbHotK;
    if (w1aff) {  // world 1, rows by fid: the single-GPU push (affine rows, prefetch, dense copy kept)
      hipExtLaunchKernelGGL(res ? k_lr_fxb_push<false, true> : k_lr_fxb_push<false, false>,
                            dim3(std::max(1u, pb1 - pb0)), dim3(kLrFxbPushT), res ? 0 : (2 * nfc + 1) * 4, s, ab,
                            ae, 0,
                            (const uint2 *)l->d_fxb_rec.as<uint2>(), (const uint16_t *)l->d_fxb_boff.as<uint16_t>(),
                            (const uint32_t *)l->d_fchunk_c0.as<uint32_t>() + l->bfchunk[bi], (uint32_t)nfc,
                            l->fxb_nbk, (uint32_t)l->max_bchunks, (const uint32_t *)l->d_localf.as<uint32_t>(),
                            (const unsigned long long *)l->d_fxb_hsum.as<unsigned long long>(),
                            (const uint32_t *)l->d_fxb_hcnt.as<uint32_t>(), grid,
                            (const uint32_t *)l->d_w1_hrow.as<uint32_t>(), nh, l->t->rows.as<float>(),
                            l->t->cfg.learning_rate, l->t->cfg.fudge, scale, std::ldexp(1.0, -l->fx_bits), 1u,
                            (uint32_t)l->w1_base, pb0, bper, l->d_fxb_fill.as<uint32_t>(),
                            (const uint32_t *)l->d_fxb_rbase.as<uint32_t>(), (uint32_t)l->vocab_keys.size(),
                            l->fxb_gbits, l->d_wdense.as<float>(),
                            res && l->fx_pf != 2 ? (const uint8_t *)l->d_pfb.as<uint8_t>() : (const uint8_t *)nullptr,
                            l->fxb_diag);
      SWPS_HIP(hipGetLastError());
      l->timer.ext_end(3, ab, ae);
      return SWPS_OK;
    }
    if (prow) {  // world 1 in place: AdaGrad on the shard rows localf names (hot key q = fid q)
      hipExtLaunchKernelGGL(res ? k_lr_fxb_push<false, true> : k_lr_fxb_push<false, false>,
                            dim3(std::max(1u, pb1 - pb0)), dim3(kLrFxbPushT), res ? 0 : (2 * nfc + 1) * 4, s, ab,
                            ae, 0,
                            (const uint2 *)l->d_fxb_rec.as<uint2>(), (const uint16_t *)l->d_fxb_boff.as<uint16_t>(),
                            (const uint32_t *)l->d_fchunk_c0.as<uint32_t>() + l->bfchunk[bi], (uint32_t)nfc,
                            l->fxb_nbk, (uint32_t)l->max_bchunks, (const uint32_t *)l->d_localf.as<uint32_t>(),
                            (const unsigned long long *)l->d_fxb_hsum.as<unsigned long long>(),
                            (const uint32_t *)l->d_fxb_hcnt.as<uint32_t>(), grid,
                            (const uint32_t *)l->d_localf.as<uint32_t>(), nh, l->t->rows.as<float>(),
                            l->t->cfg.learning_rate, l->t->cfg.fudge, scale, std::ldexp(1.0, -l->fx_bits), 0u, 0u,
                            pb0, bper, l->d_fxb_fill.as<uint32_t>(), (const uint32_t *)l->d_fxb_rbase.as<uint32_t>(),
                            (uint32_t)l->vocab_keys.size(), l->fxb_gbits, (float *)nullptr, (const uint8_t *)nullptr,
                            l->fxb_diag);
      SWPS_HIP(hipGetLastError());
      l->timer.ext_end(3, ab, ae);
      return SWPS_OK;
    }
    hipExtLaunchKernelGGL(shd ? (res ? k_lr_fxb_push<true, true> : k_lr_fxb_push<true, false>)
                              : (res ? k_lr_fxb_push<false, true> : k_lr_fxb_push<false, false>),
                          dim3(std::max(1u, pb1 - pb0)), dim3(kLrFxbPushT), res ? 0 : (2 * nfc + 1) * 4, s, ab,
                          ae, 0,
                          (const uint2 *)l->d_fxb_rec.as<uint2>(), (const uint16_t *)l->d_fxb_boff.as<uint16_t>(),
                          (const uint32_t *)l->d_fchunk_c0.as<uint32_t>() + l->bfchunk[bi], (uint32_t)nfc, l->fxb_nbk,
                          (uint32_t)l->max_bchunks,
                          (const uint32_t *)(shd ? l->d_localf.as<uint32_t>() : l->d_vid_row.as<uint32_t>()),
                          (const unsigned long long *)l->d_fxb_hsum.as<unsigned long long>(),
                          (const uint32_t *)l->d_fxb_hcnt.as<uint32_t>(), grid,
                          (const uint32_t *)l->d_fx_hrow.as<uint32_t>(), nh, shd ? d_grads : l->t->rows.as<float>(),
                          l->t->cfg.learning_rate, l->t->cfg.fudge, scale, std::ldexp(1.0, -l->fx_bits),
                          (uint32_t)l->fx_affine, l->fx_row_base, pb0, bper, l->d_fxb_fill.as<uint32_t>(),
                          (const uint32_t *)l->d_fxb_rbase.as<uint32_t>(), (uint32_t)l->vocab_keys.size(),
                          l->fxb_gbits, mir ? l->d_wmir.as<float>() : (float *)nullptr,
                          res && l->fx_pf != 2 ? (const uint8_t *)l->d_pfb.as<uint8_t>() : (const uint8_t *)nullptr,
                          l->fxb_diag);
    SWPS_HIP(hipGetLastError());
    l->timer.ext_end(3, ab, ae);
    return SWPS_OK;
  }
  uint32_t *cur = l->d_fx_n.as<uint32_t>() + (step & 1), *next = l->d_fx_n.as<uint32_t>() + ((step + 1) & 1);
  hipEvent_t fb = l->timer.ext(), fe = l->timer.ext();
  hipExtLaunchKernelGGL(l->fwd_rpt == 16 ? k_lr_fx_step<16> : k_lr_fx_step<8>, dim3((unsigned)nfc), dim3(256), 0, s, fb,
                        fe, 0,
                        (const uint2 *)l->d_fchunk.as<uint2>() + l->bfchunk[bi],
                        (const uint64_t *)l->d_row_off.as<uint64_t>(), (const int32_t *)l->d_fvid.as<int32_t>(),
                        (const uint32_t *)l->d_vcode.as<uint32_t>(), (const float *)l->d_fval.as<float>(),
                        (const float *)l->d_label.as<float>(), r0, (const float *)l->t->rows.as<float>(),
                        hot ? (const uint32_t *)l->d_fx_hrow.as<uint32_t>() : (const uint32_t *)nullptr,
                        hot ? (uint32_t)l->fx_hot_vids.size() : 0u, l->d_err.as<float>(), l->d_err2.as<float>(),
                        l->d_acc_sum.as<unsigned long long>(), l->d_acc_cnt.as<uint32_t>(),
                        l->d_fx_list.as<uint32_t>(), cur, std::ldexp(1.0, l->fx_bits),
                        l->d_fx_stamp.as<uint32_t>(), ++l->fx_tag ? l->fx_tag : ++l->fx_tag);
  l->timer.ext_end(0, fb, fe);
  hipEvent_t ab = l->timer.ext(), ae = l->timer.ext();
  hipExtLaunchKernelGGL(k_lr_fx_apply, dim3(512), dim3(256), 0, s, ab, ae, 0, (const uint32_t *)l->d_fx_list.as<uint32_t>(),
                        (const uint32_t *)cur, next, l->d_acc_sum.as<unsigned long long>(), l->d_acc_cnt.as<uint32_t>(),
                        l->t->rows.as<float>(), l->t->cfg.learning_rate, l->t->cfg.fudge, std::ldexp(1.0, -l->fx_bits));
  SWPS_HIP(hipGetLastError());
  l->timer.ext_end(3, ab, ae);
  return SWPS_OK;
}

int lr_plan_setup(swps_lr *l) {
  const uint64_t n = std::max<uint64_t>(l->max_bnnz, 1), V = std::max<uint64_t>(l->vocab_keys.size(), 1);
  const uint64_t B1 = l->B1(), ntile = (B1 + (1ULL << l->tile_bits) - 1) >> l->tile_bits;
  int vb = 1;
  while ((1ULL << vb) < V) vb++;
  l->plan_vbits = vb;
  int tbits = 1;
  while ((1ULL << tbits) < ntile) tbits++;
  if (const char *e = getenv("SWPS_LR_PLAN_SORT")) l->plan_sort = atoi(e);  // tile shape of the plan's sorts (A/B)
  if (!l->ps) SWPS_HIP(hipStreamCreateWithFlags(&l->ps, hipStreamNonBlocking));
  for (auto &p : l->pslot) {
    if (!p.ready) SWPS_HIP(hipEventCreateWithFlags(&p.ready, hipEventDisableTiming));
    if (!p.used) SWPS_HIP(hipEventCreateWithFlags(&p.used, hipEventDisableTiming));
    SWPS_TRY(p.fcode.ensure(n * 4));
    SWPS_TRY(p.hrow.ensure(kLrHot * 4));
    SWPS_TRY(p.trow.ensure(n * 2 + 16));
    SWPS_TRY(p.tval.ensure(n * 4 + 16));
    SWPS_TRY(p.tinfo.ensure(n * 4));
    SWPS_TRY(p.tdst.ensure(n * 4));
    SWPS_TRY(p.ms.ensure(n * 16));
    SWPS_TRY(p.msrow.ensure(n * 4));
    SWPS_TRY(p.ml.ensure(n * 16));
    SWPS_TRY(p.mlrow.ensure(n * 4));
    SWPS_TRY(p.cnt.ensure(16));
    SWPS_TRY(p.chunk.ensure((ntile + n / l->tile_chunk + 1) * 5 * 4));  // blocks: <= tiles + records / chunk
  }
  for (DevMem *m : {&l->p_ks1, &l->p_permK, &l->p_tkey, &l->p_tks, &l->p_val2, &l->p_v2s, &l->p_rowK, &l->p_ph,
                    &l->p_pidT, &l->p_invT, &l->p_kstart, &l->p_kwhole, &l->p_krow, &l->p_khot})
    SWPS_TRY(m->ensure(n * 4));
  SWPS_TRY(l->p_packed.ensure(n * 8));
  SWPS_TRY(l->p_pk.ensure(n * 8));
  SWPS_TRY(l->p_hist.ensure(kPlanHotBins * 4));
  SWPS_TRY(l->p_thr.ensure(16));
  SWPS_TRY(l->p_tfirst.ensure(ntile * 4 + 4));
  // the row of every record (the CSR expanded once, like row_off itself)
  const uint64_t nr = l->label.size(), N = l->row_off[nr];
  SWPS_TRY(l->d_rid.ensure(std::max<uint64_t>(N, 1) * 4));
  k_lr_rowid<<<nblk(nr), 256, 0, l->s>>>(l->d_row_off.as<uint64_t>(), nr, l->d_rid.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  // temporary storage for the largest of the plan's sorts and scans (sized once: a grow inside a
  // step would free memory the other stream may still use)
  size_t b = 0, mx = 0;
  const rocprim::counting_iterator<uint32_t> iota(0u);
  SWPS_HIP(sort_pairs_tiled(l->plan_sort, nullptr, b, l->p_ks1.as<uint32_t>(), l->p_ks1.as<uint32_t>(), iota,
                            l->p_permK.as<uint32_t>(), n, vb, l->ps));
  mx = std::max(mx, b);
  b = 0;
  SWPS_HIP(sort_pairs_tiled(l->plan_sort, nullptr, b, l->p_tkey.as<uint32_t>(), l->p_tks.as<uint32_t>(),
                            (const uint32_t *)l->p_val2.as<uint32_t>(), l->p_v2s.as<uint32_t>(), n, tbits, l->ps));
  mx = std::max(mx, b);
  b = 0;
  SWPS_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, b, l->p_ph.as<uint32_t>(), l->p_pidT.as<uint32_t>(), (int)n,
                                            l->ps));
  mx = std::max(mx, b);
  b = 0;
  SWPS_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, b, l->p_packed.as<uint64_t>(), l->p_pk.as<uint64_t>(), (int)n,
                                            l->ps));
  mx = std::max(mx, b);
  SWPS_TRY(l->p_tmp.ensure(mx));
  SWPS_TRY(l->d_tpart.ensure(n * 8));
  SWPS_HIP(hipDeviceSynchronize());  // the allocations above precede every plan
  l->plan_ready = true;
  return SWPS_OK;
}

// the plan of training step `step` (batch step % nbatches) into slot step & 1, on the plan stream
int lr_plan(swps_lr *l, uint64_t step) {
  swps_lr::PlanSlot &p = l->pslot[step & 1];
  const uint64_t nr = l->label.size(), bi = step % l->nbatches, B1 = l->B1();
  const uint64_t r0 = bi * B1, r1 = std::min<uint64_t>(nr, r0 + B1), nrb = r1 - r0;
  const uint64_t z0 = l->row_off[r0], n = l->row_off[r1] - z0;
  const int tb = l->tile_bits;
  const uint32_t chunk = l->tile_chunk;
  const uint64_t ntile = (nrb + (1ULL << tb) - 1) >> tb;
  hipStream_t P = l->ps;
  if (p.pending_use) SWPS_HIP(hipStreamWaitEvent(P, p.used, 0));  // its reader, step - 2, is done
  p.pending_use = false;
  if (l->plan_sync) {  // the plan reads the shard rows of the vids (swps_lr_init, compute stream)
    if (!l->ev_rows) SWPS_HIP(hipEventCreateWithFlags(&l->ev_rows, hipEventDisableTiming));
    SWPS_HIP(hipEventRecord(l->ev_rows, l->s));
    SWPS_HIP(hipStreamWaitEvent(P, l->ev_rows, 0));
    l->plan_sync = false;
  }
  p.nch = 0;
  for (uint64_t tl = 0; tl < ntile; tl++) {  // the tiles launch's grid (host: the batch's CSR offsets)
    const uint64_t rs = r0 + (tl << tb), re = r0 + std::min<uint64_t>(nrb, (tl + 1) << tb);
    p.nch += (l->row_off[re] - l->row_off[rs] + chunk - 1) / chunk;
  }
  hipEvent_t e0 = l->timer.begin(P);
  if (n) {
    int tbits = 1;
    while ((1ULL << tbits) < ntile) tbits++;
    uint32_t *ks1 = l->p_ks1.as<uint32_t>(), *permK = l->p_permK.as<uint32_t>();
    uint32_t *tkey = l->p_tkey.as<uint32_t>(), *val2 = l->p_val2.as<uint32_t>(), *v2s = l->p_v2s.as<uint32_t>();
    uint32_t *ph = l->p_ph.as<uint32_t>(), *pidT = l->p_pidT.as<uint32_t>(), *invT = l->p_invT.as<uint32_t>();
    uint64_t *packed = l->p_packed.as<uint64_t>(), *pk = l->p_pk.as<uint64_t>();
    const bool hot = l->hot != 0;
    k_plan_reset<<<1, 1024, 0, P>>>(l->d_row_off.as<uint64_t>(), r0, nrb, tb, chunk, ntile,
                                    l->p_tfirst.as<uint32_t>(), p.cnt.as<uint32_t>(), l->p_hist.as<uint32_t>(),
                                    p.hrow.as<uint32_t>(), hot ? (uint32_t)kLrHot : 0u);
    SWPS_HIP(hipGetLastError());
    const rocprim::counting_iterator<uint32_t> iota(0u);
    size_t b = l->p_tmp.bytes;  // K order: the batch's records stable by vid, straight from the CSR
    SWPS_HIP(sort_pairs_tiled(l->plan_sort, l->p_tmp.p, b, (const uint32_t *)(l->d_fvid.as<int32_t>() + z0), ks1,
                              iota, permK, n, l->plan_vbits, P));
    k_plan_tile<<<nblk(n), 256, 0, P>>>(permK, ks1, l->d_rid.as<uint32_t>(), z0, r0, n, tb, tkey, val2,
                                         l->p_rowK.as<uint32_t>());
    b = l->p_tmp.bytes;  // T order: K order stable by tile
    SWPS_HIP(sort_pairs_tiled(l->plan_sort, l->p_tmp.p, b, (const uint32_t *)tkey, l->p_tks.as<uint32_t>(),
                              (const uint32_t *)val2, v2s, n, tbits, P));
    k_plan_torder<<<nblk(n), 256, 0, P>>>(v2s, l->p_tks.as<uint32_t>(), l->p_rowK.as<uint32_t>(), permK,
                                           l->d_fval.as<float>(), l->d_row_off.as<uint64_t>(), r0, z0, n, tb, chunk,
                                           p.trow.as<uint16_t>(), p.tval.as<float>(), ph, invT);
    SWPS_HIP(hipGetLastError());
    b = l->p_tmp.bytes;
    SWPS_HIP(hipcub::DeviceScan::InclusiveSum(l->p_tmp.p, b, ph, pidT, (int)n, P));
    k_plan_kflags<<<nblk(n), 256, 0, P>>>(ks1, invT, ph, n, packed);
    b = l->p_tmp.bytes;
    SWPS_HIP(hipcub::DeviceScan::InclusiveSum(l->p_tmp.p, b, packed, pk, (int)n, P));
    k_plan_kstart<<<nblk(n), 256, 0, P>>>(pk, n, l->p_kstart.as<uint32_t>());
    const unsigned kg = std::min<unsigned>(nblk(n), 512);
    k_plan_kinfo<<<kg, 256, 0, P>>>(l->p_kstart.as<uint32_t>(), pk, n, ks1, l->d_vid_row.as<uint32_t>(),
                                     l->p_kwhole.as<uint32_t>(), l->p_krow.as<uint32_t>(), (uint4 *)p.ms.p,
                                     p.msrow.as<uint32_t>(), (uint4 *)p.ml.p, p.mlrow.as<uint32_t>(),
                                     p.cnt.as<uint32_t>(), hot ? l->p_hist.as<uint32_t>() : nullptr);
    if (hot) {
      k_plan_hot_thresh<<<1, 64, 0, P>>>(l->p_hist.as<uint32_t>(), l->nhot, l->p_thr.as<uint32_t>());
      k_plan_hot_assign<<<kg, 256, 0, P>>>(l->p_kstart.as<uint32_t>(), pk, n, l->p_krow.as<uint32_t>(), l->nhot,
                                            l->p_thr.as<uint32_t>(), l->p_khot.as<int32_t>(), p.hrow.as<uint32_t>());
    }
    k_plan_records<<<nblk(n), 256, 0, P>>>(pk, permK, invT, pidT, n, l->p_kwhole.as<uint32_t>(),
                                            l->p_krow.as<uint32_t>(), hot ? l->p_khot.as<int32_t>() : nullptr,
                                            p.fcode.as<uint32_t>(), p.tinfo.as<uint32_t>(), p.tdst.as<uint32_t>());
    k_plan_chunks<<<nblk(p.nch), 256, 0, P>>>(l->d_row_off.as<uint64_t>(), r0, nrb, z0, tb, chunk, ntile,
                                               l->p_tfirst.as<uint32_t>(), pidT, n, p.nch, p.chunk.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
  }
  l->timer.end(1, e0, P);
  SWPS_HIP(hipEventRecord(p.ready, P));
  return SWPS_OK;
}

// one training step from its plan (the static index's kernels, fed by the plan's slot), then the
// next step's plan on the plan stream while this one trains
int lr_batch_planned(swps_lr *l) {
  if (!l->plan_ready) SWPS_TRY(lr_plan_setup(l));
  const uint64_t step = l->cursor, nr = l->label.size(), bi = step % l->nbatches;
  const uint64_t r0 = bi * l->B1(), r1 = std::min<uint64_t>(nr, r0 + l->B1()), nrb = r1 - r0;
  const uint64_t z0 = l->row_off[r0], nnz = l->row_off[r1] - z0;
  hipStream_t s = l->s;
  if (l->plan_next <= step) {
    SWPS_TRY(lr_plan(l, step));
    l->plan_next = step + 1;
  }
  swps_lr::PlanSlot &p = l->pslot[step & 1];
  l->cursor++;
  SWPS_HIP(hipStreamWaitEvent(s, p.ready, 0));
  if (nnz) {
    const uint64_t nfc = l->bfchunk[bi + 1] - l->bfchunk[bi];
    hipEvent_t fb = l->timer.ext(), fe = l->timer.ext();
    const bool hot = l->hot != 0;
    auto kc = l->fwd_rpt == 4 ? k_lr_forward_c<4> : l->fwd_rpt == 16 ? k_lr_forward_c<16> : k_lr_forward_c<kLrFwdRpt>;
    hipExtLaunchKernelGGL(kc, dim3((unsigned)nfc), dim3(256), 0, s, fb, fe, 0,
                          (const uint2 *)l->d_fchunk.as<uint2>() + l->bfchunk[bi],
                          (const uint64_t *)l->d_row_off.as<uint64_t>(),
                          (const uint32_t *)(p.fcode.as<uint32_t>() - z0), (const float *)l->d_fval.as<float>(),
                          (const float *)l->d_label.as<float>(), r0, (const float *)l->t->rows.as<float>(), 2,
                          l->d_err.as<float>(), l->d_err2.as<float>(),
                          hot ? (const uint32_t *)p.hrow.as<uint32_t>() : (const uint32_t *)nullptr,
                          hot ? l->nhot : 0u);
    l->timer.ext_end(0, fb, fe);
    LrReduce ra{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, l->t->rows.as<float>(),
                l->t->cfg.learning_rate, l->t->cfg.fudge, nullptr, nullptr, nullptr, nullptr, 1,
                nullptr, nullptr, l->d_err.as<float>()};
    LrTiles tt{p.trow.as<uint16_t>(), p.tval.as<float>(), p.chunk.as<uint32_t>(), p.tinfo.as<uint32_t>(),
               p.tdst.as<uint32_t>(), l->d_tpart.as<double>(), l->d_err.as<float>(), r0, nrb, l->tile_bits, 0};
    hipEvent_t tb0 = l->timer.ext(), te0 = l->timer.ext(), tb1 = l->timer.ext(), te1 = l->timer.ext();
    auto kt = l->tile_chunk == 512    ? k_lr_tiles<2>
              : l->tile_chunk == 1024 ? k_lr_tiles<4>
              : l->tile_chunk == 1280 ? k_lr_tiles<5>
              : l->tile_chunk == 1536 ? k_lr_tiles<6>
              : l->tile_chunk == 1792 ? k_lr_tiles<7>
              : l->tile_chunk == 4096 ? k_lr_tiles<16>
                                      : k_lr_tiles<8>;
    if (p.nch) hipExtLaunchKernelGGL(kt, dim3((unsigned)p.nch), dim3(256), 0, s, tb0, te0, 0, ra, tt);
    // the finisher's counts live on the device: LB blocks stride over the long keys, the rest
    // over the short ones
    const uint32_t LB = 256, SB = 512;
    hipExtLaunchKernelGGL(k_lr_tiles_fin, dim3(LB + SB), dim3(256), 0, s, p.nch ? tb1 : tb0, p.nch ? te1 : te0, 0, ra,
                          (const uint4 *)p.ms.p, (const uint32_t *)p.msrow.as<uint32_t>(), 0u, (const uint4 *)p.ml.p,
                          (const uint32_t *)p.mlrow.as<uint32_t>(), 0u, LB, (const double *)l->d_tpart.as<double>(),
                          (uint64_t)0, (const uint32_t *)p.cnt.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    l->timer.ext_end(3, tb0, te0);
    if (p.nch) {
      l->timer.ext_more(3, tb1, te1);
    } else if (tb1) {
      (void)hipEventDestroy(tb1);
      (void)hipEventDestroy(te1);
    }
  }
  SWPS_HIP(hipEventRecord(p.used, s));
  p.pending_use = true;
  if (l->plan_next == step + 1) {  // the next step's plan, beside this step
    SWPS_TRY(lr_plan(l, step + 1));
    l->plan_next = step + 2;
  }
  return SWPS_OK;
}

int lr_batch(swps_lr *l, const float *d_vals = nullptr, float *d_grads = nullptr) {
  if (!l->sharded) {
    SWPS_TRY(lr_fwd_chunks(l));
    if (lr_fx_usable(l)) return lr_batch_fx(l);
    if (lr_plan_usable(l)) return lr_batch_planned(l);
  } else if (l->fx_sharded) {
    return lr_batch_fx(l, d_vals, d_grads);
  }
  if (!l->index_built) SWPS_TRY(lr_index(l));  // the static per-batch index, built once
  const uint64_t nr = l->label.size();
  const uint64_t bi = l->cursor % l->nbatches;
  const uint64_t r0 = bi * l->B1(), r1 = std::min<uint64_t>(nr, r0 + l->B1());
  const uint64_t nz0 = l->row_off[r0], nnz = l->row_off[r1] - nz0;
  hipStream_t s = l->s;
  float *rows = l->t->rows.as<float>();
  const uint32_t *fidx = l->d_frow.as<uint32_t>();
  int stride = 2;
  l->cursor++;
  if (l->sharded) {  // install the owners' pull values; read weights from the cache
    const uint64_t U = l->bU[bi];
    if (U)
      k_lr_install<<<nblk(U), 256, 0, s>>>(l->d_K.as<int32_t>() + l->kofs[bi], U, d_vals, l->d_wcache.as<float>(),
                                           l->d_local.as<int32_t>(), 1);
    SWPS_HIP(hipGetLastError());
    rows = l->d_wcache.as<float>();
    fidx = (const uint32_t *)l->d_fvid.as<int32_t>();
    stride = 1;
  } else if (!l->rows_mapped) {  // the shard rows of every record's feature and every run's key, once
    const uint64_t n = l->row_off[nr], R = l->brun[l->nbatches];
    SWPS_TRY(l->d_frow.ensure(std::max<uint64_t>(n, 1) * 4));
    SWPS_TRY(l->d_urow.ensure(std::max<uint64_t>(R, 1) * 4));
    k_lr_map_rows<<<nblk(n), 256, 0, s>>>(l->d_fvid.as<int32_t>(), n, l->d_vid_row.as<uint32_t>(),
                                          l->d_frow.as<uint32_t>());
    k_lr_map_rows<<<nblk(R), 256, 0, s>>>((const int32_t *)l->d_ruk.as<uint32_t>(), R, l->d_vid_row.as<uint32_t>(),
                                          l->d_urow.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    if (l->hot && !l->bnhot.empty()) {
      SWPS_TRY(l->d_fhot.ensure(std::max<uint64_t>(n, 1) * 4));
      SWPS_TRY(l->d_hrow.ensure(std::max<uint64_t>(l->nbatches, 1) * kLrHot * 4));
      k_lr_hot_codes<<<nblk(n), 256, 0, s>>>(l->d_frun.as<uint32_t>(), l->d_hot_of_run.as<int32_t>(),
                                              l->d_frow.as<uint32_t>(), n, l->d_fhot.as<uint32_t>());
      k_lr_hot_rows<<<nblk(l->nbatches * kLrHot), 256, 0, s>>>(l->d_hgrun.as<uint32_t>(), l->nbatches * kLrHot,
                                                                l->d_urow.as<uint32_t>(), l->d_hrow.as<uint32_t>());
    }
    if (l->tiles_ready && l->tile_npieces)
      k_lr_tile_dst<<<nblk(l->tile_npieces), 256, 0, s>>>(l->d_tinfo.as<uint32_t>(), l->d_tslot.as<uint32_t>(),
                                                           l->d_tgrun.as<uint32_t>(), l->tile_npieces,
                                                           l->d_urow.as<uint32_t>(), l->d_tdst.as<uint32_t>());
    if (l->tiles_ready) {
      const uint64_t nms = l->bmulti[l->nbatches], nml = l->bmlong[l->nbatches];
      if (nms)
        k_lr_tile_mrow<<<nblk(nms), 256, 0, s>>>((const uint4 *)l->d_tmulti.p, nms, l->d_urow.as<uint32_t>(),
                                                  l->d_tmsrow.as<uint32_t>());
      if (nml)
        k_lr_tile_mrow<<<nblk(nml), 256, 0, s>>>((const uint4 *)l->d_tmlong.p, nml, l->d_urow.as<uint32_t>(),
                                                  l->d_tmlrow.as<uint32_t>());
    }
    SWPS_HIP(hipGetLastError());
    l->rows_mapped = true;
    fidx = l->d_frow.as<uint32_t>();
  }
  if (nnz == 0) return SWPS_OK;
  SWPS_TRY(l->d_longs.ensure((l->max_bnnz + 1) * 4));
  hipEvent_t e0 = l->timer.begin(s);
  const uint64_t nrb = r1 - r0;
  const uint32_t mf = l->bmaxf[bi];  // the batch's longest row
  SWPS_TRY(l->d_val_s.ensure((l->max_bnnz + 4) * 4));
  const bool scat = l->fwd_records && l->rows_per_wave == 1 && mf <= 64;  // the forward writes the records
  if (!scat) SWPS_TRY(lr_fwd_chunks(l));
  const uint64_t nfc = l->fwd_c && l->bfchunk.size() > bi + 1 ? l->bfchunk[bi + 1] - l->bfchunk[bi] : 0;
  if (nfc && !scat && l->rows_per_wave == 1 && !l->fwd_diag && !l->stage) {  // record-contiguous chunks of rows
    hipEvent_t fb = l->timer.ext(), fe = l->timer.ext();
    const bool hot = l->hot && !l->sharded && !l->bnhot.empty() && l->bnhot[bi];
    auto kc = l->fwd_rpt == 4 ? k_lr_forward_c<4> : l->fwd_rpt == 16 ? k_lr_forward_c<16> : k_lr_forward_c<kLrFwdRpt>;
    hipExtLaunchKernelGGL(kc, dim3((unsigned)nfc), dim3(256), 0, s, fb, fe, 0,
                          (const uint2 *)l->d_fchunk.as<uint2>() + l->bfchunk[bi],
                          (const uint64_t *)l->d_row_off.as<uint64_t>(), hot ? l->d_fhot.as<uint32_t>() : fidx,
                          (const float *)l->d_fval.as<float>(), (const float *)l->d_label.as<float>(), r0,
                          (const float *)rows, stride, l->d_err.as<float>(), l->d_err2.as<float>(),
                          hot ? (const uint32_t *)(l->d_hrow.as<uint32_t>() + bi * kLrHot) : (const uint32_t *)nullptr,
                          hot ? l->bnhot[bi] : 0u);
    l->timer.ext_end(0, fb, fe);
    if (fb) (void)hipEventDestroy(e0);
    e0 = nullptr;
  } else if (!scat && l->rows_per_wave == 1 && mf <= 42 && l->fwd_groups > 1 && !l->fwd_diag) {  // G groups per wave
    hipEvent_t fb = l->timer.ext(), fe = l->timer.ext();
    auto kf = l->fwd_groups == 4 ? k_lr_forward_g<3, 4> : k_lr_forward_g<3, 2>;
    const uint64_t G = l->fwd_groups == 4 ? 4 : 2;
    const float *fw = rows;
    const uint32_t *fi = fidx;
    int fs = stride;
    const uint32_t nruns = (uint32_t)(l->brun[bi + 1] - l->brun[bi]);
    if (l->stage && !l->sharded && nruns) {  // the batch's weights staged densely (stamped with the forward)
      SWPS_TRY(l->d_wstage.ensure((uint64_t)l->max_bruns * 4));
      hipExtLaunchKernelGGL(k_lr_stage, dim3(nblk(nruns)), dim3(256), 0, s, fb, (hipEvent_t) nullptr, 0,
                            (const uint32_t *)(l->d_urow.as<uint32_t>() + l->brun[bi]), nruns, (const float *)rows,
                            l->d_wstage.as<float>());
      fw = l->d_wstage.as<float>() - l->brun[bi];  // indexed by the records' global run
      fi = l->d_frun.as<uint32_t>();
      fs = 1;
    }
    const bool hot = l->hot && !l->sharded && !(l->stage && nruns) && !l->bnhot.empty() && l->bnhot[bi];
    if (hot) fi = l->d_fhot.as<uint32_t>();
    hipExtLaunchKernelGGL(kf, dim3((unsigned)nblk((nrb + 3 * G - 1) / (3 * G) * 64)), dim3(256), 0, s,
                          l->stage && !l->sharded && nruns ? (hipEvent_t) nullptr : fb, fe, 0,
                          (const uint64_t *)l->d_row_off.as<uint64_t>(), fi, (const float *)l->d_fval.as<float>(),
                          (const float *)l->d_label.as<float>(), r0, nrb, fw, fs, l->d_err.as<float>(),
                          l->d_err2.as<float>(),
                          hot ? (const uint32_t *)(l->d_hrow.as<uint32_t>() + bi * kLrHot) : (const uint32_t *)nullptr,
                          hot ? l->bnhot[bi] : 0u);
    l->timer.ext_end(0, fb, fe);
    if (fb) (void)hipEventDestroy(e0);
    e0 = nullptr;
  } else if (!scat && l->rows_per_wave == 1 && mf <= 42) {  // its own start / end stamps when profiled
    hipEvent_t fb = l->timer.ext(), fe = l->timer.ext();
    hipExtLaunchKernelGGL(k_lr_forward_r<3, true>, dim3((unsigned)nblk((nrb + 2) / 3 * 64)), dim3(256), 0, s, fb, fe, 0,
                          (const uint64_t *)l->d_row_off.as<uint64_t>(), fidx, (const float *)l->d_fval.as<float>(),
                          (const float *)l->d_label.as<float>(), r0, nrb, (const float *)rows, stride,
                          l->d_err.as<float>(), l->d_err2.as<float>(), l->fwd_diag & 3, (const uint32_t *)nullptr, (uint64_t)0,
                          (float *)nullptr);
    l->timer.ext_end(0, fb, fe);
    if (fb) (void)hipEventDestroy(e0);
    e0 = nullptr;
  } else if (scat && mf <= 42)  // 3 rows per wave, the ordered sums through LDS, records scattered (default)
    k_lr_forward_r<3, true, true><<<nblk((nrb + 2) / 3 * 64), 256, 0, s>>>(
        l->d_row_off.as<uint64_t>(), fidx, l->d_fval.as<float>(), l->d_label.as<float>(), r0, nrb, rows, stride,
        l->d_err.as<float>(), l->d_err2.as<float>(), 0, l->d_spos.as<uint32_t>(), nz0, l->d_val_s.as<float>());
  else if (scat)
    k_lr_forward_r<2, true, true><<<nblk((nrb + 1) / 2 * 64), 256, 0, s>>>(
        l->d_row_off.as<uint64_t>(), fidx, l->d_fval.as<float>(), l->d_label.as<float>(), r0, nrb, rows, stride,
        l->d_err.as<float>(), l->d_err2.as<float>(), 0, l->d_spos.as<uint32_t>(), nz0, l->d_val_s.as<float>());
  else if (l->rows_per_wave == 1 && mf <= 42)  // the same without the records (k_lr_records forms them)
    k_lr_forward_r<3, true><<<nblk((nrb + 2) / 3 * 64), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), fidx,
                                                                      l->d_fval.as<float>(), l->d_label.as<float>(),
                                                                      r0, nrb, rows, stride, l->d_err.as<float>(),
                                                                      l->d_err2.as<float>());
  else if (l->rows_per_wave == 1 && mf <= 64)
    k_lr_forward_r<2, true><<<nblk((nrb + 1) / 2 * 64), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), fidx,
                                                                      l->d_fval.as<float>(), l->d_label.as<float>(),
                                                                      r0, nrb, rows, stride, l->d_err.as<float>(),
                                                                      l->d_err2.as<float>());
  else if (l->rows_per_wave == 4)  // a lane per row
    k_lr_forward_l<40><<<(unsigned)((nrb + 63) / 64), 64, 0, s>>>(l->d_row_off.as<uint64_t>(), fidx,
                                                                  l->d_fval.as<float>(), l->d_label.as<float>(), r0,
                                                                  nrb, rows, stride, l->d_err.as<float>(),
                                                                  l->d_err2.as<float>());
  else if (l->rows_per_wave && mf <= 42 && l->rows_per_wave != 2)
    k_lr_forward_r<3><<<nblk((nrb + 2) / 3 * 64), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), fidx, l->d_fval.as<float>(),
                                                                l->d_label.as<float>(), r0, nrb, rows, stride,
                                                                l->d_err.as<float>(), l->d_err2.as<float>(),
                                                                l->fwd_diag);
  else if (l->rows_per_wave && mf <= 64)
    k_lr_forward_r<2><<<nblk((nrb + 1) / 2 * 64), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), fidx, l->d_fval.as<float>(),
                                                                l->d_label.as<float>(), r0, nrb, rows, stride,
                                                                l->d_err.as<float>(), l->d_err2.as<float>());
  else
    k_lr_forward<<<nblk(nrb * 64), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), fidx, l->d_fval.as<float>(),
                                                 l->d_label.as<float>(), r0, nrb, rows, stride, l->d_err.as<float>(),
                                                 l->d_err2.as<float>());
  SWPS_HIP(hipGetLastError());
  l->timer.end(0, e0, s);
  hipEvent_t e3 = l->timer.begin(s);
  // the run counter lives past the last possible long-run index
  uint32_t *nlong = l->d_longs.as<uint32_t>() + l->max_bnnz;
  const bool fused = l->cfg.fast_sums && l->fused_reduce && !l->blong.empty();
  if (!fused) SWPS_HIP(hipMemsetAsync(nlong, 0, 4, s));
  const uint64_t q0 = l->brun[bi];
  // the batch's records from val_s + (nz0 & 3): their 16-B groups line up with srow / sval's
  float *val = l->d_val_s.as<float>() + (scat ? 0 : (nz0 & 3));
  hipEvent_t pb = nullptr;  // the push group's start stamp (the records kernel's start)
  const bool inl = fused && !scat && l->inline_records;  // the reduce forms the records itself
  LrReduce ra{l->d_ruk.as<uint32_t>() + q0, l->d_rcnt.as<uint32_t>() + q0, l->d_roff.as<uint32_t>() + q0,
              l->d_bnruns.as<uint32_t>() + bi, val,
              l->sharded ? nullptr : l->d_urow.as<uint32_t>() + q0,
              l->t->rows.as<float>(), l->t->cfg.learning_rate, l->t->cfg.fudge, l->d_local.as<int32_t>(),
              l->sharded ? d_grads : nullptr, nlong, l->d_longs.as<uint32_t>(), l->cfg.fast_sums,
              l->d_srow.as<uint32_t>() + nz0, l->d_sval.as<float>() + nz0, l->d_err.as<float>()};
  if (l->cfg.fast_sums && l->tiles_ready && !scat && !l->inline_records) {  // row tiles (the default)
    const uint32_t nch = (uint32_t)(l->bchunk[bi + 1] - l->bchunk[bi]);
    const uint32_t nm = (uint32_t)(l->bmulti[bi + 1] - l->bmulti[bi]);
    LrTiles tt{l->d_trow.as<uint16_t>(), l->d_tval.as<float>(), l->d_tchunk.as<uint32_t>() + l->bchunk[bi] * 5,
               l->d_tinfo.as<uint32_t>(), (l->sharded ? l->d_tslot : l->d_tdst).as<uint32_t>(), l->d_tpart.as<double>(),
               l->d_err.as<float>(),
               r0, nrb, l->tile_bits, l->fwd_diag};
    // each kernel stamped by itself: the group's time is the sum of the two kernels' (not the span
    // from the first one's start to the second one's end, which holds the dispatch gap between them)
    hipEvent_t tb0 = l->timer.ext(), te0 = l->timer.ext(), tb1 = nullptr, te1 = nullptr;
    const bool fin = l->bmulti[bi + 1] > l->bmulti[bi] || l->bmlong[bi + 1] > l->bmlong[bi];
    if (nch && fin) {
      tb1 = l->timer.ext();
      te1 = l->timer.ext();
    }
    if (nch) {
      const bool b512 = l->tile_threads == 512;  // 4 records per thread, 512 threads: 2,048-record blocks
      auto kt = b512                    ? k_lr_tiles<4, 512>
                : l->tile_chunk == 512  ? k_lr_tiles<2>
                : l->tile_chunk == 1024 ? k_lr_tiles<4>
                : l->tile_chunk == 1280 ? k_lr_tiles<5>
                : l->tile_chunk == 1536 ? k_lr_tiles<6>
                : l->tile_chunk == 1792 ? k_lr_tiles<7>
                : l->tile_chunk == 4096 ? k_lr_tiles<16>
                                        : k_lr_tiles<8>;
      hipExtLaunchKernelGGL(kt, dim3(nch), dim3(b512 ? 512 : 256), 0, s, tb0, te0, 0, ra, tt);
    }
    const uint32_t nl = (uint32_t)(l->bmlong[bi + 1] - l->bmlong[bi]);
    if (nm || nl) {
      const uint32_t LB = std::min<uint32_t>((nl + 3) / 4, 1024);
      hipExtLaunchKernelGGL(k_lr_tiles_fin, dim3(LB + (nm ? nblk(nm) : 0)), dim3(256), 0, s,
                            nch ? tb1 : tb0, nch ? te1 : te0, 0, ra,
                            (const uint4 *)l->d_tmulti.p + l->bmulti[bi], (const uint32_t *)l->d_tmsrow.as<uint32_t>() + l->bmulti[bi], nm,
                            (const uint4 *)l->d_tmlong.p + l->bmlong[bi], (const uint32_t *)l->d_tmlrow.as<uint32_t>() + l->bmlong[bi], nl,
                            LB, (const double *)l->d_tpart.as<double>(), (uint64_t)q0, (const uint32_t *)nullptr);
    }
    SWPS_HIP(hipGetLastError());
    if (nch || fin) {
      l->timer.ext_end(3, tb0, te0);
      l->timer.ext_more(3, tb1, te1);
    } else if (tb0) {
      (void)hipEventDestroy(tb0);
      (void)hipEventDestroy(te0);
    }
    if (e3) (void)hipEventDestroy(e3);
    return SWPS_OK;
  }
  if (!scat && !inl) {
    pb = l->timer.ext();
    hipExtLaunchKernelGGL(k_lr_records, dim3((unsigned)(((nz0 + nnz + 3) / 4 - nz0 / 4 + 255) / 256)), dim3(256), 0, s,
                          pb, (hipEvent_t) nullptr, 0, (const uint32_t *)l->d_srow.as<uint32_t>(),
                          (const float *)l->d_sval.as<float>(), nz0, nz0 + nnz, (const float *)l->d_err.as<float>(),
                          val - (nz0 & 3), l->fwd_diag);
  }
  if (fused) {
    const uint32_t NL = (uint32_t)(l->blong[bi + 1] - l->blong[bi]);
    const uint32_t LB = std::min<uint32_t>(NL, 2048);
    const unsigned sblocks = (unsigned)std::min<uint64_t>(nblk(nnz), 4096);
    if (inl) {  // one kernel: stamped start and end
      hipEvent_t rb = l->timer.ext(), re = l->timer.ext();
      hipExtLaunchKernelGGL(k_lr_reduce_fused<true>, dim3(LB + sblocks), dim3(256), 0, s, rb, re, 0, ra,
                            (const uint32_t *)(l->d_slong.as<uint32_t>() + l->blong[bi]), NL, LB);
      SWPS_HIP(hipGetLastError());
      l->timer.ext_end(3, rb, re);
      if (e3) (void)hipEventDestroy(e3);
      return SWPS_OK;
    }
    if (pb) {  // records .. reduce, stamped by the kernels themselves
      hipEvent_t pe = l->timer.ext();
      hipExtLaunchKernelGGL(k_lr_reduce_fused<false>, dim3(LB + sblocks), dim3(256), 0, s, (hipEvent_t) nullptr, pe, 0,
                            ra, (const uint32_t *)(l->d_slong.as<uint32_t>() + l->blong[bi]), NL, LB);
      SWPS_HIP(hipGetLastError());
      l->timer.ext_end(3, pb, pe);
      if (e3) (void)hipEventDestroy(e3);
      return SWPS_OK;
    }
    k_lr_reduce_fused<false><<<LB + sblocks, 256, 0, s>>>(ra, l->d_slong.as<uint32_t>() + l->blong[bi], NL, LB);
    SWPS_HIP(hipGetLastError());
    l->timer.end(3, e3, s);
    return SWPS_OK;
  }
  if (pb) (void)hipEventDestroy(pb);  // exact mode: the stream events below
  k_lr_reduce_short<<<(unsigned)std::min<uint64_t>(nblk(nnz), 4096), 256, 0, s>>>(ra);
  if (l->cfg.fast_sums)
    k_lr_reduce_long_fast<<<(unsigned)std::min<uint64_t>(nblk(nnz * 256 / kLrShort), 4096), 256, 0, s>>>(ra);
  else
    k_lr_reduce_long<<<(unsigned)std::min<uint64_t>(nblk(nnz * 64 / kLrShort), 2048), 256, 0, s>>>(ra);
  SWPS_HIP(hipGetLastError());
  l->timer.end(3, e3, s);
  return SWPS_OK;
}

}  // namespace

extern "C" {

int swps_lr_create(swps_table *t, const swps_lr_cfg *cfg, swps_lr **out) {
  if (!t || !cfg || !out) return fail(SWPS_E_CFG, "null argument");
  *out = nullptr;
  if (t->cfg.layout != SWPS_LAYOUT_LR) return fail(SWPS_E_CFG, "table layout must be SWPS_LAYOUT_LR");
  SWPS_TRY(check_app_table(t));
  if (t->cfg.dtype != SWPS_F32) return fail(SWPS_E_UNSUPPORTED, "LR runs in the reference's fp32 (SWPS_F32)");
  if (cfg->minibatch <= 0) return fail(SWPS_E_CFG, "minibatch must be positive");
  SWPS_HIP(hipSetDevice(t->cfg.device));
  swps_lr *l = new swps_lr();
  l->t = t;
  l->cfg = *cfg;
  l->plan_req = cfg->plan;
  l->s = t->stream;
  l->timer.on = cfg->profile != 0;
  if (const char *e = getenv("SWPS_LR_PACK")) l->rows_per_wave = atoi(e);  // A/B timing, tests
  if (const char *e = getenv("SWPS_LR_DIAG")) l->fwd_diag = atoi(e);
  if (const char *e = getenv("SWPS_LR_FWD_G")) l->fwd_groups = atoi(e);  // A/B, tests
  if (const char *e = getenv("SWPS_LR_FWD_C")) l->fwd_c = atoi(e);      // A/B, tests
  if (const char *e = getenv("SWPS_LR_STAGE")) l->stage = atoi(e);        // A/B, tests
  if (const char *e = getenv("SWPS_LR_HOT")) l->hot = atoi(e);            // A/B, tests
  if (const char *e = getenv("SWPS_LR_NHOT")) l->nhot = (uint32_t)std::min(std::max(atoi(e), 1), kLrHot);
  if (const char *e = getenv("SWPS_LR_FWD_RECORDS")) l->fwd_records = atoi(e);  // A/B, tests
  if (const char *e = getenv("SWPS_LR_INLINE")) l->inline_records = atoi(e);     // A/B, tests       // timing experiments (wrong results)
  if (const char *e = getenv("SWPS_LR_FUSED")) l->fused_reduce = atoi(e) != 0;  // A/B timing, tests
  if (const char *e = getenv("SWPS_LR_TILES")) l->tiles = atoi(e);                // A/B timing, tests
  if (const char *e = getenv("SWPS_LR_PLACE")) l->place = atoi(e);                // A/B, tests
  if (const char *e = getenv("SWPS_LR_XCD")) l->xcd = atoi(e);                    // A/B, tests
  if (const char *e = getenv("SWPS_LR_TILE_CHUNK")) {
    const int c = atoi(e);
    l->tile_chunk = c == 512 || c == 1024 || c == 1280 || c == 1536 || c == 1792 || c == 2048 || c == 4096 ? (uint32_t)c
                                                                                                           : kTileChunk;
  }
  if (const char *e = getenv("SWPS_LR_TILE_THREADS")) {  // 512: blocks of 2,048 records, 4 per thread (A/B)
    l->tile_threads = atoi(e) == 512 ? 512 : 256;
    if (l->tile_threads == 512) l->tile_chunk = 2048;
  }
  if (const char *e = getenv("SWPS_LR_TILE_BITS")) l->tile_bits = std::min(std::max(atoi(e), 4), kTileMaxBits);
  // hot codes carry kLrHotBit (bit 31) in the word that otherwise holds a shard row: only while
  // every row index stays below it
  if (t->cfg.capacity > (uint64_t)kLrHotBit) l->hot = 0;
  if (hipHostMalloc((void **)&l->h_small, 64) != hipSuccess) {
    delete l;
    return fail(SWPS_E_OOM, "pinned alloc");
  }
  *out = l;
  return SWPS_OK;
}

int swps_lr_destroy(swps_lr *l) {
  if (!l) return SWPS_OK;
  (void)hipSetDevice(l->t->cfg.device);
  (void)hipStreamSynchronize(l->s);
  if (l->ps) {
    (void)hipStreamSynchronize(l->ps);
    (void)hipStreamDestroy(l->ps);
  }
  for (auto &p : l->pslot) {
    if (p.ready) (void)hipEventDestroy(p.ready);
    if (p.used) (void)hipEventDestroy(p.used);
  }
  if (l->ev_rows) (void)hipEventDestroy(l->ev_rows);
  l->timer.resolve();
  if (l->h_small) (void)hipHostFree(l->h_small);
  delete l->drv;
  delete l;
  (void)hipGetLastError();  // leave no sticky error from the calls above
  return SWPS_OK;
}

// parse_instance2 (lr.cpp:103-131): label "%f", then "%d:%f" pairs; blank
// and '#' lines are skipped.
int swps_lr_load_text(swps_lr *l, const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return fail(SWPS_E_IO, std::string("cannot open ") + path);
  l->label.clear();
  l->row_off.assign(1, 0);
  l->fval.clear();
  std::vector<uint32_t> feat;
  char *buf = nullptr;
  size_t cap = 0;
  ssize_t n;
  while ((n = getdelim(&buf, &cap, '\n', f)) >= 0) {
    if (n >= 1 && buf[n - 1] == '\n') buf[--n] = 0;
    const char *p = buf;
    while (*p == ' ') p++;
    if (*p == 0 || *p == '#') continue;
    float value;
    int nchar, feature;
    if (sscanf(p, "%f%n", &value, &nchar) < 1) {
      free(buf);
      fclose(f);
      return fail(SWPS_E_IO, "cannot parse line");
    }
    p += nchar;
    l->label.push_back(value);
    while (sscanf(p, "%d:%f%n", &feature, &value, &nchar) >= 2) {
      p += nchar;
      feat.push_back((uint32_t)feature);
      l->fval.push_back(value);
    }
    l->row_off.push_back(feat.size());
  }
  free(buf);
  fclose(f);
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  return lr_ingest(l, feat.data(), feat.size());
}

int swps_lr_load_csr(swps_lr *l, const float *labels, uint64_t nrows, const uint64_t *row_off, const uint32_t *feat,
                     const float *vals) {
  if (row_off[0] != 0) return fail(SWPS_E_CFG, "row_off[0] must be 0");
  l->label.assign(labels, labels + nrows);
  l->row_off.assign(row_off, row_off + nrows + 1);
  const uint64_t nnz = row_off[nrows];
  l->fval.assign(vals, vals + nnz);
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  return lr_ingest(l, feat, nnz);
}

int swps_lr_init(swps_lr *l) {
  if (!l->loaded) return fail(SWPS_E_STATE, "load data first");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  if (l->drv) return l->drv->full_pull();  // the first full pull, over the communicator
  if (l->t->comm)
    return fail(SWPS_E_UNSUPPORTED, "the table is key-sharded (swps_table_route): drive the context with "
                                    "swps_lr_shard_comm");
  const uint64_t V = l->vocab_keys.size();
  DevMem dk;
  SWPS_TRY(upload(dk, l->vocab_keys, l->s));
  // keys the table already holds (ClusterServer::load of a dump before the
  // first pull, lr.cpp:297-300 -> server.h:49-62) are found by the reference's
  // pull, not initialised: they keep their rows and draw nothing
  std::vector<uint32_t> pre;
  uint64_t held = 0;
  SWPS_TRY(swps_table_size(l->t, &held));
  if (l->cfg.init_ref && held) {
    DevMem dp;
    SWPS_TRY(dp.ensure(std::max<uint64_t>(1, V) * 4));
    SWPS_TRY(table_probe(l->t, dk.as<uint64_t>(), V, dp.as<uint32_t>(), l->s));  // misses are expected
    pre.resize(V);
    if (V) SWPS_HIP(hipMemcpyAsync(pre.data(), dp.p, V * 4, hipMemcpyDeviceToHost, l->s));
    SWPS_HIP(hipStreamSynchronize(l->s));
  }
  if (l->vid_place.size() == V)  // rows in first-appearance order (lr_ingest); init in pull order
    SWPS_TRY(table_find_or_insert_placed(l->t, dk.as<uint64_t>(), V, l->vid_place.data(),
                                         l->d_vid_row.as<uint32_t>(), l->s));
  else
    SWPS_TRY(table_find_or_insert(l->t, dk.as<uint64_t>(), V, l->d_vid_row.as<uint32_t>(), l->s));
  l->rows_mapped = false;  // vid_row changed: k_lr_map_rows again at the next batch
  if (l->ps) {  // a prefetched plan holds the old shard rows: plan again
    SWPS_HIP(hipStreamSynchronize(l->ps));
    l->plan_next = l->cursor;
  }
  l->plan_sync = true;
  l->fx_ready = false;  // the fixed-point step's per-key codes hold shard rows
  if (l->cfg.init_ref) {
    // LRPullAccessMethod::init_param (lr.cpp:48-50): w = gen_float() per miss, in first-pull order
    std::vector<uint32_t> vid_row(V), rid;
    if (V) SWPS_HIP(hipMemcpyAsync(vid_row.data(), l->d_vid_row.p, V * 4, hipMemcpyDeviceToHost, l->s));
    SWPS_HIP(hipStreamSynchronize(l->s));
    std::vector<float> rows;
    rows.reserve(V * 2);
    rid.reserve(V);
    uint64_t y = std::numeric_limits<unsigned long>::max() / 2;
    for (uint64_t j = 0; j < V; j++) {
      const uint64_t i = l->pull_order.size() == V ? l->pull_order[j] : j;  // first-pull order
      if (!pre.empty() && pre[i] != kNoRow) continue;
      y = y * kFlcgA + kLcgC;
      rows.push_back(flcg_value(y));
      rows.push_back(0.f);
      rid.push_back(vid_row[i]);
    }
    if (!rid.empty()) {
      DevMem dr, dri;
      SWPS_TRY(upload(dr, rows, l->s));
      SWPS_TRY(upload(dri, rid, l->s));
      SWPS_TRY(table_set_rows(l->t, dri.as<uint32_t>(), rid.size(), dr.p, l->s));
    }
    SWPS_HIP(hipStreamSynchronize(l->s));
  }
  l->inited = true;
  return SWPS_OK;
}

int swps_lr_train_batches(swps_lr *l, uint64_t count) {
  if (l->drv) {
    SWPS_HIP(hipSetDevice(l->t->cfg.device));
    l->mirror_stale = true;  // world 1 in place, rows by fid: the table may have been written since
    return l->drv->steps(count);  // collective
  }
  if (l->sharded) return fail(SWPS_E_STATE, "sharded: drive swps_lr_request/serve_pull/step/serve_push");
  if (!l->inited) return fail(SWPS_E_STATE, "call swps_lr_init first");
  if (l->nbatches == 0) return SWPS_OK;
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  l->mirror_stale = true;  // the table may have been written since the last call
  for (uint64_t i = 0; i < count; i++) SWPS_TRY(lr_batch(l));
  return SWPS_OK;
}

// lr.cpp:175-236: per epoch the mean of (y-p)^2 over the trained rows,
// accumulated in row order in double like `total_error`.
int swps_lr_epoch_error(swps_lr *l, double *err) {
  const uint64_t nr = l->label.size();
  std::vector<float> e2(nr);
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  if (nr) SWPS_HIP(hipMemcpyAsync(e2.data(), l->d_err2.p, nr * 4, hipMemcpyDeviceToHost, l->s));
  SWPS_HIP(hipStreamSynchronize(l->s));
  double tot = 0;
  for (uint64_t r = 0; r < nr; r++) tot += e2[r];
  *err = nr ? tot / (double)nr : 0.0;
  return SWPS_OK;
}

int swps_lr_train(swps_lr *l, int32_t niters, double *err_out) {
  if (l->drv) {  // lockstep epochs of steps_per_epoch steps; error of this rank's rows
    if (l->drv->spe && l->drv->cursor % l->drv->spe) return fail(SWPS_E_STATE, "not at an epoch boundary");
    for (int it = 0; it < niters; it++) {
      SWPS_TRY(l->drv->steps(l->drv->spe));
      SWPS_TRY(l->drv->sync());
      if (err_out) SWPS_TRY(swps_lr_epoch_error(l, &err_out[it]));
    }
    return swps_lr_sync(l);
  }
  if (l->sharded) return fail(SWPS_E_STATE, "sharded: drive swps_lr_request/serve_pull/step/serve_push");
  if (l->cursor % std::max<uint64_t>(1, l->nbatches)) return fail(SWPS_E_STATE, "not at an epoch boundary");
  for (int it = 0; it < niters; it++) {
    SWPS_TRY(swps_lr_train_batches(l, l->nbatches));
    if (err_out) SWPS_TRY(swps_lr_epoch_error(l, &err_out[it]));
  }
  return swps_lr_sync(l);
}

int swps_lr_sync(swps_lr *l) {
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  if (l->drv) SWPS_TRY(l->drv->sync());
  if (l->ps) SWPS_HIP(hipStreamSynchronize(l->ps));  // the prefetched next plan included
  SWPS_HIP(hipStreamSynchronize(l->s));
  l->timer.resolve();
  return SWPS_OK;
}

// LR::predict_instance (lr.cpp:376-385) with the shard's current weights.
int swps_lr_predict(swps_lr *l, float *pred_out, float *target_out, uint64_t cap) {
  const uint64_t nr = l->label.size();
  if (cap < nr) return fail(SWPS_E_CFG, "buffer too small");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  if (l->drv) {  // refresh the worker cache with a full pull (collective)
    SWPS_TRY(l->drv->sync());
    SWPS_TRY(l->drv->full_pull());
  }
  SWPS_TRY(l->d_pred.ensure(std::max<uint64_t>(1, nr) * 4));
  k_lr_predict<<<nblk(nr * 64), 256, 0, l->s>>>(l->d_row_off.as<uint64_t>(), l->d_fvid.as<int32_t>(), l->d_fval.as<float>(),
                                            nr, l->sharded ? nullptr : l->d_vid_row.as<uint32_t>(),
                                            l->sharded ? l->d_wcache.as<float>() : l->t->rows.as<float>(),
                                            l->d_pred.as<float>());
  SWPS_HIP(hipGetLastError());
  if (nr) SWPS_HIP(hipMemcpyAsync(pred_out, l->d_pred.p, nr * 4, hipMemcpyDeviceToHost, l->s));
  SWPS_HIP(hipStreamSynchronize(l->s));
  if (target_out) std::copy(l->label.begin(), l->label.end(), target_out);
  return SWPS_OK;
}

// weights of every key, sorted by key
int swps_lr_params(swps_lr *l, uint32_t *keys, float *w, float *g2, uint64_t cap, uint64_t *n) {
  const uint64_t V = l->vocab_keys.size();
  *n = V;
  if (cap < V) return fail(SWPS_E_CFG, "buffer too small");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  DevMem d;
  SWPS_TRY(d.ensure(std::max<uint64_t>(1, V) * 8));
  SWPS_TRY(table_get_rows(l->t, l->d_vid_row.as<uint32_t>(), V, d.p, l->s));
  std::vector<float> rows(V * 2);
  if (V) SWPS_HIP(hipMemcpyAsync(rows.data(), d.p, V * 8, hipMemcpyDeviceToHost, l->s));
  SWPS_HIP(hipStreamSynchronize(l->s));
  std::vector<uint64_t> order(V);
  for (uint64_t i = 0; i < V; i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return l->vocab_keys[a] < l->vocab_keys[b]; });
  for (uint64_t i = 0; i < V; i++) {
    keys[i] = (uint32_t)l->vocab_keys[order[i]];
    w[i] = rows[2 * order[i]];
    g2[i] = rows[2 * order[i] + 1];
  }
  return SWPS_OK;
}

int swps_lr_plan_info(swps_lr *l, int32_t *o) {
  o[0] = l->cfg.plan;
  o[1] = l->plan_req;
  o[2] = l->fx_bits;
  o[3] = l->fx_floor;
  o[4] = l->fx_fallback ? 1 : 0;
  return SWPS_OK;
}

int swps_lr_info(swps_lr *l, uint64_t *o) {
  o[0] = l->label.size();
  o[1] = l->vocab_keys.size();
  o[2] = l->nbatches;
  o[3] = l->row_off.empty() ? 0 : l->row_off.back();
  return SWPS_OK;
}

int swps_lr_set_profile(swps_lr *l, int32_t on) {
  SWPS_TRY(swps_lr_sync(l));
  l->timer.on = on != 0;
  return SWPS_OK;
}

int swps_lr_kernel_times(swps_lr *l, double *out, int32_t reset) {
  SWPS_TRY(swps_lr_sync(l));
  for (int k = 0; k < 4; k++) {
    out[2 * k] = l->timer.ms[k];
    out[2 * k + 1] = (double)l->timer.cnt[k];
    if (reset) {
      l->timer.ms[k] = 0;
      l->timer.cnt[k] = 0;
    }
  }
  return SWPS_OK;
}

// ============================================================================
// Key-sharded LR over several GPUs (one process per GPU; the caller moves the
// payloads, swiftmpi_amd/dist.py).  Key -> owner = BasicHashFrag node - 1
// (cluster/hashfrag.h:33-56).  Per batch: request (the batch's unique
// features, grouped by owner) -> serve_pull (owner: weights) -> step
// (install, forward, mean gradients in request order) -> serve_push (owner:
// AdaGrad once per source rank, in rank order; lr.cpp:58-81).
// ============================================================================

int swps_lr_shard(swps_lr *l, int32_t rank, int32_t world, int32_t frag_num) {
  if (!l->loaded) return fail(SWPS_E_STATE, "load data first");
  if (l->inited) return fail(SWPS_E_STATE, "shard before swps_lr_init / the first pull");
  if (world < 1 || rank < 0 || rank >= world) return fail(SWPS_E_CFG, "bad rank/world");
  if (l->cfg.init_ref)
    return fail(SWPS_E_UNSUPPORTED, "sharded mode initialises on the owners (init_ref = 0, SWPS_INIT_HASH): the "
                                    "reference's float-LCG order depends on message arrival");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  // plan none with fast sums: the learner runs the fixed-point step (no index); otherwise the
  // sharded step reads the static index
  SWPS_TRY(lr_fwd_chunks(l));
  l->fx_sharded = lr_fx_sharded_usable(l);
  if (!l->fx_sharded && !l->index_built) SWPS_TRY(lr_index(l));
  std::vector<uint32_t> map(frag_num);
  SWPS_TRY(swps_hashfrag_table(frag_num, world, map.data()));
  const uint64_t V = l->vocab_keys.size(), nb = l->nbatches, nr = l->label.size();
  std::vector<int32_t> owner(V);
  for (uint64_t i = 0; i < V; i++) owner[i] = (int32_t)map[fmix64(l->vocab_keys[i]) % (uint64_t)frag_num] - 1;
  SWPS_TRY(lr_fvid_host(l));
  // per batch: unique vids in owner order, then vid order (counting sort by owner) — batches are
  // independent: worker threads build them (each its own stamp array), then one concatenation
  l->kofs.assign(nb, 0);
  l->bU.assign(nb, 0);
  l->bcounts.assign(nb * world, 0);
  std::vector<std::vector<int32_t>> kb(nb);
  {
    const unsigned nth = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>({nb, 16, std::max(1u, std::thread::hardware_concurrency())}));
    std::atomic<uint64_t> next_b{0};
    auto work = [&]() {
      std::vector<uint32_t> stamp(V, 0u);
      std::vector<int32_t> uniq;
      std::vector<uint64_t> start(world + 1);
      for (uint64_t bi; (bi = next_b.fetch_add(1)) < nb;) {
        const uint64_t r0 = bi * l->B1(), r1 = std::min<uint64_t>(nr, r0 + l->B1());
        const uint32_t tag = (uint32_t)bi + 1u;
        uniq.clear();
        for (uint64_t i = l->row_off[r0]; i < l->row_off[r1]; i++) {
          const int32_t v = l->fvid[i];
          if (stamp[v] != tag) {
            stamp[v] = tag;
            uniq.push_back(v);
          }
        }
        std::sort(uniq.begin(), uniq.end());
        uint64_t *cnt = &l->bcounts[bi * world];
        for (int32_t v : uniq) cnt[owner[v]]++;
        start[0] = 0;
        for (int r = 0; r < world; r++) start[r + 1] = start[r] + cnt[r];
        std::vector<int32_t> &dst = kb[bi];
        dst.resize(uniq.size());
        for (int32_t v : uniq) dst[start[owner[v]]++] = v;
      }
    };
    std::vector<std::thread> th;
    for (unsigned q = 1; q < nth; q++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
  }
  l->allK.clear();
  uint64_t tot = 0;
  for (uint64_t bi = 0; bi < nb; bi++) tot += kb[bi].size();
  l->allK.reserve(tot);
  for (uint64_t bi = 0; bi < nb; bi++) {
    l->kofs[bi] = l->allK.size();
    l->bU[bi] = kb[bi].size();
    l->allK.insert(l->allK.end(), kb[bi].begin(), kb[bi].end());
    std::vector<int32_t>().swap(kb[bi]);
  }
  l->init_order.resize(V);
  for (uint64_t i = 0; i < V; i++) l->init_order[i] = (int32_t)i;
  // the full pull's keys by owner, and within an owner in fid order when the fixed-point step runs:
  // the owner inserts them in that order, so its rows follow the step's buckets (at world 1 the rows
  // are base + fid, and the in-place push updates each bucket's rows as one contiguous run)
  if (l->fx_sharded && l->fx_fid.size() == V)
    std::sort(l->init_order.begin(), l->init_order.end(), [&](int32_t a, int32_t b) {
      return owner[a] != owner[b] ? owner[a] < owner[b] : l->fx_fid[a] < l->fx_fid[b];
    });
  else
    std::stable_sort(l->init_order.begin(), l->init_order.end(),
                     [&](int32_t a, int32_t b) { return owner[a] < owner[b]; });
  l->icounts.assign(world, 0);
  for (uint64_t i = 0; i < V; i++) l->icounts[owner[i]]++;
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  SWPS_TRY(upload(l->d_K, l->allK, l->s));
  SWPS_TRY(upload(l->d_vkeys, l->vocab_keys, l->s));
  SWPS_TRY(upload(l->d_init_order, l->init_order, l->s));
  SWPS_TRY(l->d_wcache.ensure(std::max<uint64_t>(V, 1) * 4));
  SWPS_TRY(l->d_local.ensure(std::max<uint64_t>(V, 1) * 4));
  SWPS_HIP(hipMemsetAsync(l->d_wcache.p, 0, std::max<uint64_t>(V, 1) * 4, l->s));
  if (l->fx_sharded) {
    SWPS_TRY(l->d_wcache2.ensure(std::max<uint64_t>(V, 1) * 8));
    SWPS_HIP(hipMemsetAsync(l->d_wcache2.p, 0, std::max<uint64_t>(V, 1) * 8, l->s));
    SWPS_TRY(upload(l->d_fx_fidv, l->fx_fid, l->s));
    SWPS_TRY(l->d_localf.ensure(std::max<uint64_t>(V, 1) * 4));
  }
  SWPS_HIP(hipStreamSynchronize(l->s));
  l->rank = rank;
  l->world = world;
  l->sharded = true;
  return SWPS_OK;
}

int swps_lr_batch_counts(swps_lr *l, uint64_t *out, uint64_t cap, uint64_t *nb) {
  if (!l->sharded) return fail(SWPS_E_STATE, "not sharded");
  *nb = l->nbatches;
  if (cap < l->bcounts.size()) return fail(SWPS_E_CFG, "buffer too small");
  std::copy(l->bcounts.begin(), l->bcounts.end(), out);
  return SWPS_OK;
}

int swps_lr_request(swps_lr *l, int32_t init, uint64_t *counts, uint64_t *d_keys, uint64_t *n) {
  if (!l->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  if (init) {
    std::copy(l->icounts.begin(), l->icounts.end(), counts);
    *n = l->vocab_keys.size();
    if (d_keys && *n)
      k_lr_keys<<<nblk(*n), 256, 0, l->s>>>(l->d_init_order.as<int32_t>(), *n, l->d_vkeys.as<uint64_t>(), d_keys);
  } else {
    if (l->nbatches == 0) return fail(SWPS_E_STATE, "no batches");
    const uint64_t bi = l->cursor % l->nbatches;
    std::copy(l->bcounts.begin() + bi * l->world, l->bcounts.begin() + (bi + 1) * l->world, counts);
    *n = l->bU[bi];
    if (d_keys && *n)
      k_lr_keys<<<nblk(*n), 256, 0, l->s>>>(l->d_K.as<int32_t>() + l->kofs[bi], *n, l->d_vkeys.as<uint64_t>(), d_keys);
  }
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

int swps_lr_serve_pull(swps_lr *l, const uint64_t *d_keys, const uint64_t *src_counts, int32_t insert,
                       float *d_vals) {
  if (!l->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  uint64_t n = 0;
  for (int r = 0; r < l->world; r++) n += src_counts[r];
  if (!insert && l->slot >= 0) {  // a driver step slot: the same keys every epoch
    while ((uint64_t)l->slot >= l->slot_rows.size()) l->slot_rows.emplace_back(new swps_lr::SlotRows());
    auto &e = *l->slot_rows[l->slot];
    if (e.n != n || !e.rows.p) {
      SWPS_TRY(e.rows.ensure(std::max<uint64_t>(n, 1) * 4));
      SWPS_TRY(table_lookup(l->t, d_keys, n, e.rows.as<uint32_t>(), l->s));
      e.n = n;
      e.sorted_valid = false;
    }
    l->serve_n = n;
    if (!d_vals && n) {  // the driver's in-place pull (AppOps::pull_in_place): the step reads these rows
      if (l->world != 1 || !l->fx_sharded) return fail(SWPS_E_STATE, "an in-place pull needs world 1 and the fixed-point step");
      l->pull_rows = e.rows.as<uint32_t>();
      return SWPS_OK;
    }
    return table_copy_pull(l->t, e.rows.as<uint32_t>(), n, d_vals, l->s);
  }
  if (!d_vals && n) return fail(SWPS_E_STATE, "serve_pull without a value buffer needs a world-1 driver step slot");
  SWPS_TRY(l->d_serve_rows.ensure(std::max<uint64_t>(n, 1) * 4));
  uint32_t *rows = l->d_serve_rows.as<uint32_t>();
  if (insert) {  // keys are distinct within a source, not across sources
    uint64_t off = 0;
    std::vector<uint32_t> iota;
    for (int r = 0; r < l->world; r++) {
      if (l->fx_sharded) {  // new rows in request order (by fid: swps_lr_shard's init_order)
        iota.resize(src_counts[r]);
        for (uint64_t q = 0; q < src_counts[r]; q++) iota[q] = (uint32_t)q;
        SWPS_TRY(table_find_or_insert_placed(l->t, d_keys + off, src_counts[r], iota.data(), rows + off, l->s));
      } else {
        SWPS_TRY(table_find_or_insert(l->t, d_keys + off, src_counts[r], rows + off, l->s));
      }
      off += src_counts[r];
    }
    // world 1: the full pull's keys in fid order (swps_lr_shard's init_order) — when their rows came
    // out as base + fid, the in-place step runs the single-GPU affine form
    const uint64_t V = l->vocab_keys.size();
    l->w1_base = -1;
    const char *wa = getenv("SWPS_LR_W1_AFFINE");  // 0: the install / row-indexed push (A/B, tests)
    if (l->world == 1 && l->fx_sharded && n == V && V && l->fx_fid.size() == V && !(wa && atoi(wa) == 0)) {
      std::vector<uint32_t> hr(n);
      SWPS_HIP(hipMemcpyAsync(hr.data(), rows, n * 4, hipMemcpyDeviceToHost, l->s));
      SWPS_HIP(hipStreamSynchronize(l->s));
      bool aff = (uint64_t)hr[0] + V <= l->t->cfg.capacity;
      for (uint64_t j = 0; j < n && aff; j++)
        aff = hr[j] == hr[0] + (uint32_t)j && l->fx_fid[l->init_order[j]] == (uint32_t)j;
      const uint32_t nh = (uint32_t)l->fx_hot_vids.size();
      if (aff) {
        std::vector<uint32_t> hrow(std::max<uint32_t>(nh, 1));
        for (uint32_t q = 0; q < hrow.size(); q++) hrow[q] = hr[0] + q;
        SWPS_TRY(upload(l->d_w1_hrow, hrow, l->s));
        SWPS_HIP(hipStreamSynchronize(l->s));
        l->w1_base = hr[0];
        l->mirror_stale = true;
      }
    }
  } else {
    SWPS_TRY(table_lookup(l->t, d_keys, n, rows, l->s));
  }
  SWPS_TRY(table_copy_pull(l->t, rows, n, d_vals, l->s));
  l->serve_n = n;
  return SWPS_OK;
}

int swps_lr_install(swps_lr *l, const float *d_vals) {
  if (!l->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  const uint64_t V = l->vocab_keys.size();
  // the full pull's values by vid (swps_lr_predict reads them; the fixed-point step installs each
  // batch's own at its layout)
  if (V)
    k_lr_install<<<nblk(V), 256, 0, l->s>>>(l->d_init_order.as<int32_t>(), V, d_vals, l->d_wcache.as<float>(),
                                            nullptr, 1);
  SWPS_HIP(hipGetLastError());
  l->inited = true;
  return SWPS_OK;
}

int swps_lr_step(swps_lr *l, const float *d_vals, float *d_grads) {
  if (!l->sharded) return fail(SWPS_E_STATE, "not sharded");
  if (!l->inited) return fail(SWPS_E_STATE, "install the first full pull first");
  if (l->nbatches == 0) return SWPS_OK;
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  return lr_batch(l, d_vals, d_grads);
}

// d_keys: the keys of the matching serve_pull (the push request carries its keys)
int swps_lr_serve_push(swps_lr *l, const uint64_t *d_keys, const float *d_grads, const uint64_t *src_counts) {
  if (!l->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  uint64_t n = 0;
  for (int r = 0; r < l->world; r++) n += src_counts[r];
  if (n != l->serve_n) return fail(SWPS_E_STATE, "push does not match the served pull");
  if (l->pushed_in_place) {  // world 1 in place: the step's push already applied AdaGrad to these rows
    l->pushed_in_place = false;
    return SWPS_OK;
  }
  int nsrc = 0;
  for (int r = 0; r < l->world; r++) nsrc += src_counts[r] > 0;
  if (l->slot >= 0 && (uint64_t)l->slot < l->slot_rows.size() && l->slot_rows[l->slot]->n == n &&
      l->slot_rows[l->slot]->rows.p) {  // this slot's pull looked the same keys up
    auto &e = *l->slot_rows[l->slot];
    return table_push_sources(l->t, e.rows.as<uint32_t>(), n, d_grads, l->s, false, nsrc <= 1, &e.sorted,
                              &e.sorted_valid);
  }
  SWPS_TRY(l->d_serve_rows.ensure(std::max<uint64_t>(n, 1) * 4));
  SWPS_TRY(table_lookup(l->t, d_keys, n, l->d_serve_rows.as<uint32_t>(), l->s));
  // one AdaGrad step per source, in rank order, all sources in one pass
  return table_push_sources(l->t, l->d_serve_rows.as<uint32_t>(), n, d_grads, l->s, false, nsrc <= 1);
}

// the fixed-point step's algorithmic bytes for batch `batch` (what the bucketed
// form must move at least once): out[0] k_lr_fxb_step, out[1] k_lr_fxb_push, out[2] 1 when the
// bucketed form runs (2: the atomic form, 0: another plan), out[3] hot keys, out[4] buckets,
// out[5] the step's blocks, out[6] non-hot records, out[7] distinct non-hot keys
int swps_lr_fx_bytes(swps_lr *l, uint64_t batch, uint64_t *out8) {
  if (!l->loaded || batch >= l->nbatches) return fail(SWPS_E_CFG, "no such batch");
  for (int i = 0; i < 8; i++) out8[i] = 0;
  if (!(lr_fx_usable(l) || l->fx_sharded) || !l->fx_ready) return SWPS_OK;  // sharded: the same model
  SWPS_TRY(lr_fvid_host(l));
  const bool hot = l->hot != 0 && !l->fx_hot_vids.empty();
  const uint64_t nh = hot ? l->fx_hot_vids.size() : 0;
  std::vector<uint8_t> ishot(l->vocab_keys.size(), 0);
  for (uint64_t q = 0; q < nh; q++) ishot[l->fx_hot_vids[q]] = 1;
  const uint64_t r0 = batch * l->B1(), r1 = std::min<uint64_t>(l->label.size(), r0 + l->B1());
  const uint64_t nnz = l->row_off[r1] - l->row_off[r0], nrows = r1 - r0;
  uint64_t nonhot = 0, uniq = 0;
  std::unordered_set<int32_t> u;
  for (uint64_t c = l->row_off[r0]; c < l->row_off[r1]; c++) {
    const int32_t v = l->fvid[c];
    if (ishot[v]) continue;
    nonhot++;
    u.insert(v);
  }
  uniq = u.size();
  const uint64_t nch = l->bfchunk[batch + 1] - l->bfchunk[batch];
  const uint64_t grid = std::min<uint64_t>(nch, l->fxb_grid), nbk = l->fxb_nbk;
  if (l->fx_atomic) {
    out8[2] = 2;
    return SWPS_OK;
  }
  // step: per record its fid, x_i and weight (12 B), per row its offset, label, e, e^2 (20 B), per
  // non-hot record its (fid, e*x_i) written (8 B), the chunks' bucket offsets, the hot partials
  // (the bucket regions, fxb_res: no offsets — each chunk's span comes from an atomic per bucket)
  const uint64_t offs = l->fxb_res ? 0 : 2 * (nbk + 1) * nch;
  out8[0] = 12 * nnz + 20 * nrows + 8 * nonhot + offs + 12 * nh * grid;
  // push: the records and offsets read back, each distinct non-hot key's [w | g2] read and written,
  // the hot partials read, the hot keys' rows read and written
  out8[1] = 8 * nonhot + offs + 16 * uniq + 12 * nh * grid + 16 * nh;
  out8[2] = 1;
  out8[3] = nh;
  out8[4] = nbk;
  out8[5] = grid;
  out8[6] = nonhot;
  out8[7] = uniq;
  return SWPS_OK;
}

int swps_lr_exchange_stats(swps_lr *l, int32_t on, double *out4) {
  if (!l->drv) return fail(SWPS_E_STATE, "not driven by swps_lr_shard_comm");
  SWPS_TRY(l->drv->sync());
  if (out4) {
    out4[0] = (double)l->drv->bytes_remote;
    out4[1] = (double)l->drv->bytes_total;
    out4[2] = (double)l->drv->calls;
    out4[3] = l->drv->xms;
  }
  if (on >= 0) {
    l->drv->xprof = on != 0;
    l->drv->bytes_remote = l->drv->bytes_total = l->drv->calls = 0;
    l->drv->xms = 0;
  }
  return SWPS_OK;
}

int swps_lr_shard_comm(swps_lr *l, swps_comm *c, int32_t frag_num) {
  if (!c) return fail(SWPS_E_CFG, "null communicator");
  if (comm_device(c) != l->t->cfg.device) return fail(SWPS_E_CFG, "communicator and table are on different devices");
  if (l->t->comm && l->t->comm != c) return fail(SWPS_E_CFG, "the table is routed over another communicator");
  if (l->drv) return fail(SWPS_E_STATE, "swps_lr_shard_comm was already called on this context");
  SWPS_TRY(swps_lr_shard(l, comm_rank(c), comm_world(c), frag_num));
  ShardDriver *d = new ShardDriver();
  d->c = c;
  AppOps &o = d->ops;
  o.h = l;
  o.cs = l->s;
  o.width = 1;
  o.val_bytes = 4;
  o.grad_bytes = 4;
  o.batch_counts = [](void *h, uint64_t *out, uint64_t cap, uint64_t *nb) {
    return swps_lr_batch_counts((swps_lr *)h, out, cap, nb);
  };
  o.request = [](void *h, int32_t init, uint64_t *cnt, uint64_t *k, uint64_t *n) {
    return swps_lr_request((swps_lr *)h, init, cnt, k, n);
  };
  o.serve_pull = [](void *h, const uint64_t *k, const uint64_t *sc, int32_t ins, void *v) {
    return swps_lr_serve_pull((swps_lr *)h, k, sc, ins, (float *)v);
  };
  o.install = [](void *h, const void *v) { return swps_lr_install((swps_lr *)h, (const float *)v); };
  o.step = [](void *h, const void *v, void *g) { return swps_lr_step((swps_lr *)h, (const float *)v, (float *)g); };
  o.serve_push = [](void *h, const uint64_t *k, const void *g, const uint64_t *sc) {
    return swps_lr_serve_push((swps_lr *)h, k, (const float *)g, sc);
  };
  // per-slot row lookups and push grouping (SWPS_LR_SLOT_ROWS=0: look the rows up every call)
  const char *sr = getenv("SWPS_LR_SLOT_ROWS");
  if (!(sr && atoi(sr) == 0))
    o.set_slot = [](void *h, int64_t slot) {
      ((swps_lr *)h)->slot = slot;
      return (int)SWPS_OK;
    };
  // world 1 with the fixed-point step: pull and push in place on the shard rows (the driver passes
  // no value buffer; SWPS_PULL_IN_PLACE=0 keeps the copy, the payload and the owner's apply)
  const char *pip = getenv("SWPS_PULL_IN_PLACE");
  o.pull_in_place = l->fx_sharded && !(pip && atoi(pip) == 0);
  const int rc = d->setup();
  if (rc) {
    delete d;
    return rc;
  }
  l->drv = d;
  return SWPS_OK;
}

void *swps_lr_stream(swps_lr *l) { return (void *)l->s; }

}  // extern "C"
