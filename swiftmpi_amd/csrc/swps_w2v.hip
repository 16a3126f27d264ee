// word2vec CBOW negative sampling on one MI355X: the reference's
// pull -> learn_instance -> push minibatch loop (apps/word2vec/
// word2vec_global.h:552-731, nthreads = 1 semantics) as a chain of HIP
// kernels over HBM-resident data.
//
// Per minibatch n (trained lines T_n, gathered key set K_n, U = |K_n|):
//   k_pull      cache[vid] <- table row (h, v) for vid in K_n; local[vid] = u
//               (global_pull_access.h:80-101: params[key]=val, grads reset)
//   k_keep      float-LCG subsample test per token, LCG jumped to the
//               token's stream offset (word2vec_global.h:725-731)
//   scans       kept positions per line -> main-LCG draw offset per kept
//               position (1 draw per line + (1+negative) per kept position)
//   k_forward   one wave per kept position: neu1 = sum of context v rows,
//               dots with the positive and the negative h rows (fp64),
//               exp-table sigmoid, neu1e; writes neu1/neu1e rows and one
//               (key, pair index) record per target and per context
//               (word2vec_global.h:663-718)
//   radix sort  records by local key index (stable: position order kept)
//   k_gather    chunked segmented sums  h_grad[k] = sum g*neu1[p],
//               v_grad[k] = sum neu1e[p]  into per-chunk partials (no atomics)
//   k_push      partials summed in chunk order, mean over the counts
//               (word2vec_global.h:122-134), AdaGrad on the table row
//               (word2vec_global.h:176-185)
// Params are read only from the frozen cache during a batch, exactly like the
// reference worker.  Negatives outside K_n read the stale cache and their
// gradients are dropped (the reference resets them at the next pull).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <memory>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <limits>
#include <map>
#include <unordered_map>
#include <type_traits>
#include <unordered_set>

#include <hip/hip_ext.h>

#include "swps_internal.h"
#include "swps_rand.h"
#include "swps_sort.h"
#include "swps_wave.h"

using namespace swps;

namespace {

constexpr int kMaxJump = 64;
// forward slot entry tag: a table row index (not a worker-cache vid); see slot_row
constexpr int32_t kTabRow = 0x40000000;
__constant__ uint64_t c_jumpA[kMaxJump + 1];
__constant__ uint64_t c_jumpC[kMaxJump + 1];

template <typename T> struct V16;
template <> struct V16<float> {
  using V = float4;
  static constexpr int E = 4;
};
template <> struct V16<double> {
  using V = double2;
  static constexpr int E = 2;
};


__global__ void k_build_unigram(const uint64_t *__restrict__ starts, uint32_t V, uint64_t T, int32_t *__restrict__ table) {
  uint64_t a = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (; a < T; a += stride) {
    uint32_t lo = 0, hi = V;  // largest i with starts[i] <= a
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (starts[mid] <= a)
        lo = mid;
      else
        hi = mid;
    }
    table[a] = (int32_t)lo;
  }
}

// Coarse index over the run-length unigram table: idx[b] = the word holding
// slot b << shift (the same "largest i with starts[i] <= a" as
// k_build_unigram), b in [0, nb].  A draw then binary-searches starts[] only
// between idx[b] and idx[b+1] (a few runs at 1024 slots per bucket) — 2.4 MB
// of L2-resident index instead of one random 4-B read into the 400-MB table.
__global__ void k_build_uidx(const uint64_t *__restrict__ starts, uint32_t V, int shift, uint64_t nb1,
                             int32_t *__restrict__ idx) {
  const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb1) return;
  const uint64_t a = b << shift;
  uint32_t lo = 0, hi = V;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (starts[mid] <= a)
      lo = mid;
    else
      hi = mid;
  }
  idx[b] = (int32_t)lo;
}

constexpr int kUShift = 10;  // unigram coarse index: 1024 slots per bucket

__device__ __forceinline__ int32_t unigram_lookup(const uint64_t *__restrict__ starts, const int32_t *__restrict__ idx,
                                                  int shift, uint32_t V, uint64_t slot) {
  const uint64_t b = slot >> shift;
  uint32_t lo = (uint32_t)idx[b], hi = min((uint32_t)idx[b + 1] + 1u, V);
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (starts[mid] <= slot)
      lo = mid;
    else
      hi = mid;
  }
  return (int32_t)lo;
}

// cache <- table rows (h, v) for the listed vids; local[vid] = u when set_local
template <typename T>
__global__ __launch_bounds__(256) void k_pull(const int32_t *__restrict__ K, uint32_t U,
                                              const uint32_t *__restrict__ vid_row, const T *__restrict__ rows,
                                              int D, T *__restrict__ cache_h, T *__restrict__ cache_v,
                                              int32_t *__restrict__ local, int set_local, int cs) {
  using V = typename V16<T>::V;
  constexpr int E = V16<T>::E;
  const int lane = threadIdx.x & 63;
  const int NC = D / E;
  for (uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < U; u += (uint64_t)gridDim.x * 4) {
    const int32_t vid = K ? K[u] : (int32_t)u;
    const V *src = (const V *)(rows + (uint64_t)vid_row[vid] * 4 * D);
    V *dh = (V *)(cache_h + (uint64_t)vid * cs);  // cs: the cache row stride (swps_w2v::cs)
    V *dv = (V *)(cache_v + (uint64_t)vid * cs);
    for (int c = lane; c < cs / E; c += 64) {  // the pad too (zeros): whole-line stores
      const bool in = c < NC;
      dh[c] = in ? src[c] : V{};
      dv[c] = in ? src[NC + c] : V{};
    }
    if (set_local && lane == 0) local[vid] = (int32_t)u;
  }
}

// float-LCG keep flags for the epoch (to_sample, word2vec_global.h:725-731):
// token t consumes the (t+1)-th draw after the epoch's start state.  k_keep_mb:
// each thread jumps once to the start of its run of kKeepRun tokens, then steps.
constexpr int kKeepRun = 16;
// float-LCG (subsampling) jumps by 2^i draws, x -> c_f2A[i] x + c_f2C[i] (set at create)
__constant__ uint64_t c_f2A[64];
__constant__ uint64_t c_f2C[64];
__device__ __forceinline__ uint64_t flcg_jump_p2(uint64_t x, uint64_t k) {
  for (int i = 0; k; i++, k >>= 1)
    if (k & 1) x = c_f2A[i] * x + c_f2C[i];
  return x;
}
// A wave takes 64 * kKeepIt consecutive tokens, lane l the tokens base + l + 64 j (coalesced loads and
// stores); the lane's float-LCG state jumps once to its first token, then 64 draws per step.
constexpr int kKeepIt = 16;
__global__ __launch_bounds__(256) void k_keep(const int32_t *__restrict__ tok, uint64_t nt,
                                              const float *__restrict__ ran, uint64_t fstate, int sample_on,
                                              int32_t *__restrict__ kflag) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lane = g & 63, base = (g >> 6) * (64ULL * kKeepIt);
  if (base > nt) return;
  uint64_t y = sample_on ? flcg_jump_p2(fstate, base + lane) : 0;  // the state after token base+lane-1's draw
  const uint64_t A64 = c_f2A[6], C64 = c_f2C[6];
#pragma unroll 4
  for (int j = 0; j < kKeepIt; j++) {
    const uint64_t i = base + lane + 64ULL * (uint64_t)j;
    if (i > nt) break;
    int32_t keep = 0;  // kflag[nt] = 0: the scan's end
    if (i < nt) {
      keep = 1;
      if (sample_on) keep = flcg_value(y * kFlcgA + kLcgC) > ran[tok[i]];  // word2vec_global.h:725-731
    }
    kflag[i] = keep;
    y = A64 * y + C64;
  }
}

// word2vec.h:621-629 to_sample with per-minibatch counts: freq =
// count_in_batch / (int)_num_words, where _num_words (never reset) is
// tw[b] for batch b of this epoch; btok[b] = first token of batch b.
__global__ void k_keep_mb(const int32_t *__restrict__ bcnt, uint64_t nt, const int64_t *__restrict__ btok,
                          uint32_t nb, const int32_t *__restrict__ tw, float sample, uint64_t fstate, int sample_on,
                          int32_t *__restrict__ kflag) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t i0 = r * kKeepRun;
  if (i0 > nt) return;
  uint64_t y = sample_on ? lcg_jump(fstate, i0, kFlcgA, kLcgC) : 0;
  uint32_t b = 0, hi = nb;  // batch of token i0
  while (hi - b > 1) {
    const uint32_t mid = (b + hi) >> 1;
    if ((uint64_t)btok[mid] <= i0)
      b = mid;
    else
      hi = mid;
  }
  for (uint64_t i = i0; i < i0 + kKeepRun && i <= nt; i++) {
    if (i == nt) {
      kflag[i] = 0;
      break;
    }
    int32_t keep = 1;
    if (sample_on) {
      while (b + 1 < nb && (uint64_t)btok[b + 1] <= i) b++;
      y = y * kFlcgA + kLcgC;
      const float freq = (float)bcnt[i] / (float)tw[b];
      const float ran = (float)(1 - sqrt((double)(sample / freq)));
      keep = flcg_value(y) > ran;
    }
    kflag[i] = keep;
  }
}

// main-LCG draws per line: 1 (learn_instance's initial b) + kept*(1+negative)
__global__ void k_line_draws(const int64_t *__restrict__ line_off, uint64_t nl, const int32_t *__restrict__ kscan,
                             int N, uint64_t *__restrict__ ldraw) {
  uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > nl) return;
  if (j == nl) {
    ldraw[j] = 0;
    return;
  }
  uint64_t kept = (uint64_t)(kscan[line_off[j + 1]] - kscan[line_off[j]]);
  ldraw[j] = 1 + kept * (uint64_t)(N + 1);
}

// kept-count prefix at each batch boundary (token offsets given)
__global__ void k_bounds(const int32_t *__restrict__ kscan, const int64_t *__restrict__ btok, uint64_t n,
                         int32_t *__restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = kscan[btok[i]];
}

// x mod d for a fixed divisor d < 2^63 with the precomputed m = floor((2^64-1)/d):
// q = mulhi(x, m) underestimates x/d by at most 2, so two corrections are exact.
__device__ __forceinline__ uint64_t fast_mod(uint64_t x, uint64_t d, uint64_t m) {
  const uint64_t q = __umul64hi(x, m);
  uint64_t r = x - q * d;
  if (r >= d) r -= d;
  if (r >= d) r -= d;
  return r;
}

struct RecArgs {
  const int32_t *tok, *tok_line;
  const int64_t *line_off;
  const int32_t *pos_tok;
  uint32_t P;
  const int32_t *kscan;   // epoch-wide
  const uint64_t *ldoff;  // epoch-wide
  uint64_t lstate;        // main LCG state at the epoch start
  int W, N;
  uint64_t mW;  // floor((2^64-1)/W)
  const int32_t *unigram;
  uint64_t uni_size, mT;
  const uint64_t *bstarts;  // minibatch-vocab mode: run starts of the batch's table [bU+1] (else nullptr)
  const int32_t *buk;       // the batch's vids in std::map key order (the table's word order)
  uint32_t bU;
  const uint64_t *ustarts;  // run-length unigram table + its coarse index (k_build_uidx), or nullptr: read unigram[]
  const int32_t *uidx;
  int ushift;
  uint32_t uV;
  const uint2 *alias;       // SWPS_SAMPLER_ALIAS: {prob bits, alias} per word of the (batch) vocab, else nullptr
  uint32_t alias_n;
  const int32_t *local;
  uint32_t U;
  const uint32_t *vid_row;  // direct table reads (single GPU): slots of pulled keys hold kTabRow | table row
  int32_t *rec;     // [P][RS]: word, ctx x 2W (-1 = none), target x (N+1) (-1 = skipped); each a cache vid
                    // or kTabRow | table row (slot_row)
  uint32_t *pkeys, *pvals;  // position-major: h record (p,d) at p*(N+1)+d; v record (p,j) at (N+1)*P + p*2W+j
  int32_t *trace;
  unsigned long long *rows_touched;
  const int2 *tloc;  // per batch token (from t0): {local key, position-record source} (k_tok_local), or nullptr
  uint64_t t0;
};

// Per token of the batch: its local key and the source its position-record slot holds (kTabRow |
// shard row for a pulled key on a single GPU, else its vid) — looked up once per token, so
// k_records_t reads a position's contexts and word as contiguous entries instead of two random
// lookups each
__global__ void k_tok_local(const int32_t *__restrict__ tok, uint64_t nt, const int32_t *__restrict__ local,
                            const uint32_t *__restrict__ vid_row, int2 *__restrict__ tloc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nt) return;
  const int32_t v = tok[i], u = local[v];
  tloc[i] = make_int2(u, (u >= 0 && vid_row) ? (kTabRow | (int32_t)vid_row[v]) : v);
}

// One thread per kept position: replays learn_instance's LCG draws
// (word2vec_global.h:669,686-691) from the jumped state — b, the negatives
// from the unigram table, the context slots a = b..2W-b (a != W) inside the
// line — and writes the position record plus the (local key, record index)
// gradient records (key U = not in the batch's pulled key set: dropped, as the
// reference's pull reset drops them).
// The [RS]-int position records are built in LDS (thread stride RS) and
// stored by the whole block as one contiguous run: per-thread stores at a
// 4*RS-byte stride wrote partial cache lines (PMC: 1.25 GB written per batch
// for 0.28 GB of records and gradient records).
__global__ __launch_bounds__(256) void k_records(RecArgs a) {
  extern __shared__ int32_t srec[];
  const uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x;
  const uint64_t p = p0 + threadIdx.x;
  const int RS = 2 * a.W + a.N + 2;
  int nctx = 0, ntgt = 0;
  if (p < a.P) {
    const uint64_t P = a.P;
    const int W = a.W, N = a.N;
    const uint64_t HOFF = P * (uint64_t)(N + 1);
    const uint64_t t = (uint64_t)a.pos_tok[p];
    const int32_t l = a.tok_line[t];
    const int64_t ls = a.line_off[l];
    const int n = (int)(a.line_off[l + 1] - ls), pos = (int)((int64_t)t - ls);
    const int32_t word = a.tok[t];
    const uint64_t rank = (uint64_t)(a.kscan[t] - a.kscan[ls]);
    uint64_t x = lcg_jump(a.lstate, a.ldoff[l] + 1 + rank * (uint64_t)(N + 1), kLcgA, kLcgC);
    x = x * kLcgA + kLcgC;
    const int b = (int)fast_mod(x, (uint64_t)W, a.mW);
    int32_t *r = srec + threadIdx.x * RS;
    r[0] = word;
    for (int j = 0; j < 2 * W; j++) {
      int32_t cv = -1;
      if (j < 2 * (W - b)) {
        int aa = b + j;
        if (aa >= W) aa++;
        const int c = pos - W + aa;
        if (c >= 0 && c < n) cv = a.tok[ls + c];
      }
      uint32_t key = a.U;
      int32_t src = cv;
      if (cv >= 0) {
        nctx++;
        const int32_t u = a.local[cv];
        if (u >= 0) {
          key = (uint32_t)u;
          if (a.vid_row) src = kTabRow | (int32_t)a.vid_row[cv];
        }
      }
      r[1 + j] = src;
      const uint64_t k = HOFF + p * (uint64_t)(2 * W) + j;
      a.pkeys[k] = key;
      if (a.pvals) a.pvals[k] = (uint32_t)k;
    }
    for (int d = 0; d <= N; d++) {
      int32_t tv = word;
      if (d > 0) {
        x = x * kLcgA + kLcgC;
        const uint64_t slot = fast_mod(x >> 16, a.uni_size, a.mT);
        if (a.alias) {  // Walker/Vose alias over unigram^0.75: bucket from the LCG's high word; the
                        // coin from a mix of the whole state (the LCG's low bits have short periods)
          const uint32_t bkt = (uint32_t)(((x >> 32) * (uint64_t)a.alias_n) >> 32);
          const uint2 e = a.alias[bkt];
          const float coin = (float)(uint32_t)(splitmix64(x) >> 40) * (1.0f / 16777216.0f);
          const int32_t w = coin < __uint_as_float(e.x) ? (int32_t)bkt : (int32_t)e.y;
          tv = a.bstarts ? a.buk[w] : w;
        } else if (a.bstarts) {  // word2vec.h:398-425 table over the minibatch vocab, run-length form
          uint32_t lo = 0, hi = a.bU;  // largest u with bstarts[u] <= slot
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (a.bstarts[mid] <= slot)
              lo = mid;
            else
              hi = mid;
          }
          tv = a.buk[lo];
        } else if (a.uidx) {
          tv = unigram_lookup(a.ustarts, a.uidx, a.ushift, a.uV, slot);
        } else {
          tv = a.unigram[slot];
        }
        if (a.trace) a.trace[p * N + d - 1] = tv;
        if (tv == word) tv = -1;
      }
      uint32_t key = a.U;
      int32_t src = tv;
      if (tv >= 0) {
        ntgt++;
        const int32_t u = a.local[tv];
        if (u >= 0) {
          key = (uint32_t)u;
          if (a.vid_row) src = kTabRow | (int32_t)a.vid_row[tv];
        }
      }
      r[1 + 2 * W + d] = src;
      const uint64_t k = p * (uint64_t)(N + 1) + d;
      a.pkeys[k] = key;
      if (a.pvals) a.pvals[k] = (uint32_t)k;
    }
  }
  __syncthreads();
  {
    const uint32_t n = (uint32_t)min<uint64_t>(blockDim.x, a.P - min(p0, a.P)) * (uint32_t)RS;
    int32_t *dst = a.rec + p0 * RS;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = srec[i];
  }
  // rows the forward will read (roofline accounting), one atomic per wave
  unsigned long long c = (unsigned long long)nctx, g = (unsigned long long)ntgt;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    c += __shfl_xor(c, off, 64);
    g += __shfl_xor(g, off, 64);
  }
  if (a.rows_touched && (threadIdx.x & 63) == 0 && (c | g)) {  // profiled passes only
    atomicAdd(&a.rows_touched[0], c);
    atomicAdd(&a.rows_touched[1], g);
  }
}

// Main-LCG jump by k draws with per-bit constants (x -> A_i x + C_i jumps
// 2^i draws; powers of one affine map commute): the per-thread doubling loop
// of lcg_jump squared the same (A, C) pairs in every thread.
__constant__ uint64_t c_p2A[64];
__constant__ uint64_t c_p2C[64];
__device__ __forceinline__ uint64_t lcg_jump_p2(uint64_t x, uint64_t k) {
  for (int i = 0; k; i++, k >>= 1)
    if (k & 1) x = c_p2A[i] * x + c_p2C[i];
  return x;
}

// k_records for the common case — compile-time window W and negatives N, the
// reference's table sampler through the coarse index, one global vocab —
// restructured so each thread's independent loads are in flight together
// (all 2W context words, then all their local / row lookups; the N draws
// first, then the N unigram searches advanced in lockstep) instead of one
// dependent chain per slot.  Identical outputs to k_records.
template <int W, int N>
__global__ __launch_bounds__(256) void k_records_t(RecArgs a) {
  extern __shared__ int32_t srec[];
  constexpr int RS = 2 * W + N + 2;
  const uint64_t p0 = (uint64_t)blockIdx.x * blockDim.x;
  const uint64_t p = p0 + threadIdx.x;
  int nctx = 0, ntgt = 0;
  if (p < a.P) {
    const uint64_t P = a.P;
    const uint64_t HOFF = P * (uint64_t)(N + 1);
    const uint64_t t = (uint64_t)a.pos_tok[p];
    const int32_t l = a.tok_line[t];
    const int64_t ls = a.line_off[l];
    const int n = (int)(a.line_off[l + 1] - ls), pos = (int)((int64_t)t - ls);
    const int32_t word = a.tok[t];
    const uint64_t rank = (uint64_t)(a.kscan[t] - a.kscan[ls]);
    uint64_t x = lcg_jump_p2(a.lstate, a.ldoff[l] + 1 + rank * (uint64_t)(N + 1));
    x = x * kLcgA + kLcgC;
    const int b = (int)fast_mod(x, (uint64_t)W, a.mW);
    int32_t *r = srec + threadIdx.x * RS;
    r[0] = word;
    // ---- contexts: a = b .. 2W-b (a != W) inside the line ----
    int32_t cv[2 * W], cu[2 * W], cs[2 * W];
    if (a.tloc) {  // the per-token lookups (k_tok_local): contiguous in the line
#pragma unroll
      for (int j = 0; j < 2 * W; j++) {
        cv[j] = -1;
        cu[j] = -1;
        cs[j] = -1;
        if (j < 2 * (W - b)) {
          int aa = b + j;
          if (aa >= W) aa++;
          const int c = pos - W + aa;
          if (c >= 0 && c < n) {
            const int2 x = a.tloc[(uint64_t)(ls + c) - a.t0];
            cv[j] = 0;  // present (its vid is not needed: cs holds the slot's source)
            cu[j] = x.x;
            cs[j] = x.y;
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 2 * W; j++) {
        cv[j] = -1;
        if (j < 2 * (W - b)) {
          int aa = b + j;
          if (aa >= W) aa++;
          const int c = pos - W + aa;
          if (c >= 0 && c < n) cv[j] = a.tok[ls + c];
        }
      }
#pragma unroll
      for (int j = 0; j < 2 * W; j++) cu[j] = cv[j] >= 0 ? a.local[cv[j]] : -1;
#pragma unroll
      for (int j = 0; j < 2 * W; j++)
        cs[j] = (cu[j] >= 0 && a.vid_row) ? (kTabRow | (int32_t)a.vid_row[cv[j]]) : cv[j];
    }
    // ---- targets: the word, then N draws from the unigram table ----
    uint64_t slot[N + 1];
    uint32_t lo[N + 1], hi[N + 1];
#pragma unroll
    for (int d = 1; d <= N; d++) {
      x = x * kLcgA + kLcgC;
      slot[d] = fast_mod(x >> 16, a.uni_size, a.mT);
      const uint64_t bk = slot[d] >> a.ushift;
      lo[d] = (uint32_t)a.uidx[bk];
      hi[d] = min((uint32_t)a.uidx[bk + 1] + 1u, a.uV);
    }
    for (bool more = true; more;) {  // the N binary searches (unigram_lookup) step together
      more = false;
#pragma unroll
      for (int d = 1; d <= N; d++) {
        if (hi[d] - lo[d] > 1) {
          const uint32_t mid = (lo[d] + hi[d]) >> 1;
          if (a.ustarts[mid] <= slot[d])
            lo[d] = mid;
          else
            hi[d] = mid;
          more |= hi[d] - lo[d] > 1;
        }
      }
    }
    int32_t tv[N + 1];
    tv[0] = word;
#pragma unroll
    for (int d = 1; d <= N; d++) {
      tv[d] = (int32_t)lo[d];
      if (a.trace) a.trace[p * N + d - 1] = tv[d];
      if (tv[d] == word) tv[d] = -1;
    }
    int32_t tu[N + 1];
    int32_t ts[N + 1];
    if (a.tloc) {  // the word itself: its token's entry
      const int2 x = a.tloc[t - a.t0];
      tu[0] = x.x;
      ts[0] = x.y;
    }
#pragma unroll
    for (int d = a.tloc ? 1 : 0; d <= N; d++) tu[d] = tv[d] >= 0 ? a.local[tv[d]] : -1;
#pragma unroll
    for (int d = a.tloc ? 1 : 0; d <= N; d++)
      ts[d] = (tu[d] >= 0 && a.vid_row) ? (kTabRow | (int32_t)a.vid_row[tv[d]]) : tv[d];
    // ---- stores: position record (LDS), gradient records (position-major) ----
#pragma unroll
    for (int j = 0; j < 2 * W; j++) {
      nctx += cv[j] >= 0;
      r[1 + j] = cs[j];
      const uint64_t k = HOFF + p * (uint64_t)(2 * W) + j;
      a.pkeys[k] = cu[j] >= 0 ? (uint32_t)cu[j] : a.U;
      if (a.pvals) a.pvals[k] = (uint32_t)k;
    }
#pragma unroll
    for (int d = 0; d <= N; d++) {
      ntgt += tv[d] >= 0;
      r[1 + 2 * W + d] = ts[d];
      const uint64_t k = p * (uint64_t)(N + 1) + d;
      a.pkeys[k] = tu[d] >= 0 ? (uint32_t)tu[d] : a.U;
      if (a.pvals) a.pvals[k] = (uint32_t)k;
    }
  }
  __syncthreads();
  {
    const uint32_t nn = (uint32_t)min<uint64_t>(blockDim.x, a.P - min(p0, a.P)) * (uint32_t)RS;
    int32_t *dst = a.rec + p0 * RS;
    for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) dst[i] = srec[i];
  }
  unsigned long long c = (unsigned long long)nctx, g = (unsigned long long)ntgt;
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    c += __shfl_xor(c, off, 64);
    g += __shfl_xor(g, off, 64);
  }
  if (a.rows_touched && (threadIdx.x & 63) == 0 && (c | g)) {  // profiled passes only
    atomicAdd(&a.rows_touched[0], c);
    atomicAdd(&a.rows_touched[1], g);
  }
}

// Chunk ci = elements [E*ci, E*ci+E) of a D-element row, held by one lane as
// one register chunk and converted to / from fp64.  16 B of the table type per
// lane; when fp32 rows carry fp64 intermediates (E = 4 doubles) the row is
// stored as two planes [D/2 | D/2] of double2 so every load/store instruction
// of a wave is contiguous.
template <typename X, int E> struct Chk;
template <> struct Chk<float, 4> {
  using R = float4;
  static __device__ __forceinline__ R ld(const float *row, int ci, int) { return ((const float4 *)row)[ci]; }
  static __device__ __forceinline__ double at(const R &r, int k) { return (double)((const float *)&r)[k]; }
  static __device__ __forceinline__ void st(float *row, int ci, int, const double (&v)[4]) {
    ((float4 *)row)[ci] = make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
  }
};
template <> struct Chk<double, 4> {
  struct R {
    double2 a, b;
  };
  static __device__ __forceinline__ R ld(const double *row, int ci, int D) {
    R r;
    r.a = ((const double2 *)row)[ci];
    r.b = ((const double2 *)(row + D / 2))[ci];
    return r;
  }
  static __device__ __forceinline__ double at(const R &r, int k) { return ((const double *)&r)[k]; }
  static __device__ __forceinline__ void st(double *row, int ci, int D, const double (&v)[4]) {
    ((double2 *)row)[ci] = make_double2(v[0], v[1]);
    ((double2 *)(row + D / 2))[ci] = make_double2(v[2], v[3]);
  }
};
template <> struct Chk<double, 2> {
  using R = double2;
  static __device__ __forceinline__ R ld(const double *row, int ci, int) { return ((const double2 *)row)[ci]; }
  static __device__ __forceinline__ double at(const R &r, int k) { return ((const double *)&r)[k]; }
  static __device__ __forceinline__ void st(double *row, int ci, int, const double (&v)[2]) {
    ((double2 *)row)[ci] = make_double2(v[0], v[1]);
  }
};

template <typename T, typename A> struct FwdArgs {
  const int32_t *rec;
  int P;
  const T *cache_h, *cache_v;
  const T *tab;  // the table's rows [cap][4D]: source of rows tagged kTabRow (single-GPU direct reads)
  const float *exptab;
  int D, W, N;
  float alpha;
  A *neu1, *neu1e;
  float *pg;
  int xcd;  // 1: XCD-contiguous block order (xcd_block)
  int ld;   // neu1/neu1e row stride in elements (D rounded up to 128 B: whole cache lines per row)
  int cs;   // worker-cache row stride in elements (the same rounding)
  int full;  // k_forward_t: neu1/neu1e stores cover the row pad (zeros): whole lines (SWPS_FULL_LINES)
};

// Source row of a forward slot: a record entry tagged kTabRow is a row index
// into the table (the batch's pulled keys: the table row IS the value the
// pull would have copied — the push of this batch has not run yet); any other
// entry >= 0 is a vid into the worker cache (stale rows of keys outside the
// batch key set, global_pull_access.h:88-97).
template <typename T, typename A>
__device__ __forceinline__ const T *slot_row(const FwdArgs<T, A> &a, int32_t e, bool ctx) {
  if (e & kTabRow) return a.tab + (uint64_t)(e & ~kTabRow) * 4 * a.D + (ctx ? a.D : 0);
  return (ctx ? a.cache_v : a.cache_h) + (uint64_t)e * a.cs;
}

// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md
// §Workgroup dispatch: b and b+8 share one).  Renumber so each XCD walks one
// contiguous range of positions: neighbouring kept positions share most of
// their context rows (the window slides by one token), so those rows are
// re-read from the XCD's own L2 instead of crossing to HBM/MALL.  A bijection
// on [0, G) for any G; speed only, never correctness.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t G) {
  const uint32_t q = G >> 3, r = G & 7, x = b & 7, i = b >> 3;
  return x * q + min(x, r) + i;
}

// One wave per kept position (the body of learn_instance's position loop,
// word2vec_global.h:663-718).  Context v rows are loaded in groups of G slots
// whose loads are issued together and summed into neu1 in slot order; then
// the targets, up to 8 at a time: their h rows, the 8 per-lane partial dots
// with neu1 (fp64) reduced together (wave_sum8), g from the exp table, and
// neu1e += g*h.  Writes neu1, neu1e (gradient sources) and g.
template <typename T, typename A, int NCH, int G>
__global__ __launch_bounds__(256) void k_forward_b8(FwdArgs<T, A> a) {
  constexpr int E = V16<T>::E;
  using CT = Chk<T, E>;
  using CA = Chk<A, E>;
  const int lane = threadIdx.x & 63;
  const uint32_t blk = a.xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int p = __builtin_amdgcn_readfirstlane((int)(blk * 4 + (threadIdx.x >> 6)));
  if (p >= a.P) return;
  const int D = a.D, W = a.W, N = a.N, NC = D / E;
  const int S = 2 * W + N + 1;  // slots: contexts then targets
  const int32_t *r = a.rec + (uint64_t)p * (S + 1);
  double acc[NCH][E], ne[NCH][E];
#pragma unroll
  for (int c = 0; c < NCH; c++)
#pragma unroll
    for (int k = 0; k < E; k++) {
      acc[c][k] = 0.0;
      ne[c][k] = 0.0;
    }
  // Slots in groups of G whose row loads are issued together: context slots
  // (v rows) add into neu1 in slot order; target slots (h rows) of the group
  // then get their per-lane partial dots with the finished neu1, reduced
  // together (wave_sum8), g from the exp table, and neu1e += g*h.
  static_assert(G == 8, "wave_sum8 reduces eight targets");
  for (int s0 = 0; s0 < S; s0 += G) {
    typename CT::R rows[G][NCH];
    int32_t vid[G];
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int slot = s0 + q;
      vid[q] = slot < S ? r[1 + slot] : -1;
      if (vid[q] >= 0) {
        const T *src = slot_row(a, vid[q], slot < 2 * W);
#pragma unroll
        for (int c = 0; c < NCH; c++) {
          const int ci = lane + c * 64;
          if (ci < NC) rows[q][c] = CT::ld(src, ci, D);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < G; q++) {
      if (s0 + q >= 2 * W || vid[q] < 0) continue;
#pragma unroll
      for (int c = 0; c < NCH; c++)
        if (lane + c * 64 < NC)
#pragma unroll
          for (int k = 0; k < E; k++) acc[c][k] += CT::at(rows[q][c], k);
    }
    if (s0 + G <= 2 * W) continue;  // no target in this group
    double part[G];
    uint32_t tmask = 0;  // wave-uniform: target slots of this group that are present
#pragma unroll
    for (int q = 0; q < G; q++) {
      double pq = 0.0;
      if (s0 + q >= 2 * W && vid[q] >= 0) {
        tmask |= 1u << q;
#pragma unroll
        for (int c = 0; c < NCH; c++)
          if (lane + c * 64 < NC)
#pragma unroll
            for (int k = 0; k < E; k++) {
              const double prod = acc[c][k] * CT::at(rows[q][c], k);
              pq += prod;
            }
      }
      part[q] = pq;
    }
    const double tot = wave_sum8(part, lane);
    // lanes 8q..8q+7 hold slot s0+q's dot: g per learn_instance (word2vec_global.h:693-701)
    const int d = s0 + (lane >> 3) - 2 * W;
    float f = 0;
    f += tot;
    const int label = d == 0 ? 1 : 0;
    float g;
    if (f > 6)
      g = (label - 1) * a.alpha;
    else if (f < -6)
      g = (label - 0) * a.alpha;
    else
      g = (label - a.exptab[(int)((f + 6) * (1000 / 6 / 2))]) * a.alpha;
#pragma unroll
    for (int q = 0; q < G; q++) {
      if (!((tmask >> q) & 1)) continue;
      const float gq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(g), 8 * q));
#pragma unroll
      for (int c = 0; c < NCH; c++)
        if (lane + c * 64 < NC)
#pragma unroll
          for (int k = 0; k < E; k++) {
            const double prod = (double)gq * CT::at(rows[q][c], k);
            ne[c][k] += prod;
          }
    }
    if ((lane & 7) == 0 && d >= 0 && d <= N) a.pg[(uint64_t)p * (N + 1) + d] = (tmask >> (lane >> 3)) & 1 ? g : 0.f;
  }
#pragma unroll
  for (int c = 0; c < NCH; c++) {
    const int ci = lane + c * 64;
    if (ci < NC) {
      CA::st(a.neu1 + (uint64_t)p * a.ld, ci, D, acc[c]);
      CA::st(a.neu1e + (uint64_t)p * a.ld, ci, D, ne[c]);
    }
  }
}

// The form with one wave reduction per target: faster than k_forward_b8 with
// fp32 intermediates (4.3 vs 6.4 ms per 5M-token batch, same box), slower with
// fp64 ones — launch_forward picks per mode.
template <typename T, typename A, int NCH, int G>
__global__ __launch_bounds__(256) void k_forward(FwdArgs<T, A> a) {
  constexpr int E = V16<T>::E;
  using CT = Chk<T, E>;
  using CA = Chk<A, E>;
  const int lane = threadIdx.x & 63;
  const uint32_t blk = a.xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int p = __builtin_amdgcn_readfirstlane((int)(blk * 4 + (threadIdx.x >> 6)));
  if (p >= a.P) return;
  const int D = a.D, W = a.W, N = a.N, NC = D / E;
  const int S = 2 * W + N + 1;  // slots: contexts then targets
  const int32_t *r = a.rec + (uint64_t)p * (S + 1);
  double acc[NCH][E], ne[NCH][E];
#pragma unroll
  for (int c = 0; c < NCH; c++)
#pragma unroll
    for (int k = 0; k < E; k++) {
      acc[c][k] = 0.0;
      ne[c][k] = 0.0;
    }
  float gk = 0.f;
  for (int s0 = 0; s0 < S; s0 += G) {
    typename CT::R rows[G][NCH];
    int32_t vid[G];
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int slot = s0 + q;
      vid[q] = slot < S ? r[1 + slot] : -1;
      if (vid[q] >= 0) {
        const T *src = slot_row(a, vid[q], slot < 2 * W);
#pragma unroll
        for (int c = 0; c < NCH; c++) {
          const int ci = lane + c * 64;
          if (ci < NC) rows[q][c] = CT::ld(src, ci, D);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int slot = s0 + q;
      if (vid[q] < 0) continue;
      if (slot < 2 * W) {
#pragma unroll
        for (int c = 0; c < NCH; c++)
          if (lane + c * 64 < NC)
#pragma unroll
            for (int k = 0; k < E; k++) acc[c][k] += CT::at(rows[q][c], k);
      } else {
        const int d = slot - 2 * W;
        double part = 0.0;
#pragma unroll
        for (int c = 0; c < NCH; c++)
          if (lane + c * 64 < NC)
#pragma unroll
            for (int k = 0; k < E; k++) {
              const double prod = acc[c][k] * CT::at(rows[q][c], k);
              part += prod;
            }
        part = wave_sum_pl(part);
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
#pragma unroll
        for (int c = 0; c < NCH; c++)
          if (lane + c * 64 < NC)
#pragma unroll
            for (int k = 0; k < E; k++) {
              const double prod = (double)g * CT::at(rows[q][c], k);
              ne[c][k] += prod;
            }
        if (lane == d) gk = g;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; c++) {
    const int ci = lane + c * 64;
    if (ci < NC) {
      CA::st(a.neu1 + (uint64_t)p * a.ld, ci, D, acc[c]);
      CA::st(a.neu1e + (uint64_t)p * a.ld, ci, D, ne[c]);
    }
  }
  if (lane <= N) a.pg[(uint64_t)p * (N + 1) + lane] = gk;
}

// Fast mode (fp32 rows, fp32 intermediates) when D = 256*NCH + tail with
// 0 < tail <= 64 (D = 300: one float4 chunk + a 44-lane float tail): a lane's
// slice of a row is NCH float4 + one float, 5 registers per row at D = 300
// instead of the 8 two whole float4 chunks take, so more rows are in flight
// per CU.  Same memory layout (natural element order) as the chunked form.
template <int NCH> struct FSlice {
  float4 v[NCH];
  float t;
  __device__ __forceinline__ void ld(const float *row, int lane, bool tl) {
#pragma unroll
    for (int c = 0; c < NCH; c++) v[c] = ((const float4 *)row)[lane + c * 64];
    t = row[256 * NCH + (tl ? lane : 0)];  // lanes past the tail load a valid duplicate: no branch
  }
  __device__ __forceinline__ void st(float *row, int lane, bool tl) const {
#pragma unroll
    for (int c = 0; c < NCH; c++) ((float4 *)row)[lane + c * 64] = v[c];
    if (tl) row[256 * NCH + lane] = t;
  }
  // the same into a row of ld >= D elements whose pad (elements D..ld) is written as zeros:
  // whole-line stores (a partial last line is a masked write that HBM completes as a
  // read-modify-write of its ECC word; measured on the cache rows: pull 0.19 -> 0.16 ms)
  __device__ __forceinline__ void st_full(float *row, int lane, bool tl, int ld) const {
#pragma unroll
    for (int c = 0; c < NCH; c++) ((float4 *)row)[lane + c * 64] = v[c];
    if (256 * NCH + lane < ld) row[256 * NCH + lane] = tl ? t : 0.f;
  }
};
template <int NCH> struct FAcc {
  double v[NCH][4];
  double t;
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
      for (int k = 0; k < 4; k++) v[c][k] = 0.0;
    t = 0.0;
  }
  __device__ __forceinline__ void add(const FSlice<NCH> &r, bool tl) {
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      v[c][0] += (double)r.v[c].x;
      v[c][1] += (double)r.v[c].y;
      v[c][2] += (double)r.v[c].z;
      v[c][3] += (double)r.v[c].w;
    }
    t += (double)r.t;  // garbage past the tail is never stored nor dotted
  }
  __device__ __forceinline__ void axpy(double g, const FSlice<NCH> &r, bool tl) {
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const double p0 = g * (double)r.v[c].x, p1 = g * (double)r.v[c].y, p2 = g * (double)r.v[c].z,
                   p3 = g * (double)r.v[c].w;
      v[c][0] += p0;
      v[c][1] += p1;
      v[c][2] += p2;
      v[c][3] += p3;
    }
    const double p = g * (double)r.t;
    t += p;
  }
  __device__ __forceinline__ double dot(const FSlice<NCH> &r, bool tl) const {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const double p0 = v[c][0] * (double)r.v[c].x, p1 = v[c][1] * (double)r.v[c].y,
                   p2 = v[c][2] * (double)r.v[c].z, p3 = v[c][3] * (double)r.v[c].w;
      s += p0;
      s += p1;
      s += p2;
      s += p3;
    }
    const double p = t * (double)r.t;
    s += tl ? p : 0.0;
    return s;
  }
  __device__ __forceinline__ void st(float *row, int lane, bool tl) const {
#pragma unroll
    for (int c = 0; c < NCH; c++)
      ((float4 *)row)[lane + c * 64] = make_float4((float)v[c][0], (float)v[c][1], (float)v[c][2], (float)v[c][3]);
    if (tl) row[256 * NCH + lane] = (float)t;
  }
  __device__ __forceinline__ void st_full(float *row, int lane, bool tl, int ld) const {  // FSlice::st_full
#pragma unroll
    for (int c = 0; c < NCH; c++)
      ((float4 *)row)[lane + c * 64] = make_float4((float)v[c][0], (float)v[c][1], (float)v[c][2], (float)v[c][3]);
    if (256 * NCH + lane < ld) row[256 * NCH + lane] = tl ? (float)t : 0.f;
  }
};

// k_forward (fast mode) on FSlice rows.
template <int NCH, int G, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_forward_t(FwdArgs<float, float> a) {
  const int lane = threadIdx.x & 63;
  const uint32_t blk = a.xcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int p = __builtin_amdgcn_readfirstlane((int)(blk * 4 + (threadIdx.x >> 6)));
  if (p >= a.P) return;
  const int D = a.D, W = a.W, N = a.N;
  const bool tl = 256 * NCH + lane < D;
  const int S = 2 * W + N + 1;  // slots: contexts then targets
  const int32_t *r = a.rec + (uint64_t)p * (S + 1);
  FAcc<NCH> acc, ne;
  acc.zero();
  ne.zero();
  float gk = 0.f;
  for (int s0 = 0; s0 < S; s0 += G) {
    FSlice<NCH> rows[G];
    int32_t vid[G];
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int slot = s0 + q;
      vid[q] = __builtin_amdgcn_readfirstlane(slot < S ? r[1 + slot] : -1);
      if (vid[q] >= 0) rows[q].ld(slot_row(a, vid[q], slot < 2 * W), lane, tl);
    }
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int slot = s0 + q;
      if (vid[q] < 0) continue;
      if (slot < 2 * W) {
        acc.add(rows[q], tl);
      } else {
        const int d = slot - 2 * W;
        const double part = wave_sum_pl(acc.dot(rows[q], tl));
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
        ne.axpy((double)g, rows[q], tl);
        if (lane == d) gk = g;
      }
    }
  }
  acc.st_full(a.neu1 + (uint64_t)p * a.ld, lane, tl, a.full ? a.ld : a.D);
  ne.st_full(a.neu1e + (uint64_t)p * a.ld, lane, tl, a.full ? a.ld : a.D);
  if (lane <= N) a.pg[(uint64_t)p * (N + 1) + lane] = gk;
}

constexpr uint32_t kGroupDesc = 16;  // = kGroup (k_combine's group size)

// item descriptors {first record, end record | kind << 31, (key, kind) index j, chunk}:
// one thread per item (hot keys have thousands of chunks), j found by binary
// search over the item offsets ioff[0..2U].
struct MultiOrder {  // k_item_desc: sort keys of the multi-chunk items by their first record's position
  uint32_t *key, *item;  // [max_items]: coarse position (kMultiPad for the rest) and item index; null = unsorted
  const uint32_t *vals;  // the sorted records
  uint32_t SH, SV;  // record slots per position: N+1 targets (h), 2W contexts (v)
  uint64_t HOFF;
  int shift;  // coarse position = p >> shift (< kMultiPad)
};
constexpr uint32_t kMultiPad = 0xFFFFu;  // 16-bit sort keys: items outside the multi list sort last

// the (key, kind) run of every item without a search: each run with items marks its first item
// (run_of zeroed before), then an inclusive max-scan carries the mark over the run's other items
__global__ void k_item_heads(const uint32_t *__restrict__ ioff, uint32_t R, uint32_t *__restrict__ run_of) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= R) return;
  const uint32_t a = ioff[j];
  if (ioff[j + 1] > a) run_of[a] = j;
}

__global__ void k_item_desc(const uint32_t *__restrict__ seg, const uint32_t *__restrict__ ioff, uint32_t U,
                            uint32_t CH, uint32_t CHM, uint64_t max_items, uint4 *__restrict__ desc, uint32_t *__restrict__ lead,
                            uint32_t *__restrict__ multi, MultiOrder mo, const uint32_t *__restrict__ run_of = nullptr) {
  const uint64_t item = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = item < max_items && item < ioff[2ull * U];
  uint32_t lo = 0, hi = 2 * U;  // largest j with ioff[j] <= item
  if (live && run_of)
    lo = run_of[item];
  else if (live)
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (ioff[mid] <= item)
        lo = mid;
      else
        hi = mid;
    }
  if (multi) {
    // items of (key, kind) runs with more than one chunk, for k_gather_t when
    // k_push_tg sums the single-chunk runs itself (list order is irrelevant:
    // every item writes only its own partial slot); one atomic per wave
    const bool m = live && ioff[lo + 1] - ioff[lo] > 1;
    if (mo.key && item < max_items) {
      uint32_t key = kMultiPad;
      if (m) {  // the chunk's first record: index p*SH + d (h), HOFF + p*SV + j (v)
        const uint32_t jj = lo, u = jj >> 1, kind = jj & 1, k = (uint32_t)item - ioff[jj];
        const uint32_t pi = mo.vals[seg[(2 * kind) * U + u] + k * CHM];
        key = (kind ? (uint32_t)((uint64_t)pi - mo.HOFF) / mo.SV : pi / mo.SH) >> mo.shift;
      }
      mo.key[item] = key;
      mo.item[item] = (uint32_t)item;
    }
    const uint64_t bal = __ballot(m);
    if (bal) {
      const int lane = threadIdx.x & 63;
      const int first = __ffsll((long long)bal) - 1;
      uint32_t base = 0;
      if (lane == first) base = atomicAdd(&multi[0], (uint32_t)__popcll(bal));
      base = (uint32_t)__shfl((int)base, first, 64);
      if (m && !mo.key) multi[1 + base + (uint32_t)__popcll(bal & ((1ULL << lane) - 1))] = (uint32_t)item;
    }
  }
  if (!live) return;
  const uint32_t jj = lo, u = jj >> 1, kind = jj & 1, k = (uint32_t)item - ioff[jj];
  const uint32_t s = seg[(2 * kind) * U + u], e = seg[(2 * kind + 1) * U + u];
  const uint32_t ck = ioff[jj + 1] - ioff[jj] > 1 ? CHM : CH;  // single-item runs hold up to CH records
  const uint32_t cs = s + k * ck;
  desc[item] = make_uint4(cs, min(cs + ck, e) | (kind << 31), jj, k);
  // hot (key, kind) runs of more than kGroup chunks: k_combine pre-sums each
  // group of kGroup partials into its leader (the list order does not
  // matter: every leader writes only its own slot)
  if (lead && ioff[jj + 1] - ioff[jj] > kGroupDesc && k % kGroupDesc == 0) lead[1 + atomicAdd(&lead[0], 1u)] = (uint32_t)item;
}

template <typename A> struct GatherArgs {
  const uint4 *desc;
  const uint32_t *ioff, *vals;
  uint32_t U;
  const A *neu1, *neu1e;
  const float *pg;
  uint64_t HOFF;
  uint32_t P;
  int D;
  A *partial;
  int ld;  // neu1/neu1e row stride (FwdArgs::ld)
  const uint32_t *lead;  // hot-group leaders (k_item_desc): [0] = count, then items
  uint32_t max_items;    // capacity of desc / partial: a bound on ioff[2U] every reader clamps to
  const uint32_t *multi;  // k_gather_t: only these items ([0] = count; the multi-chunk runs'), or null = all
  uint32_t SH, SV;        // record slots per position: N+1 (h records), 2W (v records)
  const uint32_t *order;  // k_gather: all items in this order ([1..]: the multi-item sort's output), or null
};

// One wave per chunk of <= 128 records of one (key, kind): the fp64 sum, in
// record (= position) order, of g*neu1[p] (h records: accu_h(g*neu1),
// word2vec_global.h:705) or neu1e[p] (v records: accu_v(neu1e), :716).
// Record indices and g are loaded for the whole chunk up front; rows are
// fetched UNR at a time.
template <typename T, typename A, int NCH, int UNR>
__global__ __launch_bounds__(256) void k_gather(GatherArgs<A> a) {
  constexpr int E = V16<T>::E;
  using CA = Chk<A, E>;
  const int lane = threadIdx.x & 63;
  const int NC = a.D / E;
  const uint32_t NI = min(a.ioff[2 * a.U], a.max_items);
  for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < NI; q += gridDim.x * 4) {
    // the multi-chunk items first, in first-record position order (Infinity-Cache reuse), then the rest
    const uint32_t item = a.order ? __builtin_amdgcn_readfirstlane(a.order[1 + q]) : q;
    const uint4 d = a.desc[__builtin_amdgcn_readfirstlane(item)];
    const uint32_t s = d.x, e = d.y & 0x7FFFFFFFu, kind = d.y >> 31, n = e - s;
    uint32_t p0 = 0, p1 = 0;
    float g0 = 1.f, g1 = 1.f;
    // records are position-major: index = p*SH + d (h), HOFF + p*SV + j (v)
    if (lane < (int)n) {
      const uint32_t pi = a.vals[s + lane];
      if (kind == 0) {
        p0 = pi / a.SH;
        g0 = a.pg[pi];
      } else {
        p0 = (uint32_t)(pi - a.HOFF) / a.SV;
      }
    }
    if (lane + 64 < (int)n) {
      const uint32_t pi = a.vals[s + 64 + lane];
      if (kind == 0) {
        p1 = pi / a.SH;
        g1 = a.pg[pi];
      } else {
        p1 = (uint32_t)(pi - a.HOFF) / a.SV;
      }
    }
    const A *base = kind == 0 ? a.neu1 : a.neu1e;
    double acc[NCH][E];
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
      for (int k = 0; k < E; k++) acc[c][k] = 0.0;
    for (uint32_t r0 = 0; r0 < n; r0 += UNR) {
      typename CA::R rv[UNR][NCH];
      double gg[UNR];
#pragma unroll
      for (int q = 0; q < UNR; q++) {
        const uint32_t idx = min(r0 + q, n - 1);
        const uint32_t pr = idx < 64 ? __shfl(p0, (int)idx, 64) : __shfl(p1, (int)(idx - 64), 64);
        gg[q] = (double)(idx < 64 ? __shfl(g0, (int)idx, 64) : __shfl(g1, (int)(idx - 64), 64));
        const A *src = base + (uint64_t)pr * a.ld;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
          const int ci = lane + c * 64;
          if (ci < NC) rv[q][c] = CA::ld(src, ci, a.D);
        }
      }
#pragma unroll
      for (int q = 0; q < UNR; q++) {
        if (r0 + q < n) {
#pragma unroll
          for (int c = 0; c < NCH; c++)
            if (lane + c * 64 < NC)
#pragma unroll
              for (int k = 0; k < E; k++) {
                if (kind == 0) {
                  const double prod = gg[q] * CA::at(rv[q][c], k);
                  acc[c][k] += prod;
                } else {
                  acc[c][k] += CA::at(rv[q][c], k);
                }
              }
        }
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const int ci = lane + c * 64;
      if (ci < NC) CA::st(a.partial + (uint64_t)item * a.D, ci, a.D, acc[c]);
    }
  }
}

// Record info of one gather item: position and g of its records 0..127
// (lanes hold records lane and 64+lane).
struct ItemRecs {
  uint32_t p0, p1;
  float g0, g1;
};
__device__ __forceinline__ uint4 uniform4(uint4 d) {  // wave-uniform value: keep its branches scalar
  return make_uint4(__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                    __builtin_amdgcn_readfirstlane(d.z), __builtin_amdgcn_readfirstlane(d.w));
}

__device__ __forceinline__ ItemRecs run_recs(const uint32_t *vals, const float *pg, uint32_t SH, uint32_t SV,
                                             uint64_t HOFF, uint32_t s, uint32_t n, uint32_t kind, int lane) {
  ItemRecs r{0, 0, 1.f, 1.f};
  // records are position-major: index = p*SH + d (h), HOFF + p*SV + j (v)
  if (lane < (int)n) {
    const uint32_t pi = vals[s + lane];
    if (kind == 0) {
      r.p0 = pi / SH;
      r.g0 = pg[pi];
    } else {
      r.p0 = (uint32_t)(pi - HOFF) / SV;
    }
  }
  if (lane + 64 < (int)n) {
    const uint32_t pi = vals[s + 64 + lane];
    if (kind == 0) {
      r.p1 = pi / SH;
      r.g1 = pg[pi];
    } else {
      r.p1 = (uint32_t)(pi - HOFF) / SV;
    }
  }
  return r;
}

__device__ __forceinline__ ItemRecs item_recs(const GatherArgs<float> &a, uint4 d, int lane) {
  const uint32_t s = d.x, e = d.y & 0x7FFFFFFFu, kind = d.y >> 31, n = e - s;
  return run_recs(a.vals, a.pg, a.SH, a.SV, a.HOFF, s, n, kind, lane);
}

// k_gather (fast mode) on FSlice rows, software-pipelined across items: most
// items are short (Zipf tail keys: a few records), so the next item's
// descriptor and record info are fetched while this item's rows are in flight
// instead of after them (desc -> vals -> pg -> rows was four dependent
// memory round trips per item).
template <int NCH, int UNR>
__global__ __launch_bounds__(256) void k_gather_t(GatherArgs<float> a) {
  const int lane = threadIdx.x & 63;
  const bool tl = 256 * NCH + lane < a.D;
  const uint32_t NI = min(a.multi ? a.multi[0] : a.ioff[2 * a.U], a.max_items);
  const uint32_t stride = gridDim.x * 4;
  uint32_t qi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= NI) return;
  // the multi-chunk items only (fused push), or every item in multi-first position order, or item order
  const uint32_t *list = a.multi ? a.multi : a.order;
  auto item_at = [&](uint32_t q) { return list ? list[1 + __builtin_amdgcn_readfirstlane(q)] : q; };
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
    FAcc<NCH> acc;
    acc.zero();
    ItemRecs rn;
    for (uint32_t r0 = 0; r0 < n; r0 += UNR) {
      FSlice<NCH> rv[UNR];
      double gg[UNR];
#pragma unroll
      for (int q = 0; q < UNR; q++) {
        const uint32_t idx = min(r0 + q, n - 1);
        // idx is wave-uniform: read the record's position and g with v_readlane (scalar results)
        const uint32_t pr = idx < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)ri.p0, (int)idx)
                                     : (uint32_t)__builtin_amdgcn_readlane((int)ri.p1, (int)(idx - 64));
        gg[q] = (double)__int_as_float(idx < 64 ? __builtin_amdgcn_readlane(__float_as_int(ri.g0), (int)idx)
                                                : __builtin_amdgcn_readlane(__float_as_int(ri.g1), (int)(idx - 64)));
        rv[q].ld(base + (uint64_t)pr * a.ld, lane, tl);
      }
      if (r0 == 0) rn = item_recs(a, dn, lane);  // next item's record info, behind this item's first rows
#pragma unroll
      for (int q = 0; q < UNR; q++) {
        if (r0 + q < n) {
          if (kind == 0)
            acc.axpy(gg[q], rv[q], tl);
          else
            acc.add(rv[q], tl);
        }
      }
    }
    if (n == 0) rn = item_recs(a, dn, lane);
    acc.st(a.partial + (uint64_t)item * a.D, lane, tl);
    if (!more) break;
    qi = qn;
    item = nx;
    d = dn;
    ri = rn;
  }
}

constexpr uint32_t kGroup = 16;  // hot keys: partials are pre-summed in groups of 16
// k_combine: a stride loop over the leader list k_item_desc collected
constexpr unsigned kCombineGrid = 1024;

// Hot (key, kind) runs with more than kGroup chunks: each group leader sums
// its group's partials in chunk order into its own slot (second level).
template <typename T, typename A, int NCH>
__global__ __launch_bounds__(256) void k_combine(GatherArgs<A> a) {
  constexpr int E = V16<T>::E;
  using CA = Chk<A, E>;
  const int lane = threadIdx.x & 63;
  const int NC = a.D / E;
  const uint32_t NL = min(a.lead[0], a.max_items / 8 + 1);
  for (uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6); q < NL; q += gridDim.x * 4) {
    const uint32_t item = a.lead[1 + __builtin_amdgcn_readfirstlane(q)];
    const uint4 d = a.desc[__builtin_amdgcn_readfirstlane(item)];
    const uint32_t j = d.z;
    const uint32_t i1 = a.ioff[j + 1];
    const uint32_t end = min(item + kGroup, i1);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const int ci = lane + c * 64;
      if (ci >= NC) continue;
      typename CA::R rv[kGroup];
#pragma unroll
      for (uint32_t q2 = 0; q2 < kGroup; q2++) rv[q2] = CA::ld(a.partial + (uint64_t)min(item + q2, end - 1) * a.D, ci, a.D);
      double sum[E];
#pragma unroll
      for (int kk = 0; kk < E; kk++) sum[kk] = 0.0;
#pragma unroll
      for (uint32_t q2 = 0; q2 < kGroup; q2++)
        if (item + q2 < end)
#pragma unroll
          for (int kk = 0; kk < E; kk++) sum[kk] += CA::at(rv[q2], kk);
      CA::st(a.partial + (uint64_t)item * a.D, ci, a.D, sum);
    }
  }
}

constexpr int kMaxSplitOwners = 64;
template <typename T, typename A> struct PushArgs {
  const int32_t *K;
  uint32_t U;
  const uint32_t *vid_row, *seg, *ioff;
  const A *partial;
  T *rows;
  int32_t *local;
  int D;
  double lr, fudge;
  A *grads;  // TO_GRADS: mean gradients [U][2D] in the intermediate type (the push request payload)
  T *cache_h, *cache_v;  // direct table reads (single GPU): every pushed key's pre-update h, v rows go to
  int cs;                // the worker cache (the value its pull would have left there), row stride cs
  // k_push_tg: the sorted records and the forward's rows, to sum single-chunk runs in place
  const uint32_t *vals;
  const float *pg;
  const A *neu1, *neu1e;
  uint64_t HOFF;
  uint32_t P;
  int ld;
  const uint32_t *krow;  // k_push_thp: shard row per batch key (k_batch_setup)
  uint32_t SH, SV;       // record slots per position (GatherArgs)
  int full;              // cache-row stores cover the pad too (zeros): SWPS_FULL_LINES
  // k_push_thp<TO_GRADS> in two passes (sharded learner, world > 1): pass 1 = the first
  // ohalf[r] keys of every owner r's key range [obnd[r], obnd[r+1]) (K is grouped by owner),
  // pass 2 = the rest; 0 = every key.  Their all-to-alls then overlap pass 2.
  uint32_t group;  // runs of more than `group` partials read k_combine's group leaders (kGroup), else all
  int gpass;
  uint32_t nown;
  uint32_t obnd[kMaxSplitOwners + 1], ohalf[kMaxSplitOwners];
};

// Mean gradient (word2vec_global.h:122-134) + AdaGrad ascent
// (word2vec_global.h:176-185) per key, fp64 math; one wave per key.
// TO_GRADS: stop at the mean and write the push payload (sharded mode: the
// owner GPU applies AdaGrad, see swps_w2v_serve_push).
template <typename T, typename A, int NCH, bool TO_GRADS>
__global__ __launch_bounds__(256) void k_push(PushArgs<T, A> a) {
  constexpr int E = V16<T>::E;
  using CT = Chk<T, E>;
  using CA = Chk<A, E>;
  constexpr int PU = 8;
  const int lane = threadIdx.x & 63;
  const int D = a.D, NC = D / E;
  for (uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < a.U; u += (uint64_t)gridDim.x * 4) {
    const int32_t vid = a.K[u];
    if (lane == 0) a.local[vid] = -1;
    const uint32_t hc = a.seg[1 * a.U + u] - a.seg[0 * a.U + u];
    const uint32_t vc = a.seg[3 * a.U + u] - a.seg[2 * a.U + u];
    if (hc == 0 && vc == 0 && !TO_GRADS && !a.cache_h) continue;
    T *row = TO_GRADS ? nullptr : a.rows + (uint64_t)a.vid_row[vid] * 4 * D;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const int ci = lane + c * 64;
      if (ci >= NC) continue;
      for (int half = 0; half < 2; half++) {
        const uint32_t cnt = half ? vc : hc;
        if (!TO_GRADS && a.cache_h) {  // the pulled (pre-update) value stays in the worker cache
          using V = typename V16<T>::V;
          ((V *)((half ? a.cache_v : a.cache_h) + (uint64_t)vid * a.cs))[ci] = ((const V *)(row + half * D))[ci];
        }
        if (cnt == 0) {
          if (TO_GRADS)
#pragma unroll
            for (int k = 0; k < E; k++) a.grads[u * 2 * D + half * D + ci * E + k] = (A)0;
          continue;
        }
        const uint32_t i0 = a.ioff[2 * u + half], i1 = a.ioff[2 * u + half + 1];
        const uint32_t stride = (i1 - i0) > a.group ? kGroup : 1;
        double sum[E];
#pragma unroll
        for (int k = 0; k < E; k++) sum[k] = 0.0;
        for (uint32_t it0 = i0; it0 < i1; it0 += PU * stride) {
          typename CA::R pv[PU];
#pragma unroll
          for (int q = 0; q < PU; q++) {
            const uint32_t it = min(it0 + q * stride, i1 - 1);
            pv[q] = CA::ld(a.partial + (uint64_t)it * D, ci, D);
          }
#pragma unroll
          for (int q = 0; q < PU; q++)
            if (it0 + q * stride < i1)
#pragma unroll
              for (int k = 0; k < E; k++) sum[k] += CA::at(pv[q], k);
        }
        if (TO_GRADS) {
#pragma unroll
          for (int k = 0; k < E; k++) a.grads[u * 2 * D + half * D + ci * E + k] = (A)(sum[k] / (double)cnt);
          continue;
        }
        T *w = row + half * D, *w2 = row + (2 + half) * D;
        const typename CT::R wr = CT::ld(w, ci, D), w2r = CT::ld(w2, ci, D);
        double wn[E], w2n[E];
#pragma unroll
        for (int k = 0; k < E; k++) {
          const double g = (double)(A)(sum[k] / (double)cnt);  // the mean in the push payload's type
          const double gsq = g * g;
          const double acc2 = CT::at(w2r, k) + gsq;
          const double step = (g * a.lr) / sqrt(acc2 + a.fudge);
          w2n[k] = acc2;
          wn[k] = CT::at(wr, k) + step;
        }
        CT::st(w2, ci, D, w2n);
        CT::st(w, ci, D, wn);
      }
    }
  }
}

// k_push (fast mode, fp32 rows and partials, single GPU) on FSlice rows: both
// halves' first partial and their w / w2 rows are loaded together before any
// arithmetic (k_push walks chunk x half with a dependent load -> store round
// trip each, and its second 64-lane chunk keeps 11 lanes busy at D = 300).
// Same per-element arithmetic and partial order as k_push: bit-identical.
template <int NCH>
__global__ __launch_bounds__(256) void k_push_t(PushArgs<float, float> a) {
  constexpr int PU = 8;
  const int lane = threadIdx.x & 63;
  const int D = a.D;
  const bool tl = 256 * NCH + lane < D;
  for (uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < a.U; u += (uint64_t)gridDim.x * 4) {
    const int32_t vid = a.K[u];
    if (lane == 0) a.local[vid] = -1;
    const uint32_t s0 = a.seg[0 * a.U + u], s1 = a.seg[1 * a.U + u], s2 = a.seg[2 * a.U + u], s3 = a.seg[3 * a.U + u];
    const uint32_t cnt[2] = {s1 - s0, s3 - s2};
    if (cnt[0] == 0 && cnt[1] == 0 && !a.cache_h) continue;
    float *row = a.rows + (uint64_t)a.vid_row[vid] * 4 * D;
    uint32_t i0[2], i1[2];
    FSlice<NCH> wr[2], w2r[2], pf[2];
#pragma unroll
    for (int half = 0; half < 2; half++) {
      i0[half] = a.ioff[2 * u + half];
      i1[half] = a.ioff[2 * u + half + 1];
      if (cnt[half] || a.cache_h) wr[half].ld(row + half * D, lane, tl);
      if (cnt[half]) {
        pf[half].ld(a.partial + (uint64_t)i0[half] * D, lane, tl);
        w2r[half].ld(row + (2 + half) * D, lane, tl);
      }
    }
    if (a.cache_h) {  // the pulled (pre-update) value stays in the worker cache
      wr[0].st_full(a.cache_h + (uint64_t)vid * a.cs, lane, tl, a.full ? a.cs : D);
      wr[1].st_full(a.cache_v + (uint64_t)vid * a.cs, lane, tl, a.full ? a.cs : D);
    }
#pragma unroll
    for (int half = 0; half < 2; half++) {
      if (cnt[half] == 0) continue;
      FAcc<NCH> acc;
      acc.zero();
      acc.add(pf[half], tl);
      const uint32_t stride = (i1[half] - i0[half]) > a.group ? kGroup : 1;
      for (uint32_t it0 = i0[half] + stride; it0 < i1[half]; it0 += PU * stride) {
        FSlice<NCH> pv[PU];
#pragma unroll
        for (int q = 0; q < PU; q++)
          pv[q].ld(a.partial + (uint64_t)min(it0 + q * stride, i1[half] - 1) * D, lane, tl);
#pragma unroll
        for (int q = 0; q < PU; q++)
          if (it0 + q * stride < i1[half]) acc.add(pv[q], tl);
      }
      const double inv = (double)cnt[half];
      float *w = row + half * D, *w2 = row + (2 + half) * D;
      auto upd = [&](double sum, float wv, float w2v, float &wo, float &w2o) {
        const double g = (double)(float)(sum / inv);  // the mean in the push payload's type
        const double acc2 = (double)w2v + g * g;
        const double step = (g * a.lr) / sqrt(acc2 + a.fudge);
        w2o = (float)acc2;
        wo = (float)((double)wv + step);
      };
#pragma unroll
      for (int c = 0; c < NCH; c++) {
        float4 wo, w2o;
        upd(acc.v[c][0], wr[half].v[c].x, w2r[half].v[c].x, wo.x, w2o.x);
        upd(acc.v[c][1], wr[half].v[c].y, w2r[half].v[c].y, wo.y, w2o.y);
        upd(acc.v[c][2], wr[half].v[c].z, w2r[half].v[c].z, wo.z, w2o.z);
        upd(acc.v[c][3], wr[half].v[c].w, w2r[half].v[c].w, wo.w, w2o.w);
        ((float4 *)w2)[lane + c * 64] = w2o;
        ((float4 *)w)[lane + c * 64] = wo;
      }
      if (tl) {
        float wo, w2o;
        upd(acc.t, wr[half].t, w2r[half].t, wo, w2o);
        w2[256 * NCH + lane] = w2o;
        w[256 * NCH + lane] = wo;
      }
    }
  }
}

// k_push_t with the gather of single-chunk runs folded in: a (key, kind) run of
// at most kChunk records is summed here, straight from the forward's neu1 /
// neu1e rows (the same fp64 sum in record order, rounded to the fp32 partial
// it would have stored), so k_gather_t only runs the multi-chunk items and
// the single-chunk partials are never written nor re-read.  Bit-identical to
// k_gather_t + k_combine + k_push_t.
template <int NCH, int UNR, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_push_tg(PushArgs<float, float> a) {
  constexpr int PU = 8;
  const int lane = threadIdx.x & 63;
  const int D = a.D;
  const bool tl = 256 * NCH + lane < D;
  for (uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < a.U; u += (uint64_t)gridDim.x * 4) {
    const int32_t vid = a.K[u];
    if (lane == 0) a.local[vid] = -1;
    const uint32_t sg[4] = {a.seg[0 * a.U + u], a.seg[1 * a.U + u], a.seg[2 * a.U + u], a.seg[3 * a.U + u]};
    const uint32_t cnt[2] = {sg[1] - sg[0], sg[3] - sg[2]};
    if (cnt[0] == 0 && cnt[1] == 0 && !a.cache_h) continue;
    float *row = a.rows + (uint64_t)a.vid_row[vid] * 4 * D;
    uint32_t i0[2], i1[2];
    bool one[2];
    FSlice<NCH> wr[2], w2r[2], pf[2];
    ItemRecs ri[2];
#pragma unroll
    for (int half = 0; half < 2; half++) {
      i0[half] = a.ioff[2 * u + half];
      i1[half] = a.ioff[2 * u + half + 1];
      one[half] = i1[half] - i0[half] == 1;
      if (cnt[half] || a.cache_h) wr[half].ld(row + half * D, lane, tl);
      if (cnt[half]) {
        if (one[half])
          ri[half] = run_recs(a.vals, a.pg, a.SH, a.SV, a.HOFF, sg[2 * half], cnt[half], half, lane);
        else
          pf[half].ld(a.partial + (uint64_t)i0[half] * D, lane, tl);
        w2r[half].ld(row + (2 + half) * D, lane, tl);
      }
    }
    if (a.cache_h) {  // the pulled (pre-update) value stays in the worker cache
      wr[0].st_full(a.cache_h + (uint64_t)vid * a.cs, lane, tl, a.full ? a.cs : D);
      wr[1].st_full(a.cache_v + (uint64_t)vid * a.cs, lane, tl, a.full ? a.cs : D);
    }
#pragma unroll
    for (int half = 0; half < 2; half++) {
      if (cnt[half] == 0) continue;
      FAcc<NCH> acc;
      acc.zero();
      if (one[half]) {
        const uint32_t n = cnt[half];
        const float *base = half == 0 ? a.neu1 : a.neu1e;
        FAcc<NCH> c;
        c.zero();
        for (uint32_t r0 = 0; r0 < n; r0 += UNR) {
          FSlice<NCH> rv[UNR];
          float gf[UNR];
#pragma unroll
          for (int q = 0; q < UNR; q++) {
            const uint32_t idx = min(r0 + q, n - 1);
            const uint32_t pr = idx < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)ri[half].p0, (int)idx)
                                         : (uint32_t)__builtin_amdgcn_readlane((int)ri[half].p1, (int)(idx - 64));
            gf[q] = __int_as_float(idx < 64
                                               ? __builtin_amdgcn_readlane(__float_as_int(ri[half].g0), (int)idx)
                                               : __builtin_amdgcn_readlane(__float_as_int(ri[half].g1), (int)(idx - 64)));
            rv[q].ld(base + (uint64_t)pr * a.ld, lane, tl);
          }
#pragma unroll
          for (int q = 0; q < UNR; q++) {
            if (r0 + q < n) {
              if (half == 0)
                c.axpy((double)gf[q], rv[q], tl);
              else
                c.add(rv[q], tl);
            }
          }
        }
#pragma unroll
        for (int cc = 0; cc < NCH; cc++)
#pragma unroll
          for (int k = 0; k < 4; k++) acc.v[cc][k] = (double)(float)c.v[cc][k];  // the fp32 partial
        acc.t = (double)(float)c.t;
      } else {
        acc.add(pf[half], tl);
        const uint32_t stride = (i1[half] - i0[half]) > a.group ? kGroup : 1;
        for (uint32_t it0 = i0[half] + stride; it0 < i1[half]; it0 += PU * stride) {
          FSlice<NCH> pv[PU];
#pragma unroll
          for (int q = 0; q < PU; q++)
            pv[q].ld(a.partial + (uint64_t)min(it0 + q * stride, i1[half] - 1) * D, lane, tl);
#pragma unroll
          for (int q = 0; q < PU; q++)
            if (it0 + q * stride < i1[half]) acc.add(pv[q], tl);
        }
      }
      const double inv = (double)cnt[half];
      float *w = row + half * D, *w2 = row + (2 + half) * D;
      auto upd = [&](double sum, float wv, float w2v, float &wo, float &w2o) {
        const double g = (double)(float)(sum / inv);  // the mean in the push payload's type
        const double acc2 = (double)w2v + g * g;
        const double step = (g * a.lr) / sqrt(acc2 + a.fudge);
        w2o = (float)acc2;
        wo = (float)((double)wv + step);
      };
#pragma unroll
      for (int c = 0; c < NCH; c++) {
        float4 wo, w2o;
        upd(acc.v[c][0], wr[half].v[c].x, w2r[half].v[c].x, wo.x, w2o.x);
        upd(acc.v[c][1], wr[half].v[c].y, w2r[half].v[c].y, wo.y, w2o.y);
        upd(acc.v[c][2], wr[half].v[c].z, w2r[half].v[c].z, wo.z, w2o.z);
        upd(acc.v[c][3], wr[half].v[c].w, w2r[half].v[c].w, wo.w, w2o.w);
        ((float4 *)w2)[lane + c * 64] = w2o;
        ((float4 *)w)[lane + c * 64] = wo;
      }
      if (tl) {
        float wo, w2o;
        upd(acc.t, wr[half].t, w2r[half].t, wo, w2o);
        w2[256 * NCH + lane] = w2o;
        w[256 * NCH + lane] = wo;
      }
    }
  }
}

// k_push_tg with one wave per (key, half): the h half (h, h2sum: the target
// records' g*neu1 sums) and the v half (v, v2sum: the context records' neu1e
// sums) of a key's AdaGrad update touch disjoint elements, so they run as
// independent waves — half the live registers per wave (occupancy) and twice
// the waves.  Same arithmetic per element: bit-identical to k_push_tg.
template <int NCH, int UNR>
__global__ __launch_bounds__(256) void k_push_th(PushArgs<float, float> a) {
  constexpr int PU = 8;
  const int lane = threadIdx.x & 63;
  const int D = a.D;
  const bool tl = 256 * NCH + lane < D;
  const uint64_t n2 = 2ull * a.U;
  for (uint64_t uh = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); uh < n2; uh += (uint64_t)gridDim.x * 4) {
    const uint64_t u = uh >> 1;
    const int half = (int)(uh & 1);
    const int32_t vid = a.K[u];
    if (lane == 0 && half == 0) a.local[vid] = -1;
    const uint32_t s0 = a.seg[(2 * half) * a.U + u], s1 = a.seg[(2 * half + 1) * a.U + u];
    const uint32_t cnt = s1 - s0;
    if (cnt == 0 && !a.cache_h) continue;
    float *row = a.rows + (uint64_t)a.vid_row[vid] * 4 * D;
    const uint32_t i0 = a.ioff[2 * u + half], i1 = a.ioff[2 * u + half + 1];
    const bool one = i1 - i0 == 1;
    FSlice<NCH> wr, w2r, pf;
    ItemRecs ri;
    wr.ld(row + half * D, lane, tl);
    if (cnt) {
      if (one)
        ri = run_recs(a.vals, a.pg, a.SH, a.SV, a.HOFF, s0, cnt, half, lane);
      else
        pf.ld(a.partial + (uint64_t)i0 * D, lane, tl);
      w2r.ld(row + (2 + half) * D, lane, tl);
    }
    if (a.cache_h) wr.st_full((half ? a.cache_v : a.cache_h) + (uint64_t)vid * a.cs, lane, tl, a.full ? a.cs : D);
    if (cnt == 0) continue;
    FAcc<NCH> acc;
    acc.zero();
    if (one) {
      const float *base = half == 0 ? a.neu1 : a.neu1e;
      FAcc<NCH> c;
      c.zero();
      for (uint32_t r0 = 0; r0 < cnt; r0 += UNR) {
        FSlice<NCH> rv[UNR];
        float gf[UNR];
#pragma unroll
        for (int q = 0; q < UNR; q++) {
          const uint32_t idx = min(r0 + q, cnt - 1);
          const uint32_t pr = idx < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)ri.p0, (int)idx)
                                       : (uint32_t)__builtin_amdgcn_readlane((int)ri.p1, (int)(idx - 64));
          gf[q] = __int_as_float(idx < 64 ? __builtin_amdgcn_readlane(__float_as_int(ri.g0), (int)idx)
                                          : __builtin_amdgcn_readlane(__float_as_int(ri.g1), (int)(idx - 64)));
          rv[q].ld(base + (uint64_t)pr * a.ld, lane, tl);
        }
#pragma unroll
        for (int q = 0; q < UNR; q++) {
          if (r0 + q < cnt) {
            if (half == 0)
              c.axpy((double)gf[q], rv[q], tl);
            else
              c.add(rv[q], tl);
          }
        }
      }
#pragma unroll
      for (int cc = 0; cc < NCH; cc++)
#pragma unroll
        for (int k = 0; k < 4; k++) acc.v[cc][k] = (double)(float)c.v[cc][k];  // the fp32 partial
      acc.t = (double)(float)c.t;
    } else {
      acc.add(pf, tl);
      const uint32_t stride = (i1 - i0) > a.group ? kGroup : 1;
      for (uint32_t it0 = i0 + stride; it0 < i1; it0 += PU * stride) {
        FSlice<NCH> pv[PU];
#pragma unroll
        for (int q = 0; q < PU; q++) pv[q].ld(a.partial + (uint64_t)min(it0 + q * stride, i1 - 1) * D, lane, tl);
#pragma unroll
        for (int q = 0; q < PU; q++)
          if (it0 + q * stride < i1) acc.add(pv[q], tl);
      }
    }
    const double inv = (double)cnt;
    float *w = row + half * D, *w2 = row + (2 + half) * D;
    auto upd = [&](double sum, float wv, float w2v, float &wo, float &w2o) {
      const double g = (double)(float)(sum / inv);  // the mean in the push payload's type
      const double acc2 = (double)w2v + g * g;
      const double step = (g * a.lr) / sqrt(acc2 + a.fudge);
      w2o = (float)acc2;
      wo = (float)((double)wv + step);
    };
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      float4 wo, w2o;
      upd(acc.v[c][0], wr.v[c].x, w2r.v[c].x, wo.x, w2o.x);
      upd(acc.v[c][1], wr.v[c].y, w2r.v[c].y, wo.y, w2o.y);
      upd(acc.v[c][2], wr.v[c].z, w2r.v[c].z, wo.z, w2o.z);
      upd(acc.v[c][3], wr.v[c].w, w2r.v[c].w, wo.w, w2o.w);
      ((float4 *)w2)[lane + c * 64] = w2o;
      ((float4 *)w)[lane + c * 64] = wo;
    }
    if (tl) {
      float wo, w2o;
      upd(acc.t, wr.t, w2r.t, wo, w2o);
      w2[256 * NCH + lane] = w2o;
      w[256 * NCH + lane] = wo;
    }
  }
}

// k_push_th software-pipelined across (key, half) items, like k_gather_t:
// a wave walks a stride of items; the next item's bounds / key / shard row are
// loaded at the top and its record info right behind this item's row loads,
// so the per-item chain (bounds -> records -> g -> rows, key -> shard row ->
// w rows) overlaps the previous item's traffic.  Same arithmetic: bit-identical.
struct PHead {
  uint32_t s0, s1, i0, i1;
  int32_t vid;
  uint32_t row;
};
// TO_GRADS (sharded learner): stop at the mean and write the push payload
// [U][h|v] (fp32), zeros for an empty half, as k_push<..., true> does; the
// owner applies AdaGrad (swps_w2v_serve_push).
// MODE 0: every (key, half); 1: all but the multi-chunk halves (they wait for k_gather_t's
// partials while this runs beside it, on another stream); 2: only the multi-chunk halves.
template <int NCH, int UNR, bool TO_GRADS = false, int MODE = 0>
__global__ __launch_bounds__(256) void k_push_thp(PushArgs<float, float> a) {
  constexpr int PU = 8;
  const int lane = threadIdx.x & 63;
  const int D = a.D;
  const bool tl = 256 * NCH + lane < D;
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
  PHead h = head(uh);
  ItemRecs ri{0, 0, 1.f, 1.f};
  if (h.s1 > h.s0 && h.i1 - h.i0 == 1) ri = run_recs(a.vals, a.pg, a.SH, a.SV, a.HOFF, h.s0, h.s1 - h.s0, (int)(uh & 1), lane);
  for (;;) {
    const uint64_t nx = uh + stride;
    const bool more = nx < n2;
    PHead hn{0, 0, 0, 0, 0, 0};
    if (more) hn = head(nx);
    const int half = (int)(uh & 1);
    const bool multi = h.i1 - h.i0 > 1;
    bool other = (MODE == 1 && multi) || (MODE == 2 && !multi);
    // the key's local slot is freed by its half-0 item in pass 1 even when pass 2 pushes that half
    // (pass 2 never frees one): every key of the batch leaves the map, as in MODE 0
    if (MODE == 1 && multi && lane == 0 && half == 0) a.local[h.vid] = -1;
    if (TO_GRADS && a.gpass) {  // the key's owner range: its first ohalf keys go in pass 1
      const uint32_t u = (uint32_t)(uh >> 1);
      uint32_t r = 0;
      while (r + 1 < a.nown && a.obnd[r + 1] <= u) r++;
      const bool first = u - a.obnd[r] < a.ohalf[r];
      other = other || (first != (a.gpass == 1));
    }
    if (other) {  // the other pass's item
      if (more && hn.s1 > hn.s0 && hn.i1 - hn.i0 == 1 && MODE != 2)
        ri = run_recs(a.vals, a.pg, a.SH, a.SV, a.HOFF, hn.s0, hn.s1 - hn.s0, (int)(nx & 1), lane);
      if (!more) break;
      uh = nx;
      h = hn;
      continue;
    }
    if (lane == 0 && half == 0 && MODE != 2) a.local[h.vid] = -1;
    const uint32_t cnt = h.s1 - h.s0;
    const bool one = h.i1 - h.i0 == 1;
    float *row = TO_GRADS ? nullptr : a.rows + (uint64_t)h.row * 4 * D;
    float *gout = TO_GRADS ? a.grads + ((uh >> 1) * 2 + half) * (uint64_t)D : nullptr;
    FSlice<NCH> wr, w2r, pf;
    ItemRecs rn{0, 0, 1.f, 1.f};
    bool rn_done = false;
    auto next_recs = [&]() {
      if (more && hn.s1 > hn.s0 && hn.i1 - hn.i0 == 1)
        rn = run_recs(a.vals, a.pg, a.SH, a.SV, a.HOFF, hn.s0, hn.s1 - hn.s0, (int)(nx & 1), lane);
      rn_done = true;
    };
    if (!TO_GRADS) {
      if (cnt || a.cache_h) wr.ld(row + half * D, lane, tl);
      if (cnt) w2r.ld(row + (2 + half) * D, lane, tl);
    }
    if (cnt && !one) pf.ld(a.partial + (uint64_t)h.i0 * D, lane, tl);
    if (!TO_GRADS && a.cache_h)  // the pre-update value, pad as zeros (whole lines)
      wr.st_full((half ? a.cache_v : a.cache_h) + (uint64_t)h.vid * a.cs, lane, tl, a.full ? a.cs : D);
    if (TO_GRADS && cnt == 0) {  // an empty half: zero mean
      FSlice<NCH> z;
#pragma unroll
      for (int c = 0; c < NCH; c++) z.v[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      z.t = 0.f;
      z.st(gout, lane, tl);
    }
    if (cnt) {
      FAcc<NCH> acc;
      acc.zero();
      if (one) {
        const float *base = half == 0 ? a.neu1 : a.neu1e;
        FAcc<NCH> c;
        c.zero();
        for (uint32_t r0 = 0; r0 < cnt; r0 += UNR) {
          FSlice<NCH> rv[UNR];
          float gf[UNR];
#pragma unroll
          for (int q = 0; q < UNR; q++) {
            const uint32_t idx = min(r0 + q, cnt - 1);
            const uint32_t pr = idx < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)ri.p0, (int)idx)
                                         : (uint32_t)__builtin_amdgcn_readlane((int)ri.p1, (int)(idx - 64));
            gf[q] = __int_as_float(idx < 64 ? __builtin_amdgcn_readlane(__float_as_int(ri.g0), (int)idx)
                                            : __builtin_amdgcn_readlane(__float_as_int(ri.g1), (int)(idx - 64)));
            rv[q].ld(base + (uint64_t)pr * a.ld, lane, tl);
          }
          if (r0 == 0) next_recs();  // behind this item's first rows
#pragma unroll
          for (int q = 0; q < UNR; q++) {
            if (r0 + q < cnt) {
              if (half == 0)
                c.axpy((double)gf[q], rv[q], tl);
              else
                c.add(rv[q], tl);
            }
          }
        }
#pragma unroll
        for (int cc = 0; cc < NCH; cc++)
#pragma unroll
          for (int k = 0; k < 4; k++) acc.v[cc][k] = (double)(float)c.v[cc][k];  // the fp32 partial
        acc.t = (double)(float)c.t;
      } else {
        next_recs();
        acc.add(pf, tl);
        const uint32_t st = (h.i1 - h.i0) > a.group ? kGroup : 1;
        for (uint32_t it0 = h.i0 + st; it0 < h.i1; it0 += PU * st) {
          FSlice<NCH> pv[PU];
#pragma unroll
          for (int q = 0; q < PU; q++) pv[q].ld(a.partial + (uint64_t)min(it0 + q * st, h.i1 - 1) * D, lane, tl);
#pragma unroll
          for (int q = 0; q < PU; q++)
            if (it0 + q * st < h.i1) acc.add(pv[q], tl);
        }
      }
      const double inv = (double)cnt;
      if (TO_GRADS) {  // the mean in the push payload's type
        FSlice<NCH> m;
#pragma unroll
        for (int c = 0; c < NCH; c++)
          m.v[c] = make_float4((float)(acc.v[c][0] / inv), (float)(acc.v[c][1] / inv), (float)(acc.v[c][2] / inv),
                               (float)(acc.v[c][3] / inv));
        m.t = (float)(acc.t / inv);
        m.st(gout, lane, tl);
      } else {
        float *w = row + half * D, *w2 = row + (2 + half) * D;
        auto upd = [&](double sum, float wv, float w2v, float &wo, float &w2o) {
          const double g = (double)(float)(sum / inv);  // the mean in the push payload's type
          const double acc2 = (double)w2v + g * g;
          const double step = (g * a.lr) / sqrt(acc2 + a.fudge);
          w2o = (float)acc2;
          wo = (float)((double)wv + step);
        };
#pragma unroll
        for (int c = 0; c < NCH; c++) {
          float4 wo, w2o;
          upd(acc.v[c][0], wr.v[c].x, w2r.v[c].x, wo.x, w2o.x);
          upd(acc.v[c][1], wr.v[c].y, w2r.v[c].y, wo.y, w2o.y);
          upd(acc.v[c][2], wr.v[c].z, w2r.v[c].z, wo.z, w2o.z);
          upd(acc.v[c][3], wr.v[c].w, w2r.v[c].w, wo.w, w2o.w);
          ((float4 *)w2)[lane + c * 64] = w2o;
          ((float4 *)w)[lane + c * 64] = wo;
        }
        if (tl) {
          float wo, w2o;
          upd(acc.t, wr.t, w2r.t, wo, w2o);
          w2[256 * NCH + lane] = w2o;
          w[256 * NCH + lane] = wo;
        }
      }
    }
    if (!rn_done) next_recs();
    if (!more) break;
    uh = nx;
    h = hn;
    ri = rn;
  }
}

#include "swps_w2v_bfp.h"

// (NCH, NT) lane layout of the BFP-mode kernels for dim D (swps_w2v_bfp.h), as 10*NCH + NT
inline int bfp_shape(int D) {
  const int nch = D / 256, rem = D % 256;
  if (rem == 0) return 10 * nch;
  if (rem <= 128) return 10 * nch + (rem + 63) / 64;
  return 10 * (nch + 1);
}
#define SWPS_BFP_SHAPES(code, F, RB) \
  switch (code) {                     \
    case 1: F(0, 1, RB); break;       \
    case 2: F(0, 2, RB); break;       \
    case 10: F(1, 0, RB); break;      \
    case 11: F(1, 1, RB); break;      \
    case 12: F(1, 2, RB); break;      \
    default: F(2, 0, RB); break;      \
  }
// every (NCH, NT, RB) instantiation of F for context w's dim and residual bytes
#define SWPS_BFP_DISPATCH(w, F)                    \
  do {                                             \
    if ((w)->bfp_rb)                               \
      SWPS_BFP_SHAPES(bfp_shape((w)->D), F, 1)     \
    else                                           \
      SWPS_BFP_SHAPES(bfp_shape((w)->D), F, 0)     \
  } while (0)

// requester side of a sharded pull: the owners' pull values [U][h|v] (K order)
// into the worker cache (global_pull_access.h:88-97: params[key] = val)
// srow != nullptr (world 1, the pull read in place): value u is the table row srow[u] of vals
// (the shard rows, [h | v | h2 | v2]: its first 2D elements)
template <typename T>
__global__ __launch_bounds__(256) void k_install(const int32_t *__restrict__ K, uint32_t U, const T *__restrict__ vals,
                                                 int D, T *__restrict__ cache_h, T *__restrict__ cache_v,
                                                 int32_t *__restrict__ local, int set_local, int cs,
                                                 const uint32_t *__restrict__ srow = nullptr) {
  using V = typename V16<T>::V;
  constexpr int E = V16<T>::E;
  const int lane = threadIdx.x & 63;
  const int NC = D / E;
  for (uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); u < U; u += (uint64_t)gridDim.x * 4) {
    const int32_t vid = K[u];
    // a key the shard holds no row for (full table: table_copy_pull's zero row) installs zeros
    const uint32_t sr = srow ? srow[u] : 0u;
    const bool have = !srow || sr != kNoRow;
    const V *src = (const V *)(vals + (srow ? (uint64_t)(have ? sr : 0u) * 4 : u * 2) * D);
    V *dh = (V *)(cache_h + (uint64_t)vid * cs);  // cs: the cache row stride (swps_w2v::cs)
    V *dv = (V *)(cache_v + (uint64_t)vid * cs);
    for (int c = lane; c < cs / E; c += 64) {  // the pad too (zeros): whole-line stores
      const bool in = have && c < NC;
      dh[c] = in ? src[c] : V{};
      dv[c] = in ? src[NC + c] : V{};
    }
    if (set_local && lane == 0) local[vid] = (int32_t)u;
  }
}

// k_install of a split pull's part (ShardDriver early / late values): value i belongs to the
// batch's key pos[i] (K order) — the same rows written as by k_install of the assembled values
template <typename T>
__global__ __launch_bounds__(256) void k_install_idx(const int32_t *__restrict__ K, const uint32_t *__restrict__ pos,
                                                     uint32_t n, const T *__restrict__ vals, int D,
                                                     T *__restrict__ cache_h, T *__restrict__ cache_v, int cs) {
  using V = typename V16<T>::V;
  constexpr int E = V16<T>::E;
  const int lane = threadIdx.x & 63;
  const int NC = D / E;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (uint64_t)gridDim.x * 4) {
    const int32_t vid = K[pos[i]];
    const V *src = (const V *)(vals + i * 2 * D);
    V *dh = (V *)(cache_h + (uint64_t)vid * cs);
    V *dv = (V *)(cache_v + (uint64_t)vid * cs);
    for (int c = lane; c < cs / E; c += 64) {
      const bool in = c < NC;
      dh[c] = in ? src[c] : V{};
      dv[c] = in ? src[NC + c] : V{};
    }
  }
}

__global__ void k_vid_keys(const int32_t *__restrict__ K, uint64_t n, const uint64_t *__restrict__ vkeys,
                           uint64_t *__restrict__ out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = vkeys[K[i]];
}

// owner side of the early / late pull split (AppOps::late_mask): stamp the table rows served
// at one slot, then flag the rows of another slot that carry the stamp
__global__ void k_stamp_rows(const uint32_t *__restrict__ rows, uint64_t n, uint32_t cap, uint32_t stamp,
                             uint32_t *__restrict__ mark) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && rows[i] < cap) mark[rows[i]] = stamp;
}
__global__ void k_flag_rows(const uint32_t *__restrict__ rows, uint64_t n, uint32_t cap, uint32_t stamp,
                            const uint32_t *__restrict__ mark, uint8_t *__restrict__ flags) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = rows[i] >= cap || mark[rows[i]] == stamp;  // an unknown row: late (safe)
}

__global__ void k_trace_copy(const int32_t *__restrict__ src, uint64_t n, int32_t *__restrict__ dst) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

inline unsigned nblk(uint64_t threads, unsigned bs = 256) { return (unsigned)std::max<uint64_t>(1, (threads + bs - 1) / bs); }

// ---- per-kernel HIP-event timing ----------------------------------------
enum { KT_KEEP = 0, KT_FWD, KT_SORT, KT_GATHER, KT_PUSH, KT_PULL, KT_REC, KT_N };

// neu1/neu1e row stride: D elements rounded up to whole 128-B cache lines, so
// the forward writes and the gather reads full lines only (1200-B fp32 rows at
// D = 300 straddled 10-11 lines: PMC showed 28 % extra forward write bytes).
inline int row_ld(int D, size_t es, bool pad = true) {
  const int q = pad ? (int)(128 / es) : 1;
  return (D + q - 1) / q * q;
}

// fp64 intermediates (parity mode): neu1/neu1e, partials and the push payload in fp64
inline bool inter64(const swps_w2v_cfg &c) { return c.fp64_intermediates == SWPS_INTER_FP64; }

struct Timer {
  bool on = false;
  std::vector<hipEvent_t> pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  double ms[KT_N] = {0};
  uint64_t cnt[KT_N] = {0};
  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
  hipEvent_t begin(hipStream_t s) {
    if (!on) return nullptr;
    hipEvent_t e = get();
    (void)hipEventRecord(e, s);
    return e;
  }
  void end(int k, hipEvent_t b, hipStream_t s) {
    if (!on || !b) return;
    hipEvent_t e = get();
    (void)hipEventRecord(e, s);
    pending.push_back({k, {b, e}});
  }
  // a pair for hipExtLaunchKernelGGL: stamped by the GPU at the kernels' own start / end (no stream
  // gaps in the time, as rocprof measures it); ext_end registers it in place of begin / end
  hipEvent_t ext() { return on ? get() : nullptr; }
  void ext_end(int k, hipEvent_t b, hipEvent_t e) {
    if (b && e) pending.push_back({k, {b, e}});
  }
  void drop(hipEvent_t e) {  // an event begin() recorded that ext stamps replace
    if (e) pool.push_back(e);
  }
  void resolve() {  // caller has synchronized the stream
    for (auto &q : pending) {
      float t = 0;
      (void)hipEventElapsedTime(&t, q.second.first, q.second.second);
      ms[q.first] += t;
      cnt[q.first]++;
      pool.push_back(q.second.first);
      pool.push_back(q.second.second);
    }
    pending.clear();
  }
  ~Timer() {
    for (auto &q : pending) {
      (void)hipEventDestroy(q.second.first);
      (void)hipEventDestroy(q.second.second);
    }
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

}  // namespace

struct swps_w2v {
  swps_table *t = nullptr;
  swps_w2v_cfg cfg{};
  int D = 0, W = 0, N = 0, NCH = 1;
  bool f64 = false;
  bool tail = false;  // fast mode: FSlice kernels (D = 256*NCH + tail, 0 < tail <= 64)
  bool bfp = false;  // fp32 table, fp64_intermediates = SWPS_INTER_BFP40 / _BFP32: the BFP-row kernels (swps_w2v_bfp.h)
  int bfp_rb = 0;    // ... with an int8 residual per element (BFP40: 1) or not (BFP32: 0)
  int xcd_order = 1;  // forward blocks in XCD-contiguous order (SWPS_XCD_ORDER=0 turns it off for A/B timing)
  int push_t = 1;     // fast mode: k_push_t (SWPS_PUSH_T=0: k_push, for A/B timing)
  int gather_unr = 8;         // k_gather_t rows in flight per wave (SWPS_GATHER_UNR: 4, 8, 16; A/B timing)
  int push_wpe = 0;  // SWPS_PUSH_WPE: 0 = by batch size, 4 / 1 = k_push_b<1,1,0> at 4 waves per SIMD or not
  int push_unr = 4;  // k_push_b<1,1,0>'s record rows in flight: 4 (SWPS_PUSH_UNR8=1: 8, the previous default)
  uint32_t gather_grid = 65536;  // k_gather_t / k_combine grid cap in blocks (SWPS_GATHER_GRID; A/B: 2048..65536 -> 65536 best)
  bool cache_pad = true;  // worker-cache rows padded to 128 B (SWPS_CACHE_PAD=0: D-strided, for A/B timing)
  int cs = 0;              // worker-cache row stride in elements (set with the cache allocation)
  bool uni_index = true;  // negatives via the coarse-indexed run-length table (SWPS_UNI_INDEX=0: the 1e8-slot table)
  bool seg4 = true;       // k_seg_bounds4: 4 sorted records per thread (SWPS_SEG4=0: one, A/B)
  bool tok_local = true;  // k_tok_local + k_records_t's per-token lookups (SWPS_TOK_LOCAL=0: off, A/B)
  // k_item_desc's runs by k_item_heads + max-scan instead of a binary search (SWPS_ITEM_HEADS=1; off:
  // same-box A/B, round 4, 2 reps: B = 5000 unchanged, B = 100 3.01e8 -> 2.92e8 words/s — four more
  // launches on the prep stream)
  bool item_heads = false;
  DevMem d_irun;           // its item -> run map
  DevMem d_tloc;          // its per-token {local, source} of the batch being prepped
  bool row_pad = true;  // neu1/neu1e rows padded to 128 B (SWPS_ROW_PAD=0: D-strided, for A/B timing)
  hipStream_t s = nullptr;
  // host corpus / vocab
  std::vector<int32_t> tok;       // host ingest only (the GPU ingest leaves tokens in d_tok)
  std::vector<int32_t> tok_line;
  uint64_t ntok = 0;              // corpus tokens
  uint64_t tok_fp = 0;            // device-computed fingerprint of d_tok (checkpoint corpus check)
  bool tok_on_device = false;     // d_tok / d_tok_line / d_K were built by the GPU ingest
  std::vector<int64_t> line_off;
  std::vector<uint8_t> line_valid;
  std::vector<uint64_t> vocab_keys;
  std::vector<int32_t> counts;
  uint64_t train_words = 0;
  bool loaded = false, inited = false;
  // schedule (identical every epoch)
  struct Batch {
    uint64_t l0, l1, kofs;
    uint32_t U;
    uint64_t sofs = 0;    // minibatch-vocab mode: offset of the batch's table run starts
    uint64_t gathered = 0;  // words its gather_keys counted into _num_words
  };
  std::vector<Batch> batches;
  std::vector<int32_t> allK;
  uint64_t max_tok = 0, max_U = 0, max_lines = 0;
  uint64_t cursor = 0;  // next global batch index
  // device
  DevMem d_uidx;
  DevMem d_tok, d_tok_line, d_line_off, d_ran, d_exptab, d_unigram, d_starts, d_vid_row, d_cache_h, d_cache_v,
      d_local, d_K;
  DevMem d_btok, d_bounds;
  DevMem d_kflag, d_kscan, d_ldraw, d_ldoff, d_pos_tok, d_rec, d_neu1, d_neu1e, d_pkeys, d_pvals, d_pkeys_s,
      d_pvals_s, d_pg, d_seg, d_icnt, d_ioff, d_partial, d_desc, d_tmp, d_trace, d_rows_touched, d_gstats;
  swps::ShardDriver *drv = nullptr;  // swps_w2v_shard_comm: the library drives the exchange
  bool rec_generic = false;          // SWPS_REC_GENERIC=1: the generic k_records (A/B, tests)
  DevMem d_lead;  // hot-group leaders of the batch's gather items: [0] = count, then item indices
  DevMem d_multi;  // items of multi-chunk runs (k_gather_t's work when the push is fused): [0] = count, then items
  DevMem d_krow;   // per batch key: its shard row (vid_row[K[u]]), for k_push_thp
  int fused_push = 1;  // fast mode: the push sums single-chunk runs itself (SWPS_FUSED_PUSH=0: k_gather_t + k_push_t)
  int push_tg_var = 5;  // fused push kernel (SWPS_PUSH_TG, A/B): 5 = k_push_thp (default), 0 = k_push_tg UNR 8,
                        // 1 = k_push_tg at occupancy 4, 2 = k_push_tg UNR 4, 3 = k_push_th, 4 = k_push_th UNR 16
  uint32_t push_grid = 0;  // k_push_thp grid cap in blocks (SWPS_PUSH_GRID; 0 = by batch size)
  int fwd_g = 4;           // k_forward_t rows in flight per wave (SWPS_FWD_G: 4, 8, 16; A/B)
  // k_combine pre-sums hot runs' partials in groups of kGroup: 1 always, 0 never (the push reads every
  // partial), 2 (default) when the batch has at least combine_min records -- measured: -2.6% without it at
  // B = 5000 (21M records), +1.6% at B = 100 (0.4M), where its launch costs more than the re-reads
  int combine = 2;
  uint64_t combine_min = 1ull << 22;
  int full_lines = 1;  // neu1/neu1e and cache-row stores write the row pad as zeros (SWPS_FULL_LINES=0: off; A/B)
  int split_grads = 1;  // sharded learner (world > 1): mean gradients in two owner-half passes (SWPS_SPLIT_GRADS=0: one)
  hipEvent_t ev_half = nullptr;  // recorded between the two passes of the last step
  bool half_ready = false;       // the last step ran the two passes (the driver takes and clears it)
  int split_push = 0;  // SWPS_SPLIT_PUSH: 1 = gather beside the push always, -1 = below 64 k keys, 0 = never
                      // (default: same-box A/B at B = 100 lines 0.321 ms/step in one stream vs 0.349 split)
  hipStream_t s_side = nullptr;
  hipEvent_t ev_fwd = nullptr, ev_gat = nullptr;
  uint32_t multi_chunk = 0;  // SWPS_MULTI_CHUNK: chunk size of multi-chunk runs (1..128; 0 = kChunk)
  int multi_sort = 1;                 // order the multi-chunk items by position (SWPS_MULTI_SORT=0: off; A/B)
  uint64_t multi_sort_min = 65536;    // ... for batches of at least this many kept positions (SWPS_MULTI_SORT_MIN)
  uint64_t *h_small = nullptr;  // pinned readback
  // RNG (utils/random.h:44-47, seed 2008)
  uint64_t lstate = 2008ULL;
  uint64_t fstate = std::numeric_limits<unsigned long>::max() / 2;
  uint64_t lstate_epoch = 0;        // main LCG state at the current epoch's start
  uint64_t fstate_epoch = 0;        // float LCG state at the current epoch's start
  // sharded mode: keys owned by BasicHashFrag node rank+1
  int rank = 0, world = 1, frag_num = 0;
  bool sharded = false;
  std::vector<uint64_t> bcounts;   // [nb][world] keys requested per owner per batch
  std::vector<uint64_t> icounts;   // [world] init request per owner
  std::vector<int32_t> init_order; // vids grouped by owner
  DevMem d_vkeys, d_init_order, d_serve_rows, d_push_rows;
  DevMem d_mark;          // late_mask: a stamp per table row
  // the next step's pull values in two parts (AppOps::install_parts; consumed by that step)
  const uint32_t *pull_rows = nullptr;  // world 1: the slot's shard rows, read in place by the step's install
  struct Parts {
    const void *vals[2] = {nullptr, nullptr};
    const uint32_t *pos[2] = {nullptr, nullptr};
    uint64_t n[2] = {0, 0};
  } parts;
  uint32_t mark_stamp = 0;
  hipStream_t ss = nullptr;  // serve stream (request / serve_pull / serve_push); nullptr = s
  // the library driver's step slot (AppOps::set_slot): the keys served at a slot are the same every
  // epoch, so their row lookups and the push's grouping sort are kept per slot
  int64_t slot = -1;
  struct SlotRows {
    DevMem rows, sorted;
    uint64_t n = 0;
    bool sorted_valid = false;
  };
  std::vector<std::unique_ptr<SlotRows>> slot_rows;
  std::vector<uint32_t> plan_P;     // kept positions per batch of the current epoch
  // minibatch-vocab mode (word2vec.h MiniBatch, w2v_local.cpp)
  std::vector<int32_t> allUK;       // per batch: its vids in std::map key order (offset kofs)
  std::vector<uint64_t> bstarts;    // per batch: U+1 table run starts (offset sofs)
  std::vector<int32_t> bcnt_tok;    // per trained token: its word's count in its batch
  uint64_t gather_end = 0;          // words counted by the epoch's final (< 5 keys) gather
  DevMem d_bstarts, d_UK, d_bcnt_tok, d_tw;
  // SWPS_SAMPLER_ALIAS: alias tables (global: one over the vocab in vid order;
  // minibatch-vocab: one per batch over its map order, offset = batch kofs)
  std::vector<uint2> alias;
  DevMem d_alias;
  // the prepared (parameter-independent) half of the next minibatch
  struct Prepped {
    bool valid = false, records = false, sorted = false, msorted = false;
    uint64_t bi = 0, P = 0, nt = 0, HOFF = 0, M = 0, max_items = 0;
    uint32_t U = 0;
  } pb;
  // overlapped single-GPU driver (train_overlapped): the second set of the
  // parameter-independent per-batch buffers, swapped with the members above,
  // and the stream prep(i+1) runs on while learn(i) runs on s
  static constexpr int kPrepBufs = 15;
  DevMem alt[kPrepBufs];
  bool alt_local_ready = false;
  // train_overlapped: -1 = auto (on for minibatches of at most kOverlapTok tokens: at B = 100 lines the
  // prep chain — records, sort, index: ~12 short latency-bound launches — hides behind the learn, 0.41 ->
  // 0.36 ms/step; at B = 5000 forward and gather already fill every CU and the HBM: 4.25e8 sequential vs
  // 4.24e8 / 4.02e8 overlapped); SWPS_OVERLAP=0/1 forces it
  int overlap = -1;
  hipStream_t s_prep = nullptr;
  hipEvent_t ev_learn = nullptr, ev_prep = nullptr;
  hipEvent_t fwd_event = nullptr;  // learn_batch records it after the forward when set (overlap mode 2)
  DevMem *prep_set[kPrepBufs] = {&d_pos_tok, &d_rec,  &d_pkeys, &d_pvals, &d_pkeys_s, &d_pvals_s, &d_tmp,
                                 &d_seg,     &d_icnt, &d_ioff,  &d_desc,  &d_lead,    &d_multi, &d_krow, &d_local};
  // stats
  uint64_t st_batches = 0, st_kept = 0, st_words = 0, st_pairs = 0, st_pulled = 0, st_pushed = 0;
  uint64_t st_sums = 0, st_fused = 0, st_fused_g = 0, st_split = 0;  // batches with gradient sums; of those, fused in-place
                                                       // pushes / fused mean-gradient (sharded) pushes
  // negative trace
  uint64_t trace_cap = 0;
  std::vector<int64_t> trace;
  Timer timer;
};

namespace {

int check_cfg(swps_w2v *w) {
  const auto &c = w->cfg;
  if (c.window <= 0 || 2 * c.window > 64) return fail(SWPS_E_CFG, "window must be in [1, 32]");
  if (c.negative < 0 || c.negative + 1 > 64) return fail(SWPS_E_CFG, "negative must be in [0, 63]");
  if (c.minibatch <= 0) return fail(SWPS_E_CFG, "minibatch must be positive");
  if (c.unigram_size == 0 || c.unigram_size > (1ULL << 31)) return fail(SWPS_E_CFG, "unigram_size out of range");
  if (c.sampler != SWPS_SAMPLER_TABLE && c.sampler != SWPS_SAMPLER_ALIAS) return fail(SWPS_E_CFG, "unknown sampler");
  const int E = w->f64 ? 2 : 4;
  if (w->D % E != 0) return fail(SWPS_E_UNSUPPORTED, "dim must be a multiple of 16 bytes (4 fp32 / 2 fp64)");
  int nc = w->D / E;
  w->NCH = (nc + 63) / 64;
  if (!w->f64 && w->D > 256 && w->D % 256 != 0 && w->D % 256 <= 64) w->tail = true;
  if (const char *e = getenv("SWPS_SLICE")) w->tail = w->tail && atoi(e) != 0;  // A/B timing
  if (w->NCH > 4) return fail(SWPS_E_UNSUPPORTED, "dim too large (max 1024 fp32 / 512 fp64)");
  if (c.fp64_intermediates < SWPS_INTER_FP32 || c.fp64_intermediates > SWPS_INTER_BFP32)
    return fail(SWPS_E_CFG, "fp64_intermediates must be SWPS_INTER_FP32, _FP64, _BFP40 or _BFP32");
  if (!w->f64 && (c.fp64_intermediates == SWPS_INTER_BFP40 || c.fp64_intermediates == SWPS_INTER_BFP32)) {
    if (w->D > kBfpMaxD) return fail(SWPS_E_UNSUPPORTED, "BFP intermediates: dim at most 512");
    w->bfp = true;
    w->bfp_rb = c.fp64_intermediates == SWPS_INTER_BFP40 ? 1 : 0;
  }
  return SWPS_OK;
}

// Vocab (word2vec_global.h:385-444, nthreads = 1): word counts over valid
// lines, `_local_keys` filled in first-occurrence order; vid = position in the
// std::unordered_set iteration order (= `_wordids`, the unigram-table order).
int ingest(swps_w2v *w, const std::vector<uint64_t> &tok_keys, std::vector<int64_t> &&line_off) {
  const uint64_t nl = line_off.size() - 1;
  w->line_off = std::move(line_off);
  w->line_valid.assign(nl, 0);
  std::unordered_map<uint64_t, int32_t> cnt;
  std::unordered_set<uint64_t> local_keys;
  uint64_t tw = 0;
  for (uint64_t l = 0; l < nl; l++) {
    const int64_t a = w->line_off[l], b = w->line_off[l + 1];
    const bool valid = (b - a) >= w->cfg.min_sentence_length;
    w->line_valid[l] = valid;
    if (w->cfg.minibatch_vocab && !valid && b > a)
      return fail(SWPS_E_UNSUPPORTED, "minibatch-vocab mode: a non-empty line shorter than min_sentence_length is "
                                      "trained but never gathered (word2vec.h:521-523, UB in the reference)");
    if (!valid) continue;
    tw += (uint64_t)(b - a);
    for (int64_t i = a; i < b; i++) {
      auto it = cnt.find(tok_keys[i]);
      if (it != cnt.end())
        it->second++;
      else {
        cnt.emplace(tok_keys[i], 1);
        local_keys.insert(tok_keys[i]);
      }
    }
  }
  if (local_keys.size() < 5) return fail(SWPS_E_UNSUPPORTED, "fewer than 5 keys (word2vec_global.h:556 returns)");
  w->train_words = tw;
  w->vocab_keys.assign(local_keys.begin(), local_keys.end());
  std::unordered_map<uint64_t, int32_t> vid;
  vid.reserve(w->vocab_keys.size() * 2);
  w->counts.resize(w->vocab_keys.size());
  for (size_t i = 0; i < w->vocab_keys.size(); i++) {
    if (w->vocab_keys[i] == 0)
      return fail(SWPS_E_UNSUPPORTED, "a vocab key hashes to 0 (the reference redraws such negatives)");
    vid[w->vocab_keys[i]] = (int32_t)i;
    w->counts[i] = cnt[w->vocab_keys[i]];
  }
  const uint64_t nt = tok_keys.size();
  w->tok.resize(nt);
  w->tok_line.resize(nt);
  for (uint64_t l = 0; l < nl; l++)
    for (int64_t i = w->line_off[l]; i < w->line_off[l + 1]; i++) {
      auto it = vid.find(tok_keys[i]);
      if (it == vid.end())
        return fail(SWPS_E_UNSUPPORTED, "a word occurs only in lines shorter than min_sentence_length "
                                        "(to_sample reads past word_freq in the reference)");
      w->tok[i] = it->second;
      w->tok_line[i] = (int32_t)l;
    }
  w->ntok = nt;
  w->tok_on_device = false;
  w->loaded = true;
  return SWPS_OK;
}

// gen_unigram_table (word2vec_global.h:467-497) in run-length form: the
// 1e8-entry walk assigns word i the slots [start_i, start_{i+1}); the switch
// to word i+1 happens at the first slot a >= start_i with a/T > d1_i.
void unigram_starts(const uint64_t *keys, const int32_t *counts, size_t V, uint64_t T, std::vector<uint64_t> &starts) {
  std::vector<std::pair<uint64_t, int32_t>> by_key(V);
  for (size_t i = 0; i < V; i++) by_key[i] = {keys[i], counts[i]};
  std::sort(by_key.begin(), by_key.end());
  double pw = 0;
  for (auto &kc : by_key) pw += std::pow(kc.second, 0.75);  // std::map order
  starts.assign(V + 1, T);
  starts[0] = 0;
  double d1 = std::pow(counts[0], 0.75) / (double)pw;
  for (size_t i = 0; i + 1 < V; i++) {
    const uint64_t lo = starts[i];
    auto pred = [&](uint64_t a) { return (int64_t)a / (double)T > d1; };
    uint64_t a = (uint64_t)std::max<double>((double)lo, std::floor(d1 * (double)T));
    if (a > T) a = T;
    while (a > lo && pred(a - 1)) a--;
    while (a < T && !pred(a)) a++;
    if (a >= T) break;  // word i runs to the end; later words get no slots
    starts[i + 1] = a + 1;
    d1 += std::pow(counts[i + 1], 0.75) / (double)pw;
  }
}

// The per-epoch batch schedule of TrainModelThread(0) (word2vec_global.h:
// 591-651): line 1 trains before the first gather (its gradients are dropped
// by the pull), then a push/gather/pull every `minibatch` lines; the gather
// window is the next minibatch+3 valid lines (3 tasks, `line_count >
// minibatch`); the epoch stops after the line where cur_train_words exceeds
// train_words.
void build_schedule(swps_w2v *w) {
  const uint64_t nl = w->line_off.size() - 1;
  const int B = w->cfg.minibatch;
  w->batches.clear();
  w->allK.clear();
  auto window = [&](uint64_t li) {
    std::vector<int32_t> K;
    int count = 0;
    for (int task = 0; task < 3; task++)
      while (li < nl) {
        const uint64_t l = li++;
        if (!w->line_valid[l]) continue;
        for (int64_t i = w->line_off[l]; i < w->line_off[l + 1]; i++) K.push_back(w->tok[i]);
        if (++count > B) break;
      }
    std::sort(K.begin(), K.end());
    K.erase(std::unique(K.begin(), K.end()), K.end());
    return K;
  };
  auto emit = [&](uint64_t l0, uint64_t l1, const std::vector<int32_t> *K) {
    swps_w2v::Batch b{l0, l1, w->allK.size(), 0};
    if (K) {
      b.U = (uint32_t)K->size();
      w->allK.insert(w->allK.end(), K->begin(), K->end());
    }
    w->batches.push_back(b);
  };
  std::vector<int32_t> K;
  bool haveK = false;
  uint64_t start = 0, cur = 0, line_counter = 0, last = 0;
  for (uint64_t li = 0; li < nl; li++) {
    cur += (uint64_t)(w->line_off[li + 1] - w->line_off[li]);
    line_counter++;
    last = li + 1;
    if (line_counter == 1) {
      emit(start, li + 1, haveK ? &K : nullptr);
      K = window(li + 1);
      haveK = true;
      start = li + 1;
    }
    if (line_counter % (uint64_t)B == 0) {
      emit(start, li + 1, haveK ? &K : nullptr);
      K = window(li + 1);
      start = li + 1;
    }
    if (cur > w->train_words) break;
  }
  emit(start, last, haveK ? &K : nullptr);
  w->max_tok = w->max_U = w->max_lines = 0;
  for (auto &b : w->batches) {
    w->max_tok = std::max<uint64_t>(w->max_tok, (uint64_t)(w->line_off[b.l1] - w->line_off[b.l0]));
    w->max_U = std::max<uint64_t>(w->max_U, b.U);
    w->max_lines = std::max<uint64_t>(w->max_lines, b.l1 - b.l0);
  }
}

// Vose's alias method over weights count^0.75 (the distribution the
// reference's unigram table discretises into table_size slots): entry i =
// {P(keep i) as float bits, alias}; deterministic (stable worklists).
void build_alias(const int32_t *counts, size_t n, std::vector<uint2> &out) {
  std::vector<double> q(n);
  double sum = 0;
  for (size_t i = 0; i < n; i++) sum += (q[i] = std::pow((double)counts[i], 0.75));
  std::vector<uint32_t> small, large;
  for (size_t i = 0; i < n; i++) {
    q[i] = q[i] * (double)n / sum;
    (q[i] < 1.0 ? small : large).push_back((uint32_t)i);
  }
  const size_t o = out.size();
  out.resize(o + n);
  size_t si = 0, li = 0;
  while (si < small.size() && li < large.size()) {
    const uint32_t sm = small[si++], lg = large[li];
    float pr = (float)q[sm];
    out[o + sm] = make_uint2(__float_as_uint_host(pr), lg);
    q[lg] -= 1.0 - q[sm];
    if (q[lg] < 1.0) {
      li++;
      small.push_back(lg);
    }
  }
  for (; li < large.size(); li++) out[o + large[li]] = make_uint2(__float_as_uint_host(1.0f), large[li]);
  for (; si < small.size(); si++) out[o + small[si]] = make_uint2(__float_as_uint_host(1.0f), small[si]);
}

// word2vec.h:496-538 train_iter with nthreads = 1: gather_keys reads the next
// B+1 valid lines (word2vec.h:323-377; counts into a std::map, every word
// into _num_words), fewer than 5 keys ends the epoch, then B+1 lines (valid or
// not) are trained from the same position.  The batch's key set is its
// std::map key order; its unigram table (run starts) follows that order.
int build_schedule_mb(swps_w2v *w) {
  const uint64_t nl = w->line_off.size() - 1;
  const int B = w->cfg.minibatch;
  w->batches.clear();
  w->allK.clear();
  w->allUK.clear();
  w->bstarts.clear();
  w->alias.clear();
  w->bcnt_tok.assign(w->tok.size(), 0);
  std::map<int32_t, int32_t> freq_vid;  // counts per vid, then re-ordered by key
  uint64_t p = 0;
  std::vector<std::pair<uint64_t, int32_t>> kv;  // (key, vid)
  std::unordered_map<int32_t, int32_t> cnt_of;
  while (true) {
    cnt_of.clear();
    uint64_t G = 0;
    int count = 0;
    for (uint64_t q = p; q < nl;) {
      const uint64_t l = q++;
      if (!w->line_valid[l]) continue;
      for (int64_t i = w->line_off[l]; i < w->line_off[l + 1]; i++) {
        cnt_of[w->tok[i]]++;
        G++;
      }
      if (++count > B) break;
    }
    if (cnt_of.size() < 5) {
      w->gather_end = G;
      break;
    }
    swps_w2v::Batch b{p, std::min<uint64_t>(nl, p + (uint64_t)B + 1), w->allK.size(), (uint32_t)cnt_of.size(),
                      w->bstarts.size(), G};
    kv.clear();
    for (auto &c : cnt_of) kv.push_back({w->vocab_keys[c.first], c.first});
    std::sort(kv.begin(), kv.end());
    std::vector<uint64_t> keys(kv.size());
    std::vector<int32_t> cnts(kv.size());
    for (size_t i = 0; i < kv.size(); i++) {
      keys[i] = kv[i].first;
      cnts[i] = cnt_of[kv[i].second];
      w->allUK.push_back(kv[i].second);
      w->allK.push_back(kv[i].second);
    }
    std::vector<uint64_t> st;
    unigram_starts(keys.data(), cnts.data(), keys.size(), w->cfg.unigram_size, st);
    w->bstarts.insert(w->bstarts.end(), st.begin(), st.end());
    if (w->cfg.sampler == SWPS_SAMPLER_ALIAS) build_alias(cnts.data(), cnts.size(), w->alias);
    for (uint64_t l = b.l0; l < b.l1; l++)
      for (int64_t i = w->line_off[l]; i < w->line_off[l + 1]; i++) {
        auto it = cnt_of.find(w->tok[i]);
        if (it == cnt_of.end())
          return fail(SWPS_E_UNSUPPORTED, "a trained word is outside its minibatch's gathered vocab "
                                          "(to_sample reads past word_freq in the reference)");
        w->bcnt_tok[i] = it->second;
      }
    w->batches.push_back(b);
    p = b.l1;
  }
  if (w->batches.empty()) return fail(SWPS_E_UNSUPPORTED, "no minibatch with 5 keys (word2vec.h:532 breaks)");
  w->max_tok = w->max_U = w->max_lines = 0;
  for (auto &b : w->batches) {
    w->max_tok = std::max<uint64_t>(w->max_tok, (uint64_t)(w->line_off[b.l1] - w->line_off[b.l0]));
    w->max_U = std::max<uint64_t>(w->max_U, b.U);
    w->max_lines = std::max<uint64_t>(w->max_lines, b.l1 - b.l0);
  }
  return SWPS_OK;
}

// ============================================================================
// Corpus ingest on the GPU (word2vec_global.h:215-227
// parse_instance, :385-444 gather_keys with nthreads = 1, :335-381 the
// minibatch windows).  Same results as the host restatement above (ingest +
// build_schedule), bit for bit; the host keeps only per-line and per-word
// work (line validity, the std::unordered_set iteration order of the V
// distinct keys, the batch boundaries):
//   tokenize   text bytes -> token starts (scan), BKDR / atoi per token
//   vocab      stable radix sort of (key, position); per run: count over valid
//              lines and first valid position (integer atomics: exact);
//              host inserts the V keys into std::unordered_set in first-
//              occurrence order (its iteration order = the vid order) and
//              sends back vid per run; tok[position] = vid
//   schedule   (batch << 32 | vid) for every token of every batch's B+3-line
//              window, radix sort, unique -> each batch's sorted key set
// ============================================================================
__global__ void k_tok_fp(const int32_t *__restrict__ tok, uint64_t n, unsigned long long *__restrict__ out) {
  unsigned long long acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc += splitmix64((uint64_t)(uint32_t)tok[i] ^ (i * 0x9E3779B97F4A7C15ULL));
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, acc);  // a wrapping integer sum: order-independent
}

int tok_fingerprint(swps_w2v *w) {
  DevMem d;
  SWPS_TRY(d.ensure(8));
  SWPS_HIP(hipMemsetAsync(d.p, 0, 8, w->s));
  if (w->ntok) k_tok_fp<<<1024, 256, 0, w->s>>>(w->d_tok.as<int32_t>(), w->ntok, d.as<unsigned long long>());
  SWPS_HIP(hipGetLastError());
  uint64_t h = 0;
  SWPS_HIP(hipMemcpyAsync(&h, d.p, 8, hipMemcpyDeviceToHost, w->s));
  SWPS_HIP(hipStreamSynchronize(w->s));
  w->tok_fp = h ^ w->ntok;
  return SWPS_OK;
}

// per byte: token start (not a delimiter, after a delimiter or at 0) and
// newline flags; element nb is 0 so the exclusive scans end with the totals
__global__ void k_text_flags(const char *__restrict__ t, uint64_t nb, uint32_t *__restrict__ st,
                             uint32_t *__restrict__ nl) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > nb) return;
  if (i == nb) {
    st[i] = 0;
    nl[i] = 0;
    return;
  }
  const char c = t[i], p = i ? t[i - 1] : '\n';
  st[i] = (c != ' ' && c != '\n' && (p == ' ' || p == '\n')) ? 1u : 0u;
  nl[i] = c == '\n' ? 1u : 0u;
}

// token start positions, and line_off[l + 1] = first token after newline l
__global__ void k_text_index(const char *__restrict__ t, uint64_t nb, const uint32_t *__restrict__ st,
                             const uint32_t *__restrict__ tix, const uint32_t *__restrict__ lix,
                             uint64_t *__restrict__ tstart, int64_t *__restrict__ line_off) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  if (st[i]) tstart[tix[i]] = i;
  if (t[i] == '\n') line_off[lix[i] + 1] = (int64_t)tix[i + 1];
}

// BKDRHash (string.h:130-137: signed char) or atoi (word2vec.h:206) of one token
__global__ void k_text_keys(const char *__restrict__ t, uint64_t nb, const uint64_t *__restrict__ tstart, uint64_t n,
                            int atoi_mode, uint64_t *__restrict__ keys) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint64_t i = tstart[k];
  if (!atoi_mode) {
    uint64_t h = 0;
    for (; i < nb && t[i] != ' ' && t[i] != '\n'; i++) h = h * 13131ULL + (uint64_t)(int64_t)(signed char)t[i];
    keys[k] = h;
    return;
  }
  // glibc atoi = (int)strtol(s, 0, 10): leading isspace, sign, digits; strtol saturates
  uint64_t e = i;
  while (e < nb && t[e] != ' ' && t[e] != '\n') e++;
  while (i < e && (t[i] == '\t' || t[i] == '\v' || t[i] == '\f' || t[i] == '\r')) i++;
  bool neg = false;
  if (i < e && (t[i] == '+' || t[i] == '-')) neg = t[i++] == '-';
  const uint64_t lim = neg ? 9223372036854775808ULL : 9223372036854775807ULL;
  uint64_t v = 0;
  bool ovf = false;
  for (; i < e && t[i] >= '0' && t[i] <= '9'; i++) {
    const uint64_t d = (uint64_t)(t[i] - '0');
    if (ovf || v > (lim - d) / 10)
      ovf = true;
    else
      v = v * 10 + d;
  }
  if (ovf) v = lim;
  const int64_t sv = neg ? (int64_t)(0 - v) : (int64_t)v;
  keys[k] = (uint64_t)(int64_t)(int32_t)sv;
}

__global__ void k_gather_keys(const uint32_t *__restrict__ ids, uint64_t n, const uint64_t *__restrict__ wk,
                              uint64_t nw, uint64_t *__restrict__ keys, uint32_t *__restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t id = ids[i];
  if (id >= nw) {
    *bad = 1;
    keys[i] = 0;
  } else {
    keys[i] = wk[id];
  }
}

// line of every token (upper bound in line_off) and its validity
__global__ void k_tok_lines(const int64_t *__restrict__ off, uint64_t nl, uint64_t n, int min_len,
                            int32_t *__restrict__ tline, uint32_t *__restrict__ pos) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint64_t lo = 0, hi = nl;  // largest l with off[l] <= t (empty lines share an offset: take the last)
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if ((uint64_t)off[mid] <= t)
      lo = mid;
    else
      hi = mid;
  }
  tline[t] = (int32_t)lo;
  pos[t] = (uint32_t)t;
}

// run heads of the sorted keys, and whether each sorted token lies in a valid
// (gathered) line
__global__ void k_run_heads(const uint64_t *__restrict__ k, const uint32_t *__restrict__ ps, uint64_t n,
                            const int32_t *__restrict__ tline, const int64_t *__restrict__ off, int min_len,
                            uint32_t *__restrict__ head, uint32_t *__restrict__ valid) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    valid[n] = 0;  // the exclusive scan's tail
    return;
  }
  head[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
  const int32_t l = tline[ps[i]];
  valid[i] = off[l + 1] - off[l] >= min_len ? 1u : 0u;
}

__global__ void k_run_starts(const uint64_t *__restrict__ ks, const uint32_t *__restrict__ head,
                             const uint32_t *__restrict__ rid1, uint64_t n, uint64_t *__restrict__ ukey,
                             uint32_t *__restrict__ rstart) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !head[i]) return;
  const uint32_t r = rid1[i] - 1;
  ukey[r] = ks[i];
  rstart[r] = (uint32_t)i;
}

// per run (one thread, no atomics: a hot word's run has millions of tokens):
// tokens in valid lines = difference of the valid-flag scan; first valid
// position = the first valid element (the sort is stable: positions ascend)
__global__ void k_run_stats(const uint32_t *__restrict__ rstart, uint32_t R, uint64_t n,
                            const uint32_t *__restrict__ vscan, const uint32_t *__restrict__ valid,
                            const uint32_t *__restrict__ ps, uint32_t *__restrict__ cnt, uint32_t *__restrict__ first) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint64_t s = rstart[r], e = r + 1 < R ? rstart[r + 1] : n;
  cnt[r] = vscan[e] - vscan[s];
  uint64_t i = s;
  while (i < e && !valid[i]) i++;
  first[r] = i < e ? ps[i] : 0xFFFFFFFFu;
}

__global__ void k_tok_vid(const uint32_t *__restrict__ ps, const uint32_t *__restrict__ rid1, uint64_t n,
                          const int32_t *__restrict__ vid_of_run, int32_t *__restrict__ tok) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) tok[ps[i]] = vid_of_run[rid1[i] - 1];
}

// (batch << 32 | vid) of every token of every batch's gather window; tokens
// of invalid lines (never gathered) get the sentinel, which sorts last
__global__ void k_sched_keys(const uint64_t *__restrict__ eoff, const int64_t *__restrict__ ta, uint32_t nb,
                             uint64_t E, const int32_t *__restrict__ tok, const int32_t *__restrict__ tline,
                             const uint8_t *__restrict__ valid, uint64_t *__restrict__ out) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  uint32_t lo = 0, hi = nb;  // batch: largest b with eoff[b] <= e
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (eoff[mid] <= e)
      lo = mid;
    else
      hi = mid;
  }
  const uint64_t t = (uint64_t)ta[lo] + (e - eoff[lo]);
  out[e] = valid[tline[t]] ? ((uint64_t)lo << 32) | (uint32_t)tok[t] : ~0ULL;
}

__global__ void k_uniq_flags(const uint64_t *__restrict__ k, uint64_t n, uint32_t *__restrict__ f) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = (k[i] != ~0ULL && (i == 0 || k[i] != k[i - 1])) ? 1u : 0u;
}

__global__ void k_uniq_scatter(const uint64_t *__restrict__ k, const uint32_t *__restrict__ f,
                               const uint32_t *__restrict__ at, uint64_t n, uint64_t *__restrict__ uk,
                               int32_t *__restrict__ K) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && f[i]) {
    uk[at[i]] = k[i];
    K[at[i]] = (int32_t)(uint32_t)k[i];
  }
}

// kofs[b] = first unique key of batch b (lower bound of b << 32)
__global__ void k_batch_kofs(const uint64_t *__restrict__ uk, uint64_t nu, uint32_t nb, uint64_t *__restrict__ kofs) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > nb) return;
  const uint64_t v = (uint64_t)b << 32;
  uint64_t lo = 0, hi = nu;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (uk[mid] < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  kofs[b] = lo;
}

template <typename T> int exclusive_scan(const T *in, T *out, uint64_t n, DevMem &tmp, hipStream_t s) {
  size_t b = 0;
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b, in, out, (int)n, s));
  SWPS_TRY(tmp.ensure(b));
  b = tmp.bytes;
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(tmp.p, b, in, out, (int)n, s));
  return SWPS_OK;
}
template <typename T> int inclusive_scan(const T *in, T *out, uint64_t n, DevMem &tmp, hipStream_t s) {
  size_t b = 0;
  SWPS_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, b, in, out, (int)n, s));
  SWPS_TRY(tmp.ensure(b));
  b = tmp.bytes;
  SWPS_HIP(hipcub::DeviceScan::InclusiveSum(tmp.p, b, in, out, (int)n, s));
  return SWPS_OK;
}

// Vocab + tokens from device keys [ntok] (consumed) and host line offsets.
int ingest_gpu(swps_w2v *w, DevMem &d_keys, uint64_t nt, std::vector<int64_t> &&line_off) {
  hipStream_t s = w->s;
  const uint64_t nl = line_off.size() - 1;
  if (nt >= (1ULL << 32)) return fail(SWPS_E_UNSUPPORTED, "more than 2^32 tokens per rank");
  w->line_off = std::move(line_off);
  w->line_valid.assign(nl, 0);
  uint64_t tw = 0;
  for (uint64_t l = 0; l < nl; l++) {
    const int64_t len = w->line_off[l + 1] - w->line_off[l];
    w->line_valid[l] = len >= w->cfg.min_sentence_length;
    if (w->line_valid[l]) tw += (uint64_t)len;
  }
  SWPS_TRY(upload(w->d_line_off, w->line_off, s));
  SWPS_TRY(w->d_tok.ensure(std::max<uint64_t>(nt, 1) * 4));
  SWPS_TRY(w->d_tok_line.ensure(std::max<uint64_t>(nt, 1) * 4));
  DevMem pos, ks, ps, head, rid1, valid, vscan, tmp;
  SWPS_TRY(pos.ensure(std::max<uint64_t>(nt, 1) * 4));
  SWPS_TRY(ks.ensure(std::max<uint64_t>(nt, 1) * 8));
  SWPS_TRY(ps.ensure(std::max<uint64_t>(nt, 1) * 4));
  if (nt) {
    k_tok_lines<<<nblk(nt), 256, 0, s>>>(w->d_line_off.as<int64_t>(), nl, nt, w->cfg.min_sentence_length,
                                          w->d_tok_line.as<int32_t>(), pos.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    size_t sb = 0;
    SWPS_HIP(sort_pairs(nullptr, sb, d_keys.as<uint64_t>(), ks.as<uint64_t>(), pos.as<uint32_t>(), ps.as<uint32_t>(),
                        nt, 64, s));
    SWPS_TRY(tmp.ensure(sb));
    sb = tmp.bytes;
    SWPS_HIP(sort_pairs(tmp.p, sb, d_keys.as<uint64_t>(), ks.as<uint64_t>(), pos.as<uint32_t>(), ps.as<uint32_t>(), nt,
                        64, s));
    d_keys.release();
    pos.release();
    SWPS_TRY(head.ensure(nt * 4));
    SWPS_TRY(rid1.ensure(nt * 4));
    SWPS_TRY(valid.ensure((nt + 1) * 4));
    SWPS_TRY(vscan.ensure((nt + 1) * 4));
    k_run_heads<<<nblk(nt + 1), 256, 0, s>>>(ks.as<uint64_t>(), ps.as<uint32_t>(), nt, w->d_tok_line.as<int32_t>(),
                                              w->d_line_off.as<int64_t>(), w->cfg.min_sentence_length,
                                              head.as<uint32_t>(), valid.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    SWPS_TRY(inclusive_scan(head.as<uint32_t>(), rid1.as<uint32_t>(), nt, tmp, s));
    SWPS_TRY(exclusive_scan(valid.as<uint32_t>(), vscan.as<uint32_t>(), nt + 1, tmp, s));
  }
  uint32_t nruns = 0;
  if (nt) SWPS_HIP(hipMemcpyAsync(&nruns, rid1.as<uint32_t>() + nt - 1, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  DevMem ukey, cnt, first, rstart;
  SWPS_TRY(ukey.ensure(std::max<uint32_t>(nruns, 1) * 8));
  SWPS_TRY(cnt.ensure(std::max<uint32_t>(nruns, 1) * 4));
  SWPS_TRY(first.ensure(std::max<uint32_t>(nruns, 1) * 4));
  SWPS_TRY(rstart.ensure(std::max<uint32_t>(nruns, 1) * 4));
  if (nt) {
    k_run_starts<<<nblk(nt), 256, 0, s>>>(ks.as<uint64_t>(), head.as<uint32_t>(), rid1.as<uint32_t>(), nt,
                                           ukey.as<uint64_t>(), rstart.as<uint32_t>());
    k_run_stats<<<nblk(nruns), 256, 0, s>>>(rstart.as<uint32_t>(), nruns, nt, vscan.as<uint32_t>(),
                                             valid.as<uint32_t>(), ps.as<uint32_t>(), cnt.as<uint32_t>(),
                                             first.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
  }
  ks.release();
  head.release();
  std::vector<uint64_t> hk(nruns);
  std::vector<uint32_t> hc(nruns), hf(nruns);
  if (nruns) {
    SWPS_HIP(hipMemcpyAsync(hk.data(), ukey.p, nruns * 8ULL, hipMemcpyDeviceToHost, s));
    SWPS_HIP(hipMemcpyAsync(hc.data(), cnt.p, nruns * 4ULL, hipMemcpyDeviceToHost, s));
    SWPS_HIP(hipMemcpyAsync(hf.data(), first.p, nruns * 4ULL, hipMemcpyDeviceToHost, s));
  }
  SWPS_HIP(hipStreamSynchronize(s));
  // _local_keys: std::unordered_set filled in first-occurrence order over the
  // valid lines; its iteration order is the vid order (ingest() above)
  std::vector<uint32_t> order;
  order.reserve(nruns);
  for (uint32_t r = 0; r < nruns; r++) {
    if (hc[r] == 0)
      return fail(SWPS_E_UNSUPPORTED, "a word occurs only in lines shorter than min_sentence_length "
                                      "(to_sample reads past word_freq in the reference)");
    order.push_back(r);
  }
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return hf[a] < hf[b]; });
  std::unordered_set<uint64_t> local_keys;
  for (uint32_t r : order) local_keys.insert(hk[r]);
  if (local_keys.size() < 5) return fail(SWPS_E_UNSUPPORTED, "fewer than 5 keys (word2vec_global.h:556 returns)");
  w->train_words = tw;
  w->vocab_keys.assign(local_keys.begin(), local_keys.end());
  const uint64_t V = w->vocab_keys.size();
  std::vector<std::pair<uint64_t, int32_t>> kv(V);
  for (uint64_t i = 0; i < V; i++) {
    if (w->vocab_keys[i] == 0)
      return fail(SWPS_E_UNSUPPORTED, "a vocab key hashes to 0 (the reference redraws such negatives)");
    kv[i] = {w->vocab_keys[i], (int32_t)i};
  }
  std::sort(kv.begin(), kv.end());  // runs are in ascending key order too
  std::vector<int32_t> vid_of_run(nruns);
  w->counts.assign(V, 0);
  for (uint32_t r = 0; r < nruns; r++) {
    vid_of_run[r] = kv[r].second;
    w->counts[kv[r].second] = (int32_t)hc[r];
  }
  DevMem dv;
  SWPS_TRY(upload(dv, vid_of_run, s));
  if (nt) {
    k_tok_vid<<<nblk(nt), 256, 0, s>>>(ps.as<uint32_t>(), rid1.as<uint32_t>(), nt, dv.as<int32_t>(),
                                        w->d_tok.as<int32_t>());
    SWPS_HIP(hipGetLastError());
  }
  SWPS_HIP(hipStreamSynchronize(s));
  w->tok.clear();
  w->tok_line.clear();
  w->ntok = nt;
  w->tok_on_device = true;
  w->loaded = true;
  return SWPS_OK;
}

// build_schedule (above) with the windows' key sets made on the device
int schedule_gpu(swps_w2v *w) {
  hipStream_t s = w->s;
  const uint64_t nl = w->line_off.size() - 1;
  const int B = w->cfg.minibatch;
  w->batches.clear();
  std::vector<int64_t> ta;     // window token start per batch (batches without a key set: empty)
  std::vector<uint64_t> eoff;  // window element offsets
  eoff.push_back(0);
  auto window_end = [&](uint64_t li) {  // the line after the B+3-valid-line window from li
    int count = 0;
    for (int task = 0; task < 3; task++)
      while (li < nl) {
        const uint64_t l = li++;
        if (!w->line_valid[l]) continue;
        if (++count > B) break;
      }
    return li;
  };
  uint64_t wa = 0, we = 0;
  bool haveK = false;
  auto emit = [&](uint64_t l0, uint64_t l1, bool withK) {
    w->batches.push_back(swps_w2v::Batch{l0, l1, 0, 0});
    const int64_t a = withK ? w->line_off[wa] : 0, e = withK ? w->line_off[we] : 0;
    ta.push_back(a);
    eoff.push_back(eoff.back() + (uint64_t)(e - a));
  };
  uint64_t start = 0, cur = 0, line_counter = 0, last = 0;
  for (uint64_t li = 0; li < nl; li++) {
    cur += (uint64_t)(w->line_off[li + 1] - w->line_off[li]);
    line_counter++;
    last = li + 1;
    if (line_counter == 1) {
      emit(start, li + 1, haveK);
      wa = li + 1;
      we = window_end(li + 1);
      haveK = true;
      start = li + 1;
    }
    if (line_counter % (uint64_t)B == 0) {
      emit(start, li + 1, haveK);
      wa = li + 1;
      we = window_end(li + 1);
      start = li + 1;
    }
    if (cur > w->train_words) break;
  }
  emit(start, last, haveK);
  const uint32_t nb = (uint32_t)w->batches.size();
  const uint64_t E = eoff.back();
  DevMem d_eoff, d_ta, d_valid, keys, keys_s, flags, at, uk, tmp, kofs;
  SWPS_TRY(upload(d_eoff, eoff, s));
  SWPS_TRY(upload(d_ta, ta, s));
  SWPS_TRY(upload(d_valid, w->line_valid, s));
  uint64_t nu = 0;
  if (E) {
    SWPS_TRY(keys.ensure(E * 8));
    SWPS_TRY(keys_s.ensure(E * 8));
    k_sched_keys<<<nblk(E), 256, 0, s>>>(d_eoff.as<uint64_t>(), d_ta.as<int64_t>(), nb, E, w->d_tok.as<int32_t>(),
                                          w->d_tok_line.as<int32_t>(), d_valid.as<uint8_t>(), keys.as<uint64_t>());
    SWPS_HIP(hipGetLastError());
    size_t sb = 0;
    SWPS_HIP(sort_keys(nullptr, sb, keys.as<uint64_t>(), keys_s.as<uint64_t>(), E, 64, s));
    SWPS_TRY(tmp.ensure(sb));
    sb = tmp.bytes;
    SWPS_HIP(sort_keys(tmp.p, sb, keys.as<uint64_t>(), keys_s.as<uint64_t>(), E, 64, s));
    keys.release();
    SWPS_TRY(flags.ensure((E + 1) * 4));
    SWPS_TRY(at.ensure((E + 1) * 4));
    k_uniq_flags<<<nblk(E), 256, 0, s>>>(keys_s.as<uint64_t>(), E, flags.as<uint32_t>());
    SWPS_HIP(hipMemsetAsync(flags.as<uint32_t>() + E, 0, 4, s));
    SWPS_TRY(exclusive_scan(flags.as<uint32_t>(), at.as<uint32_t>(), E + 1, tmp, s));
    uint32_t n32 = 0;
    SWPS_HIP(hipMemcpyAsync(&n32, at.as<uint32_t>() + E, 4, hipMemcpyDeviceToHost, s));
    SWPS_HIP(hipStreamSynchronize(s));
    nu = n32;
    SWPS_TRY(uk.ensure(std::max<uint64_t>(nu, 1) * 8));
    SWPS_TRY(w->d_K.ensure(std::max<uint64_t>(nu, 1) * 4));
    k_uniq_scatter<<<nblk(E), 256, 0, s>>>(keys_s.as<uint64_t>(), flags.as<uint32_t>(), at.as<uint32_t>(), E,
                                            uk.as<uint64_t>(), w->d_K.as<int32_t>());
    SWPS_HIP(hipGetLastError());
  } else {
    SWPS_TRY(w->d_K.ensure(4));
    SWPS_TRY(uk.ensure(8));
  }
  SWPS_TRY(kofs.ensure((nb + 1ULL) * 8));
  k_batch_kofs<<<nblk(nb + 1ULL), 256, 0, s>>>(uk.as<uint64_t>(), nu, nb, kofs.as<uint64_t>());
  SWPS_HIP(hipGetLastError());
  std::vector<uint64_t> hk(nb + 1);
  SWPS_HIP(hipMemcpyAsync(hk.data(), kofs.p, (nb + 1ULL) * 8, hipMemcpyDeviceToHost, s));
  w->allK.resize(nu);
  if (nu) SWPS_HIP(hipMemcpyAsync(w->allK.data(), w->d_K.p, nu * 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  w->max_tok = w->max_U = w->max_lines = 0;
  for (uint32_t b = 0; b < nb; b++) {
    auto &bt = w->batches[b];
    bt.kofs = hk[b];
    bt.U = (uint32_t)(hk[b + 1] - hk[b]);
    w->max_tok = std::max<uint64_t>(w->max_tok, (uint64_t)(w->line_off[bt.l1] - w->line_off[bt.l0]));
    w->max_U = std::max<uint64_t>(w->max_U, bt.U);
    w->max_lines = std::max<uint64_t>(w->max_lines, bt.l1 - bt.l0);
  }
  return SWPS_OK;
}

// text file -> device keys + line offsets (load_text's split on ' ' and '\n'
// only; a file holding a NUL byte takes the host path, whose lines end at
// their first NUL like the reference's std::string(cline))
int tokenize_gpu(swps_w2v *w, const std::vector<char> &text, DevMem &d_keys, uint64_t &nt,
                 std::vector<int64_t> &line_off) {
  hipStream_t s = w->s;
  const uint64_t nb = text.size();
  DevMem d_text, st, nlf, tix, lix, tstart, d_off, tmp;
  SWPS_TRY(d_text.ensure(std::max<uint64_t>(nb, 1)));
  if (nb) SWPS_HIP(hipMemcpyAsync(d_text.p, text.data(), nb, hipMemcpyHostToDevice, s));
  SWPS_TRY(st.ensure((nb + 1) * 4));
  SWPS_TRY(nlf.ensure((nb + 1) * 4));
  SWPS_TRY(tix.ensure((nb + 1) * 4));
  SWPS_TRY(lix.ensure((nb + 1) * 4));
  k_text_flags<<<nblk(nb + 1), 256, 0, s>>>(d_text.as<char>(), nb, st.as<uint32_t>(), nlf.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  SWPS_TRY(exclusive_scan(st.as<uint32_t>(), tix.as<uint32_t>(), nb + 1, tmp, s));
  SWPS_TRY(exclusive_scan(nlf.as<uint32_t>(), lix.as<uint32_t>(), nb + 1, tmp, s));
  uint32_t tot[2];
  SWPS_HIP(hipMemcpyAsync(&tot[0], tix.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipMemcpyAsync(&tot[1], lix.as<uint32_t>() + nb, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  nt = tot[0];
  const uint64_t nnl = tot[1];
  const uint64_t nlines = nnl + ((nb && text[nb - 1] != '\n') ? 1 : 0);
  SWPS_TRY(tstart.ensure(std::max<uint64_t>(nt, 1) * 8));
  SWPS_TRY(d_off.ensure((nlines + 2) * 8));
  SWPS_HIP(hipMemsetAsync(d_off.p, 0, 8, s));
  if (nb)
    k_text_index<<<nblk(nb), 256, 0, s>>>(d_text.as<char>(), nb, st.as<uint32_t>(), tix.as<uint32_t>(),
                                           lix.as<uint32_t>(), tstart.as<uint64_t>(), d_off.as<int64_t>());
  SWPS_HIP(hipGetLastError());
  SWPS_TRY(d_keys.ensure(std::max<uint64_t>(nt, 1) * 8));
  if (nt)
    k_text_keys<<<nblk(nt), 256, 0, s>>>(d_text.as<char>(), nb, tstart.as<uint64_t>(), nt,
                                          w->cfg.key_mode == SWPS_KEY_ATOI, d_keys.as<uint64_t>());
  SWPS_HIP(hipGetLastError());
  line_off.assign(nlines + 1, 0);
  if (nnl) SWPS_HIP(hipMemcpyAsync(line_off.data(), d_off.p, (nnl + 1) * 8, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  line_off[nlines] = (int64_t)nt;  // a last line without '\n'
  return SWPS_OK;
}

int upload_corpus(swps_w2v *w) {
  hipStream_t s = w->s;
  const uint64_t V = w->vocab_keys.size();
  if (!w->tok_on_device) {
    SWPS_TRY(upload(w->d_tok, w->tok, s));
    SWPS_TRY(upload(w->d_tok_line, w->tok_line, s));
    SWPS_TRY(upload(w->d_K, w->allK, s));
  }
  SWPS_TRY(upload(w->d_line_off, w->line_off, s));
  SWPS_TRY(tok_fingerprint(w));
  std::vector<int64_t> btok;  // token offset of every batch start + the epoch end
  for (auto &b : w->batches) btok.push_back(w->line_off[b.l0]);
  btok.push_back(w->line_off[w->batches.back().l1]);
  SWPS_TRY(upload(w->d_btok, btok, s));
  // subsampling thresholds (word2vec_global.h:728-729), computed on the host
  std::vector<float> ran(V);
  for (uint64_t i = 0; i < V; i++) {
    float freq = float(w->counts[i]) / (float)w->train_words;
    ran[i] = (float)(1 - std::sqrt((double)(w->cfg.sample / freq)));
  }
  SWPS_TRY(upload(w->d_ran, ran, s));
  // ExpTable (word2vec_global.h:252-258)
  std::vector<float> ex(1000);
  for (int i = 0; i < 1000; i++) {
    float x = (i / (float)1000 * 2 - 1) * 6;
    float e = (float)std::exp((double)x);
    ex[i] = e / (e + 1);
  }
  SWPS_TRY(upload(w->d_exptab, ex, s));
  if (w->cfg.sampler == SWPS_SAMPLER_ALIAS) {
    if (!w->cfg.minibatch_vocab) {
      w->alias.clear();
      build_alias(w->counts.data(), V, w->alias);
    }
    SWPS_TRY(upload(w->d_alias, w->alias, s));
  }
  if (w->cfg.minibatch_vocab) {
    SWPS_TRY(upload(w->d_bstarts, w->bstarts, s));
    SWPS_TRY(upload(w->d_UK, w->allUK, s));
    SWPS_TRY(upload(w->d_bcnt_tok, w->bcnt_tok, s));
    SWPS_TRY(w->d_tw.ensure(w->batches.size() * 4));
  } else if (w->cfg.sampler != SWPS_SAMPLER_ALIAS) {
    std::vector<uint64_t> starts;
    unigram_starts(w->vocab_keys.data(), w->counts.data(), V, w->cfg.unigram_size, starts);
    SWPS_TRY(upload(w->d_starts, starts, s));
    SWPS_TRY(w->d_unigram.ensure(w->cfg.unigram_size * 4));
    k_build_unigram<<<4096, 256, 0, s>>>(w->d_starts.as<uint64_t>(), (uint32_t)V, w->cfg.unigram_size,
                                         w->d_unigram.as<int32_t>());
    SWPS_HIP(hipGetLastError());
    const uint64_t nb1 = ((w->cfg.unigram_size - 1) >> kUShift) + 2;
    SWPS_TRY(w->d_uidx.ensure(nb1 * 4));
    k_build_uidx<<<nblk(nb1), 256, 0, s>>>(w->d_starts.as<uint64_t>(), (uint32_t)V, kUShift, nb1,
                                           w->d_uidx.as<int32_t>());
    SWPS_HIP(hipGetLastError());
  }
  const size_t es = w->f64 ? 8 : 4;
  w->cs = row_ld(w->D, es, w->cache_pad);
  SWPS_TRY(w->d_cache_h.ensure(V * w->cs * es));
  SWPS_TRY(w->d_cache_v.ensure(V * w->cs * es));
  SWPS_TRY(w->d_local.ensure(V * 4));
  SWPS_HIP(hipMemsetAsync(w->d_local.p, 0xFF, V * 4, s));
  SWPS_TRY(w->d_vid_row.ensure(V * 4));
  SWPS_HIP(hipStreamSynchronize(s));  // host vectors above go out of scope
  return SWPS_OK;
}

template <typename T> int pull_all(swps_w2v *w) {
  const uint64_t V = w->vocab_keys.size();
  k_pull<T><<<nblk(V * 64), 256, 0, w->s>>>(nullptr, (uint32_t)V, w->d_vid_row.as<uint32_t>(), w->t->rows.as<T>(),
                                            w->D, w->d_cache_h.as<T>(), w->d_cache_v.as<T>(), w->d_local.as<int32_t>(),
                                            0, w->cs);
  SWPS_HIP(hipGetLastError());
  SWPS_HIP(hipStreamSynchronize(w->s));
  return SWPS_OK;
}

// Vec::randInit (vec1.h:229-232) for every vocab key on the GPU: rand() is
// glibc's additive generator o[i] = o[i-31] + o[i-3] (mod 2^32, output o >> 1;
// GlibcRand in swps_host.cpp), linear in its state, so output m is
// sum_j a_j o[3+j] with sum_j a_j x^j = x^(m-3) mod (x^31 - x^28 - 1):
// every thread jumps to its own run of outputs (square-and-multiply on
// 31-coefficient polynomials) and then steps the recurrence.  Output k
// (after `skip` earlier calls) is element k % 2D of key k / 2D's [h | v],
// (rand()/(float)RAND_MAX - 0.5) / D, written straight into the table row.
template <typename T>
__global__ __launch_bounds__(64) void k_rand_init(const uint32_t *__restrict__ base, uint64_t first, uint64_t total,
                                                   int D, const uint32_t *__restrict__ vid_row, T *__restrict__ rows) {
  const uint64_t k0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * kRandRun;
  if (k0 >= total) return;
  // o[m] for the 31 values before output k0: m = first + k0 - 31 + d, d = 0..30
  uint32_t ring[31];
  glibc_ring_at(base, first + k0 - 31, ring);
  const uint64_t k1 = min(total, k0 + kRandRun);
  int h = 0;  // ring[h] = o[i-31], ring[(h+28)%31] = o[i-3]
  for (uint64_t k = k0; k < k1; k++) {
    const int h28 = h + 28 >= 31 ? h + 28 - 31 : h + 28;
    const uint32_t v = ring[h] + ring[h28];
    ring[h] = v;
    h = h + 1 == 31 ? 0 : h + 1;
    const float f = (float)(int32_t)(v >> 1) / (float)2147483647;
    const uint64_t key = k / (2 * (uint64_t)D), el = k % (2 * (uint64_t)D);
    rows[(uint64_t)vid_row[key] * 4 * D + el] = (T)(((double)f - 0.5) / (double)(size_t)D);
  }
}

template <typename T>
__global__ void k_zero_sums(const uint32_t *__restrict__ vid_row, uint64_t V, int D, T *__restrict__ rows) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= V * 2 * (uint64_t)D) return;
  const uint64_t key = i / (2 * (uint64_t)D), el = i % (2 * (uint64_t)D);
  rows[(uint64_t)vid_row[key] * 4 * D + 2 * D + el] = (T)0;
}

template <typename T> int rand_init_gpu(swps_w2v *w) {
  const uint64_t V = w->vocab_keys.size();
  const int D = w->D;
  // o[3..33] after srand(seed) (GlibcRand's seeding, swps_host.cpp)
  const std::vector<uint32_t> base = glibc_base(w->cfg.rand_seed);
  const uint64_t total = V * 2 * (uint64_t)D;
  const uint64_t first = 344 + w->cfg.rand_offset;  // o index of the first output used
  DevMem d_base;
  SWPS_TRY(upload(d_base, base, w->s));
  const uint64_t nthr = (total + kRandRun - 1) / kRandRun;
  if (total) {
    k_rand_init<T><<<nblk(nthr, 64), 64, 0, w->s>>>(d_base.as<uint32_t>(), first, total, D,
                                                    w->d_vid_row.as<uint32_t>(), w->t->rows.as<T>());
    k_zero_sums<T><<<nblk(total), 256, 0, w->s>>>(w->d_vid_row.as<uint32_t>(), V, D, w->t->rows.as<T>());
  }
  SWPS_HIP(hipGetLastError());
  SWPS_HIP(hipStreamSynchronize(w->s));
  return pull_all<T>(w);
}

template <typename T> int set_hv(swps_w2v *w, const double *hv) {
  const uint64_t V = w->vocab_keys.size();
  const int D = w->D;
  std::vector<T> rows(V * 4 * D, (T)0);
  for (uint64_t i = 0; i < V; i++)
    for (int e = 0; e < 2 * D; e++) rows[i * 4 * D + e] = (T)hv[i * 2 * D + e];
  DevMem d;
  SWPS_TRY(upload(d, rows, w->s));
  SWPS_TRY(table_set_rows(w->t, w->d_vid_row.as<uint32_t>(), V, d.p, w->s));
  SWPS_HIP(hipStreamSynchronize(w->s));
  return pull_all<T>(w);
}

template <int NCH, typename T, typename A> void launch_forward(const FwdArgs<T, A> &a, hipStream_t s) {
  if (sizeof(A) == 8)  // fp64 intermediates: the batched target reduction wins
    k_forward_b8<T, A, NCH, 8><<<nblk((uint64_t)a.P * 64), 256, 0, s>>>(a);
  else
    k_forward<T, A, NCH, 8><<<nblk((uint64_t)a.P * 64), 256, 0, s>>>(a);
}
// at most max_items / kGroup leaders, 4 per block
inline bool use_combine(const swps_w2v *w, uint64_t M) {
  return w->combine == 1 || (w->combine == 2 && M >= w->combine_min);
}
inline unsigned combine_grid(uint64_t max_items) {
  return (unsigned)std::min<uint64_t>(kCombineGrid, max_items / kGroup / 4 + 1);
}
template <int NCH, typename T, typename A>
void launch_gather(const GatherArgs<A> &a, unsigned grid, unsigned cgrid, hipStream_t s) {
  constexpr int UNR = sizeof(A) * V16<T>::E > 16 ? 4 : 8;
  k_gather<T, A, NCH, UNR><<<grid, 256, 0, s>>>(a);
  if (cgrid) k_combine<T, A, NCH><<<cgrid, 256, 0, s>>>(a);
}
template <int NCH, typename T, typename A> void launch_push(const PushArgs<T, A> &a, hipStream_t s) {
  if (a.grads)
    k_push<T, A, NCH, true><<<nblk((uint64_t)a.U * 64), 256, 0, s>>>(a);
  else
    k_push<T, A, NCH, false><<<nblk((uint64_t)a.U * 64), 256, 0, s>>>(a);
}
constexpr uint32_t kChunk = 128;  // a (key, kind) run of at most kChunk records is one item
// chunk size of the longer runs: kChunk (SWPS_MULTI_CHUNK sets 1..128 for A/B: 32 and 16 at
// B = 100 lines were 4 % and 7 % slower — more partials and second-level groups, no latency win)
inline uint32_t multi_chunk(const swps_w2v *w, uint64_t) { return w->multi_chunk ? w->multi_chunk : kChunk; }
constexpr uint64_t kOverlapTok = 1000000;  // auto-overlap threshold (tokens per minibatch)

// Subsample masks and main-LCG offsets for a whole epoch.  They depend only on
// the two RNG streams (the float LCG advances one draw per processed token,
// the main LCG 1 + kept*(1+negative) draws per line), never on the
// parameters, so one pass per epoch replaces per-batch host syncs.
// Size every per-batch buffer for the epoch's largest batch once, at plan
// time, so no hipMalloc / hipFree (a device-wide sync) lands inside a step.
int presize(swps_w2v *w, uint64_t maxP) {
  if (maxP == 0) return SWPS_OK;
  const int W = w->W, N = w->N, D = w->D, RS = 2 * W + N + 2;
  const uint64_t HOFF = maxP * (uint64_t)(N + 1), M = HOFF + maxP * (uint64_t)(2 * W);
  if (M >= (1ULL << 31)) return SWPS_OK;  // prep_batch reports it
  const size_t a = (w->f64 || w->cfg.fp64_intermediates) ? 8 : 4;  // partials (split mode: fp64 too)
  const uint64_t nrow = w->bfp ? (uint64_t)bfp_ld(D, w->bfp_rb) * 4 : (uint64_t)row_ld(D, a, w->row_pad) * a;
  SWPS_TRY(w->d_pos_tok.ensure(maxP * 4));
  SWPS_TRY(w->d_rec.ensure(maxP * RS * 4));
  SWPS_TRY(w->d_pkeys.ensure(M * 4));
  SWPS_TRY(w->d_pvals.ensure(M * 4));
  SWPS_TRY(w->d_pkeys_s.ensure(M * 4));
  SWPS_TRY(w->d_pvals_s.ensure(M * 4));
  SWPS_TRY(w->d_neu1.ensure(maxP * nrow));
  SWPS_TRY(w->d_neu1e.ensure(maxP * nrow));
  SWPS_TRY(w->d_pg.ensure(HOFF * 4));
  const uint64_t U = w->max_U;
  if (U) {
    int bits = 1;
    while ((1ULL << bits) <= U) bits++;
    // smaller batches of the epoch may take the small-tile sort (swps_sort.h): size for both
    for (uint64_t n : {M, std::min<uint64_t>(M, kSmallSort - 1)}) {
      size_t sb = 0, si = 0;
      SWPS_HIP(sort_pairs(nullptr, sb, w->d_pkeys.as<uint32_t>(), w->d_pkeys_s.as<uint32_t>(),
                          w->d_pvals.as<uint32_t>(), w->d_pvals_s.as<uint32_t>(), n, bits, w->s));
      SWPS_HIP(sort_pairs_iota(nullptr, si, w->d_pkeys.as<uint32_t>(), w->d_pkeys_s.as<uint32_t>(),
                               w->d_pvals_s.as<uint32_t>(), n, bits, w->s));
      SWPS_TRY(w->d_tmp.ensure(std::max(sb, si)));
    }
    const uint64_t max_items = 2ULL * U + M / multi_chunk(w, maxP) + 1;
    SWPS_TRY(w->d_lead.ensure((max_items / 8 + 2) * 4));
    SWPS_TRY(w->d_seg.ensure(U * 16));
    SWPS_TRY(w->d_icnt.ensure((2ULL * U + 1) * 4));
    SWPS_TRY(w->d_ioff.ensure((2ULL * U + 1) * 4));
    SWPS_TRY(w->d_desc.ensure(max_items * 16));
    SWPS_TRY(w->d_partial.ensure(max_items * D * a));
    SWPS_TRY(w->d_multi.ensure((max_items + 1) * 4));
    if (w->multi_sort && maxP >= w->multi_sort_min) {  // the multi-item order sort (prep_batch)
      SWPS_TRY(w->d_pkeys.ensure(max_items * 4));
      SWPS_TRY(w->d_pvals.ensure(max_items * 4));
      SWPS_TRY(w->d_icnt.ensure(max_items * 4));
      for (uint64_t n : {max_items, std::min<uint64_t>(max_items, kSmallSort - 1)}) {
        size_t mb = 0;
        SWPS_HIP(sort_pairs(nullptr, mb, w->d_pkeys.as<uint32_t>(), w->d_icnt.as<uint32_t>(),
                            w->d_pvals.as<uint32_t>(), w->d_multi.as<uint32_t>(), n, 16, w->s));
        SWPS_TRY(w->d_tmp.ensure(mb));
      }
    }
  }
  return SWPS_OK;
}

int plan_epoch(swps_w2v *w) {
  hipStream_t s = w->s;
  const uint64_t nb = w->batches.size();
  const uint64_t L = w->batches[nb - 1].l1;             // lines processed per epoch
  const uint64_t T = (uint64_t)w->line_off[L];          // tokens processed per epoch
  const bool sample_on = w->cfg.sample >= 0;
  SWPS_TRY(w->d_kflag.ensure((T + 1) * 4));
  SWPS_TRY(w->d_kscan.ensure((T + 1) * 4));
  SWPS_TRY(w->d_ldraw.ensure((L + 1) * 8));
  SWPS_TRY(w->d_ldoff.ensure((L + 1) * 8));
  hipEvent_t ek = w->timer.begin(s);
  std::vector<int32_t> tw;
  if (w->cfg.minibatch_vocab) {
    // _num_words when batch b of epoch e trains: the first full gather, e whole
    // epochs of gathers (incl. each epoch's final short gather), this epoch's
    // gathers up to b; `int train_words = num_words()` truncates to 32 bits
    const uint64_t e = w->cursor / nb;
    uint64_t per_epoch = w->gather_end;
    for (auto &b : w->batches) per_epoch += b.gathered;
    uint64_t acc = w->train_words + e * per_epoch;
    tw.resize(nb);
    for (uint64_t b = 0; b < nb; b++) {
      acc += w->batches[b].gathered;
      tw[b] = (int32_t)(uint32_t)acc;
    }
    SWPS_HIP(hipMemcpyAsync(w->d_tw.p, tw.data(), nb * 4, hipMemcpyHostToDevice, s));
    k_keep_mb<<<nblk((T + kKeepRun) / kKeepRun), 256, 0, s>>>(w->d_bcnt_tok.as<int32_t>(), T, w->d_btok.as<int64_t>(),
                                                              (uint32_t)nb, w->d_tw.as<int32_t>(), w->cfg.sample,
                                                              w->fstate, sample_on, w->d_kflag.as<int32_t>());
  } else {
    k_keep<<<nblk((T + 64 * kKeepIt) / (64 * kKeepIt) * 64), 256, 0, s>>>(w->d_tok.as<int32_t>(), T, w->d_ran.as<float>(),
                                                                          w->fstate, sample_on, w->d_kflag.as<int32_t>());
  }
  SWPS_HIP(hipGetLastError());
  size_t tb1 = 0, tb2 = 0;
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb1, w->d_kflag.as<int32_t>(), w->d_kscan.as<int32_t>(),
                                            (int)(T + 1), s));
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, w->d_ldraw.as<uint64_t>(), w->d_ldoff.as<uint64_t>(),
                                            (int)(L + 1), s));
  SWPS_TRY(w->d_tmp.ensure(std::max(tb1, tb2)));
  size_t tb = w->d_tmp.bytes;
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(w->d_tmp.p, tb, w->d_kflag.as<int32_t>(), w->d_kscan.as<int32_t>(),
                                            (int)(T + 1), s));
  k_line_draws<<<nblk(L + 1), 256, 0, s>>>(w->d_line_off.as<int64_t>(), L, w->d_kscan.as<int32_t>(), w->N,
                                           w->d_ldraw.as<uint64_t>());
  SWPS_HIP(hipGetLastError());
  tb = w->d_tmp.bytes;
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(w->d_tmp.p, tb, w->d_ldraw.as<uint64_t>(), w->d_ldoff.as<uint64_t>(),
                                            (int)(L + 1), s));
  w->timer.end(KT_KEEP, ek, s);
  // per-batch kept counts: kscan at every batch's token boundary
  SWPS_TRY(w->d_bounds.ensure((nb + 1) * 4));
  k_bounds<<<nblk(nb + 1), 256, 0, s>>>(w->d_kscan.as<int32_t>(), w->d_btok.as<int64_t>(), nb + 1,
                                        w->d_bounds.as<int32_t>());
  SWPS_HIP(hipGetLastError());
  std::vector<int32_t> ks(nb + 1);
  SWPS_HIP(hipMemcpyAsync(ks.data(), w->d_bounds.p, (nb + 1) * 4, hipMemcpyDeviceToHost, s));
  uint64_t draws = 0;
  SWPS_HIP(hipMemcpyAsync(&draws, w->d_ldoff.as<uint64_t>() + L, 8, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  w->plan_P.resize(nb);
  uint64_t maxP = 0;
  for (uint64_t i = 0; i < nb; i++) {
    w->plan_P[i] = (uint32_t)(ks[i + 1] - ks[i]);
    maxP = std::max<uint64_t>(maxP, w->plan_P[i]);
  }
  SWPS_TRY(presize(w, maxP));
  w->lstate_epoch = w->lstate;
  w->fstate_epoch = w->fstate;
  w->lstate = lcg_jump(w->lstate, draws, kLcgA, kLcgC);
  if (sample_on) w->fstate = lcg_jump(w->fstate, T, kFlcgA, kLcgC);
  return SWPS_OK;
}

// ---- one minibatch, in two halves ------------------------------------------
// prep_batch: everything that depends only on the corpus, the RNG streams and
// the batch's key set — the epoch plan, the local key map, the position and
// gradient records (learn_instance's draws) and the inverted index (sorted
// records, segments, chunk descriptors).  learn_batch: everything that reads
// parameters — pull (or install of the owners' values), forward, gathered
// gradient sums, push.  The sharded driver issues prep(i+1) right after
// learn(i) on the compute stream, so it runs while minibatch i's push and
// i+1's pull cross the fabric (exact lockstep semantics kept).
__global__ void k_set_local(const int32_t *__restrict__ K, uint32_t U, int32_t *__restrict__ local) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < U) local[K[u]] = (int32_t)u;
}

// k_set_local and k_positions in one launch (thread i does both jobs' i-th item)
__global__ void k_batch_setup(const int32_t *__restrict__ K, uint32_t U, int32_t *__restrict__ local,
                              const int32_t *__restrict__ kscan, uint64_t t0, uint64_t nt,
                              int32_t *__restrict__ pos_tok, uint4 *__restrict__ seg0, uint32_t *__restrict__ lead,
                              uint32_t *__restrict__ multi, const uint32_t *__restrict__ vid_row,
                              uint32_t *__restrict__ krow) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < U) local[K[i]] = (int32_t)i;
  if (krow && i < U) krow[i] = vid_row[K[i]];  // the batch keys' shard rows (k_push_thp)
  if (seg0 && i < U) seg0[i] = make_uint4(0, 0, 0, 0);  // seg[4][U] u32 = U x 16 B: keys without records
  if (lead && i == 0) lead[0] = 0;
  if (multi && i == 0) multi[0] = 0;
  if (i < nt && pos_tok) {
    const int32_t a = kscan[t0 + i];
    if (kscan[t0 + i + 1] != a) pos_tok[a - kscan[t0]] = (int32_t)(t0 + i);
  }
}

// Segment bounds of every (local key, kind) run of the sorted records, one
// thread per record (records of key u: its h records, index < HOFF, then its
// v records, each run in index order: the sort is stable).  seg[0][u],
// seg[1][u] = h-record range; seg[2][u], seg[3][u] = v-record range; keys
// without records keep the zeros k_batch_setup wrote.
__global__ void k_seg_bounds(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ vals, uint32_t M,
                             uint32_t HOFF, uint32_t U, uint32_t *__restrict__ seg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const uint32_t u = keys[i];
  if (u >= U) return;  // "no key" records sort last
  const bool first = i == 0 || keys[i - 1] != u, last = i + 1 == M || keys[i + 1] != u;
  const bool isv = vals[i] >= HOFF;
  if (first) seg[u] = i;
  if (last) seg[3 * U + u] = i + 1;
  // the h/v split: the first v record, or the run's end when it has none
  if ((first && isv) || (!first && isv && vals[i - 1] < HOFF)) {
    seg[U + u] = i;
    seg[2 * U + u] = i;
  } else if (last && !isv) {
    seg[U + u] = i + 1;
    seg[2 * U + u] = i + 1;
  }
}

// k_seg_bounds with 4 consecutive records per thread (16-B loads of the sorted keys and their
// record indices; the neighbours on either side from the next / previous thread's words): the same
// bounds, a quarter of the threads and load instructions
__global__ __launch_bounds__(256) void k_seg_bounds4(const uint32_t *__restrict__ keys,
                                                     const uint32_t *__restrict__ vals, uint32_t M, uint32_t HOFF,
                                                     uint32_t U, uint32_t *__restrict__ seg) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x, i0 = q * 4;
  if (i0 >= M) return;
  constexpr uint32_t kNone = 0xFFFFFFFFu;  // past either end: no key
  uint32_t k[6], v[5];
  if (i0 + 4 <= M) {
    const uint4 kk = ((const uint4 *)keys)[q], vv = ((const uint4 *)vals)[q];
    k[1] = kk.x, k[2] = kk.y, k[3] = kk.z, k[4] = kk.w;
    v[1] = vv.x, v[2] = vv.y, v[3] = vv.z, v[4] = vv.w;
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      k[j + 1] = i0 + j < M ? keys[i0 + j] : kNone;
      v[j + 1] = i0 + j < M ? vals[i0 + j] : 0u;
    }
  }
  k[0] = i0 ? keys[i0 - 1] : kNone;
  v[0] = i0 ? vals[i0 - 1] : 0u;
  k[5] = i0 + 4 < M ? keys[i0 + 4] : kNone;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t i = i0 + j, u = k[j + 1];
    if (i >= M || u >= U) continue;  // "no key" records sort last
    const bool first = k[j] != u, last = k[j + 2] != u;
    const bool isv = v[j + 1] >= HOFF;
    if (first) seg[u] = i;
    if (last) seg[3 * U + u] = i + 1;
    if ((first && isv) || (!first && isv && v[j] < HOFF)) {
      seg[U + u] = i;
      seg[2 * U + u] = i;
    } else if (last && !isv) {
      seg[U + u] = i + 1;
      seg[2 * U + u] = i + 1;
    }
  }
}

// chunks of <= CH records per (key, kind) from the bounds; cnt[2U] = 0 (the
// scan's tail).  Profiled passes (gstats) also add the records / items to
// gstats[0..1].
__global__ void k_seg_counts(const uint32_t *__restrict__ seg, uint32_t U, uint32_t CH, uint32_t CHM,
                             uint32_t *__restrict__ cnt, unsigned long long *__restrict__ gstats) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long rc = 0, ic = 0, mr = 0, mi = 0;
  if (u == U) cnt[2 * U] = 0;
  if (u < U) {
    const uint32_t a = seg[u], lo = seg[U + u], b = seg[3 * U + u];
    // a run of <= CH records is one item; longer runs are chunks of CHM <= CH
    const uint32_t nh = lo - a, nv = b - lo;
    const uint32_t ch = nh <= CH ? (nh > 0) : (nh + CHM - 1) / CHM, cv = nv <= CH ? (nv > 0) : (nv + CHM - 1) / CHM;
    cnt[2 * u] = ch;
    cnt[2 * u + 1] = cv;
    rc = b - a;
    ic = ch + cv;
    mr = (ch > 1 ? lo - a : 0) + (cv > 1 ? b - lo : 0);  // multi-chunk runs: k_gather_t's share when fused
    mi = (ch > 1 ? ch : 0) + (cv > 1 ? cv : 0);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    rc += __shfl_xor(rc, off, 64);
    ic += __shfl_xor(ic, off, 64);
    mr += __shfl_xor(mr, off, 64);
    mi += __shfl_xor(mi, off, 64);
  }
  if (gstats && (threadIdx.x & 63) == 0 && rc) {
    atomicAdd(&gstats[0], rc);
    atomicAdd(&gstats[1], ic);
    atomicAdd(&gstats[2], mr);
    atomicAdd(&gstats[3], mi);
  }
}

int prep_batch(swps_w2v *w) {
  if (w->pb.valid) return SWPS_OK;
  const uint64_t nb = w->batches.size();
  if (w->cursor % nb == 0) SWPS_TRY(plan_epoch(w));
  const uint64_t bi = w->cursor % nb;
  const swps_w2v::Batch &B = w->batches[bi];
  hipStream_t s = w->s;
  Timer &tm = w->timer;
  const int W = w->W, N = w->N;
  const uint64_t t0 = (uint64_t)w->line_off[B.l0], t1 = (uint64_t)w->line_off[B.l1];
  const uint64_t nt = t1 - t0;
  const uint32_t U = B.U;
  const int32_t *K = w->d_K.as<int32_t>() + B.kofs;
  const uint64_t P = w->plan_P[bi];
  auto &pb = w->pb;
  pb = swps_w2v::Prepped();
  pb.bi = bi;
  pb.P = P;
  pb.U = U;
  pb.nt = nt;
  // local key map of the batch (the grads[key] slots the pull resets,
  // global_pull_access.h:88-97; cleared again by the push) and the batch's
  // kept token indices, in one launch
  const bool tracing = w->trace.size() < w->trace_cap;
  const bool recs = P > 0 && (U > 0 || tracing);
  if (recs) SWPS_TRY(w->d_pos_tok.ensure(P * 4));
  const bool will_sort = recs && U > 0;
  if (will_sort) {  // zeroed by k_batch_setup: keys without records keep empty segments
    SWPS_TRY(w->d_seg.ensure((uint64_t)U * 16));
    // leaders: at most 2 per 17 items (a run of kGroup + 1 chunks has two)
    const uint64_t mi = 2ULL * U + P * (uint64_t)(N + 1 + 2 * W) / multi_chunk(w, P) + 1;  // max items
    SWPS_TRY(w->d_lead.ensure((mi / 8 + 2) * 4));
    SWPS_TRY(w->d_multi.ensure((mi + 1) * 4));
  }
  // the fused push's per-key shard rows (single GPU)
  const bool krow = U > 0 && !w->sharded && (w->bfp || (w->tail && w->fused_push && w->push_tg_var == 5));
  if (krow) SWPS_TRY(w->d_krow.ensure((uint64_t)U * 4));
  if (U || recs) {
    k_batch_setup<<<nblk(std::max<uint64_t>(U, recs ? nt : 0)), 256, 0, s>>>(
        K, U, w->d_local.as<int32_t>(), w->d_kscan.as<int32_t>(), t0, recs ? nt : 0,
        recs ? w->d_pos_tok.as<int32_t>() : nullptr, will_sort ? w->d_seg.as<uint4>() : nullptr,
        will_sort ? w->d_lead.as<uint32_t>() : nullptr, will_sort ? w->d_multi.as<uint32_t>() : nullptr,
        w->d_vid_row.as<uint32_t>(), krow ? w->d_krow.as<uint32_t>() : nullptr);
    SWPS_HIP(hipGetLastError());
  }
  if (recs) {
    // ---- position records + gradient records (learn_instance's draws) ----
    const uint64_t HOFF = P * (uint64_t)(N + 1);
    const uint64_t M = HOFF + P * (uint64_t)(2 * W);
    const int RS = 2 * W + N + 2;
    if (M >= (1ULL << 31)) return fail(SWPS_E_UNSUPPORTED, "minibatch too large (2^31 gradient records)");
    SWPS_TRY(w->d_pos_tok.ensure(P * 4));
    SWPS_TRY(w->d_rec.ensure(P * RS * 4));
    SWPS_TRY(w->d_pkeys.ensure(M * 4));
    SWPS_TRY(w->d_pvals.ensure(M * 4));
    SWPS_TRY(w->d_pkeys_s.ensure(M * 4));
    SWPS_TRY(w->d_pvals_s.ensure(M * 4));
    if (tracing) SWPS_TRY(w->d_trace.ensure(std::max<uint64_t>(1, P * N) * 4));
    const bool use_uidx = !w->cfg.minibatch_vocab && w->cfg.sampler != SWPS_SAMPLER_ALIAS && w->uni_index &&
                          w->d_uidx.p != nullptr;
    RecArgs ra{w->d_tok.as<int32_t>(), w->d_tok_line.as<int32_t>(), w->d_line_off.as<int64_t>(),
               w->d_pos_tok.as<int32_t>(), (uint32_t)P, w->d_kscan.as<int32_t>(), w->d_ldoff.as<uint64_t>(),
               w->lstate_epoch, W, N, ~0ULL / (uint64_t)W, w->d_unigram.as<int32_t>(), w->cfg.unigram_size,
               ~0ULL / w->cfg.unigram_size,
               w->cfg.minibatch_vocab ? w->d_bstarts.as<uint64_t>() + B.sofs : nullptr,
               w->cfg.minibatch_vocab ? w->d_UK.as<int32_t>() + B.kofs : nullptr, U,
               use_uidx ? w->d_starts.as<uint64_t>() : nullptr, use_uidx ? w->d_uidx.as<int32_t>() : nullptr,
               kUShift, (uint32_t)w->vocab_keys.size(),
               w->cfg.sampler == SWPS_SAMPLER_ALIAS
                   ? w->d_alias.as<uint2>() + (w->cfg.minibatch_vocab ? B.kofs : 0)
                   : nullptr,
               w->cfg.minibatch_vocab ? U : (uint32_t)w->vocab_keys.size(),
               w->d_local.as<int32_t>(), U, w->sharded ? nullptr : w->d_vid_row.as<uint32_t>(), w->d_rec.as<int32_t>(),
               w->d_pkeys.as<uint32_t>(), sort_iota() ? nullptr : w->d_pvals.as<uint32_t>(),
               tracing ? w->d_trace.as<int32_t>() : nullptr,
               tm.on ? w->d_rows_touched.as<unsigned long long>() : nullptr, nullptr, t0};
    if (W == 5 && N == 5 && use_uidx && !w->rec_generic && w->tok_local) {  // k_records_t reads per-token lookups
      SWPS_TRY(w->d_tloc.ensure(std::max<uint64_t>(nt, 1) * 8));
      k_tok_local<<<nblk(nt), 256, 0, s>>>(w->d_tok.as<int32_t>() + t0, nt, w->d_local.as<int32_t>(),
                                           w->sharded ? nullptr : w->d_vid_row.as<uint32_t>(), w->d_tloc.as<int2>());
      SWPS_HIP(hipGetLastError());
      ra.tloc = w->d_tloc.as<int2>();
    }
    hipEvent_t er = tm.begin(s);
    if (W == 5 && N == 5 && use_uidx && !w->rec_generic)
      k_records_t<5, 5><<<nblk(P), 256, 256 * RS * sizeof(int32_t), s>>>(ra);
    else
      k_records<<<nblk(P), 256, 256 * RS * sizeof(int32_t), s>>>(ra);
    SWPS_HIP(hipGetLastError());
    tm.end(KT_REC, er, s);
    pb.records = true;
    pb.HOFF = HOFF;
    pb.M = M;
    if (tracing) {
      std::vector<int32_t> tr(P * N);
      if (!tr.empty()) {
        SWPS_HIP(hipMemcpyAsync(tr.data(), w->d_trace.p, tr.size() * 4, hipMemcpyDeviceToHost, s));
        SWPS_HIP(hipStreamSynchronize(s));
      }
      for (auto v : tr)
        if (w->trace.size() < w->trace_cap) w->trace.push_back(v);
    }
    if (U > 0) {
      // ---- inverted index: stable radix sort of records by local key ----
      int bits = 1;
      while ((1ULL << bits) <= U) bits++;
      hipEvent_t es = tm.begin(s);
      size_t sb = 0;
      if (sort_iota()) {  // the values are the record indices 0..M-1 (the records kernel wrote none)
        SWPS_HIP(sort_pairs_iota(nullptr, sb, w->d_pkeys.as<uint32_t>(), w->d_pkeys_s.as<uint32_t>(),
                                 w->d_pvals_s.as<uint32_t>(), M, bits, s));
        SWPS_TRY(w->d_tmp.ensure(sb));
        sb = w->d_tmp.bytes;
        SWPS_HIP(sort_pairs_iota(w->d_tmp.p, sb, w->d_pkeys.as<uint32_t>(), w->d_pkeys_s.as<uint32_t>(),
                                 w->d_pvals_s.as<uint32_t>(), M, bits, s));
      } else {
        SWPS_HIP(sort_pairs(nullptr, sb, w->d_pkeys.as<uint32_t>(), w->d_pkeys_s.as<uint32_t>(),
                            w->d_pvals.as<uint32_t>(), w->d_pvals_s.as<uint32_t>(), M, bits, s));
        SWPS_TRY(w->d_tmp.ensure(sb));
        sb = w->d_tmp.bytes;
        SWPS_HIP(sort_pairs(w->d_tmp.p, sb, w->d_pkeys.as<uint32_t>(), w->d_pkeys_s.as<uint32_t>(),
                            w->d_pvals.as<uint32_t>(), w->d_pvals_s.as<uint32_t>(), M, bits, s));
      }
      SWPS_TRY(w->d_icnt.ensure((2ULL * U + 1) * 4));
      SWPS_TRY(w->d_ioff.ensure((2ULL * U + 1) * 4));
      if (w->seg4)
        k_seg_bounds4<<<nblk((M + 3) / 4), 256, 0, s>>>(w->d_pkeys_s.as<uint32_t>(), w->d_pvals_s.as<uint32_t>(),
                                                        (uint32_t)M, (uint32_t)HOFF, U, w->d_seg.as<uint32_t>());
      else
        k_seg_bounds<<<nblk(M), 256, 0, s>>>(w->d_pkeys_s.as<uint32_t>(), w->d_pvals_s.as<uint32_t>(), (uint32_t)M,
                                              (uint32_t)HOFF, U, w->d_seg.as<uint32_t>());
      const uint32_t chm = multi_chunk(w, P);
      k_seg_counts<<<nblk((uint64_t)U + 1), 256, 0, s>>>(w->d_seg.as<uint32_t>(), U, kChunk, chm, w->d_icnt.as<uint32_t>(),
                                                          tm.on ? w->d_gstats.as<unsigned long long>() : nullptr);
      SWPS_HIP(hipGetLastError());
      size_t ib = 0;
      SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, ib, w->d_icnt.as<uint32_t>(), w->d_ioff.as<uint32_t>(),
                                                (int)(2 * U + 1), s));
      SWPS_TRY(w->d_tmp.ensure(ib));
      ib = w->d_tmp.bytes;
      SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(w->d_tmp.p, ib, w->d_icnt.as<uint32_t>(), w->d_ioff.as<uint32_t>(),
                                                (int)(2 * U + 1), s));
      const uint64_t max_items = 2ULL * U + M / chm + 1;
      SWPS_TRY(w->d_desc.ensure(max_items * 16));
      // multi-chunk items in the order of their first record's position when
      // the batch's neu1 / neu1e rows outgrow the Infinity Cache: concurrently
      // running gather waves then read nearby positions, so a row's ~6
      // re-reads (by the records of its other keys) hit the cache
      MultiOrder mo{};
      const bool msort = w->multi_sort && P >= w->multi_sort_min;
      if (msort) {
        SWPS_TRY(w->d_pkeys.ensure(max_items * 4));
        SWPS_TRY(w->d_pvals.ensure(max_items * 4));
        SWPS_TRY(w->d_icnt.ensure(max_items * 4));
        int shift = 0;
        while ((P >> shift) >= kMultiPad) shift++;
        mo = MultiOrder{w->d_pkeys.as<uint32_t>(), w->d_pvals.as<uint32_t>(), w->d_pvals_s.as<uint32_t>(),
                        (uint32_t)(N + 1), (uint32_t)(2 * W), HOFF, shift};
      }
      const uint32_t *run_of = nullptr;
      if (w->item_heads) {  // every item's run by a max-scan of the runs' first items (no binary search)
        SWPS_TRY(w->d_irun.ensure(max_items * 4));
        SWPS_HIP(hipMemsetAsync(w->d_irun.p, 0, max_items * 4, s));
        k_item_heads<<<nblk(2ULL * U), 256, 0, s>>>(w->d_ioff.as<uint32_t>(), 2 * U, w->d_irun.as<uint32_t>());
        size_t hb = 0;
        SWPS_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, hb, w->d_irun.as<uint32_t>(), w->d_irun.as<uint32_t>(),
                                                   hipcub::Max(), (int)max_items, s));
        SWPS_TRY(w->d_tmp.ensure(hb));
        hb = w->d_tmp.bytes;
        SWPS_HIP(hipcub::DeviceScan::InclusiveScan(w->d_tmp.p, hb, w->d_irun.as<uint32_t>(), w->d_irun.as<uint32_t>(),
                                                   hipcub::Max(), (int)max_items, s));
        run_of = w->d_irun.as<uint32_t>();
      }
      k_item_desc<<<nblk(max_items), 256, 0, s>>>(w->d_seg.as<uint32_t>(), w->d_ioff.as<uint32_t>(), U, kChunk, chm,
                                                   max_items, w->d_desc.as<uint4>(), w->d_lead.as<uint32_t>(),
                                                   w->d_multi.as<uint32_t>(), mo, run_of);
      SWPS_HIP(hipGetLastError());
      pb.msorted = msort;
      if (msort) {  // stable: equal coarse positions keep item order
        size_t mb = 0;
        SWPS_HIP(sort_pairs(nullptr, mb, w->d_pkeys.as<uint32_t>(), w->d_icnt.as<uint32_t>(),
                            w->d_pvals.as<uint32_t>(), w->d_multi.as<uint32_t>() + 1, max_items, 16, s));
        SWPS_TRY(w->d_tmp.ensure(mb));
        mb = w->d_tmp.bytes;
        SWPS_HIP(sort_pairs(w->d_tmp.p, mb, w->d_pkeys.as<uint32_t>(), w->d_icnt.as<uint32_t>(),
                            w->d_pvals.as<uint32_t>(), w->d_multi.as<uint32_t>() + 1, max_items, 16, s));
      }
      SWPS_HIP(hipGetLastError());
      tm.end(KT_SORT, es, s);
      pb.sorted = true;
      pb.max_items = max_items;
    }
  }
  if (U > 0 && !pb.sorted) {  // no records: the push sees empty segments
    SWPS_TRY(w->d_seg.ensure((uint64_t)U * 16));
    SWPS_HIP(hipMemsetAsync(w->d_seg.p, 0, (uint64_t)U * 16, s));
    SWPS_TRY(w->d_ioff.ensure((2ULL * U + 1) * 4));
    SWPS_HIP(hipMemsetAsync(w->d_ioff.p, 0, (2ULL * U + 1) * 4, s));
  }
  pb.valid = true;
  return SWPS_OK;
}

template <typename T, typename A> int learn_batch(swps_w2v *w, const void *d_vals = nullptr, A *d_grads = nullptr) {
  SWPS_TRY(prep_batch(w));
  const auto pb = w->pb;
  const swps_w2v::Batch &B = w->batches[pb.bi];
  hipStream_t s = w->s;
  Timer &tm = w->timer;
  const int D = w->D, W = w->W, N = w->N;
  const uint32_t U = pb.U;
  const uint64_t P = pb.P;
  const int32_t *K = w->d_K.as<int32_t>() + B.kofs;
  // ---- pull (global_pull_access.h:28-107 + server.h:129-154) ----
  // Single GPU: no copy — the forward reads the batch's keys straight from
  // the table rows (k_records tagged them kTabRow) and the push leaves their
  // pre-update values in the worker cache, which is exactly the state the
  // reference's pull leaves behind.  Sharded: install the owners' values.
  if (U && d_vals) {
    hipEvent_t e = tm.begin(s);
    if (w->parts.n[0] + w->parts.n[1] == U) {  // a split pull: the early and the late values
      for (int q = 0; q < 2; q++)
        if (w->parts.n[q])
          k_install_idx<T><<<nblk((uint64_t)w->parts.n[q] * 64), 256, 0, s>>>(
              K, w->parts.pos[q], (uint32_t)w->parts.n[q], (const T *)w->parts.vals[q], D, w->d_cache_h.as<T>(),
              w->d_cache_v.as<T>(), w->cs);
    } else if (w->pull_rows) {  // world 1: straight from the shard rows the serve looked up
      k_install<T><<<nblk((uint64_t)U * 64), 256, 0, s>>>(K, U, w->t->rows.as<T>(), D, w->d_cache_h.as<T>(),
                                                          w->d_cache_v.as<T>(), w->d_local.as<int32_t>(), 0, w->cs,
                                                          w->pull_rows);
    } else {
      k_install<T><<<nblk((uint64_t)U * 64), 256, 0, s>>>(K, U, (const T *)d_vals, D, w->d_cache_h.as<T>(),
                                                          w->d_cache_v.as<T>(), w->d_local.as<int32_t>(), 0, w->cs);
    }
    w->pull_rows = nullptr;
    w->parts = swps_w2v::Parts{};
    SWPS_HIP(hipGetLastError());
    tm.end(KT_PULL, e, s);
  }
  w->st_batches++;
  w->st_kept += P;
  w->st_words += pb.nt;
  w->st_pulled += U;
  if (pb.records) {
    // ---- forward (learn_instance) ----
    const int ld = w->bfp ? bfp_ld(D, w->bfp_rb) : row_ld(D, sizeof(A), w->row_pad);
    SWPS_TRY(w->d_neu1.ensure(P * ld * sizeof(A)));
    SWPS_TRY(w->d_neu1e.ensure(P * ld * sizeof(A)));
    SWPS_TRY(w->d_pg.ensure(pb.HOFF * 4));
    FwdArgs<T, A> fa{w->d_rec.as<int32_t>(), (int)P, w->d_cache_h.as<T>(), w->d_cache_v.as<T>(), w->t->rows.as<T>(),
                     w->d_exptab.as<float>(), D, W, N, w->cfg.alpha, w->d_neu1.as<A>(), w->d_neu1e.as<A>(),
                     w->d_pg.as<float>(), w->xcd_order, ld, w->cs, w->full_lines};
    hipEvent_t ef = tm.begin(s);
    if constexpr (std::is_same<T, float>::value && std::is_same<A, float>::value) {
      if (w->bfp) {
        if (w->fwd_g == 8 && w->bfp_rb == 0 && bfp_shape(D) == 11) {  // A/B: 8 rows in flight (SWPS_FWD_G=8)
          k_forward_b<1, 1, 0, 8><<<nblk(P * 64), 256, 0, s>>>(fa);
          goto forward_done;
        }
#define SWPS_F(a_, b_, r_) k_forward_b<a_, b_, r_, 4><<<nblk(P * 64), 256, 0, s>>>(fa)
        SWPS_BFP_DISPATCH(w, SWPS_F);
#undef SWPS_F
        goto forward_done;
      }
      if (w->tail) {
        if (D < 512) {
          if (w->fwd_g == 8)
            k_forward_t<1, 8, 1><<<nblk(P * 64), 256, 0, s>>>(fa);
          else if (w->fwd_g == 16)
            k_forward_t<1, 16, 1><<<nblk(P * 64), 256, 0, s>>>(fa);
          else
            k_forward_t<1, 4, 1><<<nblk(P * 64), 256, 0, s>>>(fa);  // G = 4: occupancy 7 (A/B: G = 2..8)
        } else if (D < 768)
          k_forward_t<2, 8, 1><<<nblk(P * 64), 256, 0, s>>>(fa);
        else
          k_forward_t<3, 8, 1><<<nblk(P * 64), 256, 0, s>>>(fa);
        goto forward_done;
      }
    }
    switch (w->NCH) {
      case 1: launch_forward<1>(fa, s); break;
      case 2: launch_forward<2>(fa, s); break;
      case 3: launch_forward<3>(fa, s); break;
      default: launch_forward<4>(fa, s); break;
    }
  forward_done:
    SWPS_HIP(hipGetLastError());
    tm.end(KT_FWD, ef, s);
  }
  if (w->fwd_event) SWPS_HIP(hipEventRecord(w->fwd_event, s));
  // fast mode, single GPU: the push sums the single-chunk runs itself (k_push_tg)
  const bool fast_tail = std::is_same<T, float>::value && std::is_same<A, float>::value && w->tail &&
                         w->fused_push && D < 512 && pb.sorted && !w->bfp;
  const bool sp = std::is_same<T, float>::value && std::is_same<A, float>::value && w->bfp;  // BFP rows
  const bool fused_ip = (fast_tail && !d_grads && w->push_t) || (sp && !d_grads);  // in-place AdaGrad (single GPU)
  const bool fused_g = (fast_tail && d_grads && w->push_tg_var == 5) || (sp && d_grads);  // the sharded learner's mean gradients
  const bool fused = fused_ip || fused_g;
  // small batches: the multi-chunk gather (latency-bound, a few hundred items) runs on a side stream
  // beside the push of every other (key, half); the multi-chunk halves are pushed after it
  const bool split = !sp && fused && w->push_tg_var == 5 && (w->split_push > 0 || (w->split_push < 0 && U < 65536));
  hipStream_t gs = s;  // the gather's stream
  if (split) {
    if (!w->s_side) {
      int lo = 0, hi = 0;
      SWPS_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      SWPS_HIP(hipStreamCreateWithPriority(&w->s_side, hipStreamNonBlocking, hi));
      SWPS_HIP(hipEventCreateWithFlags(&w->ev_fwd, hipEventDisableTiming));
      SWPS_HIP(hipEventCreateWithFlags(&w->ev_gat, hipEventDisableTiming));
    }
    SWPS_HIP(hipEventRecord(w->ev_fwd, s));
    SWPS_HIP(hipStreamWaitEvent(w->s_side, w->ev_fwd, 0));
    gs = w->s_side;
  }
  if (pb.sorted) {
    // ---- chunked segmented gradient sums ----
    SWPS_TRY(w->d_partial.ensure(pb.max_items * D * (sp ? 8 : sizeof(A))));
    GatherArgs<A> ga{w->d_desc.as<uint4>(), w->d_ioff.as<uint32_t>(), w->d_pvals_s.as<uint32_t>(), U,
                     w->d_neu1.as<A>(), w->d_neu1e.as<A>(), w->d_pg.as<float>(), pb.HOFF, (uint32_t)P, D,
                     w->d_partial.as<A>(), sp ? bfp_ld(D, w->bfp_rb) : row_ld(D, sizeof(A), w->row_pad), w->d_lead.as<uint32_t>(),
                     (uint32_t)pb.max_items, fused ? w->d_multi.as<uint32_t>() : nullptr, (uint32_t)(N + 1),
                     (uint32_t)(2 * W), !fused && pb.msorted ? w->d_multi.as<uint32_t>() : nullptr};
    // multi-chunk items: at most M / chm full chunks plus one partial chunk per run of > kChunk records
    const uint64_t gitems =
        fused ? std::min<uint64_t>(pb.max_items, pb.M / multi_chunk(w, P) + pb.M / kChunk + 1) : pb.max_items;
    const unsigned ggrid = (unsigned)std::min<uint64_t>(nblk(gitems * 64), (uint64_t)w->gather_grid);
    const unsigned cgrid = use_combine(w, pb.M) ? combine_grid(pb.max_items) : 0;  // 0: no second level
    hipEvent_t eg = tm.begin(gs);
    if constexpr (std::is_same<T, float>::value && std::is_same<A, float>::value) {
      if (sp) {  // profiled: the kernels' own start / end stamps
        double *part = w->d_partial.as<double>();
        hipEvent_t gb = tm.ext(), ge = tm.ext();
#define SWPS_F(a_, b_, r_)                                                                                         \
  hipExtLaunchKernelGGL(k_gather_b<a_, b_, r_, 8>, dim3(ggrid), dim3(256), 0, gs, gb, cgrid ? (hipEvent_t) nullptr : ge, \
                        0, ga, part)
        SWPS_BFP_DISPATCH(w, SWPS_F);
#undef SWPS_F
        if (cgrid)
          hipExtLaunchKernelGGL(k_combine_b, dim3(cgrid), dim3(256), 0, gs, (hipEvent_t) nullptr, ge, 0, ga, part);
        if (gb) {
          tm.ext_end(KT_GATHER, gb, ge);
          tm.drop(eg);
          eg = nullptr;
        }
        goto gather_done;
      }
      if (w->tail) {
        if (D < 512) {
          if (w->gather_unr == 4)
            k_gather_t<1, 4><<<ggrid, 256, 0, gs>>>(ga);
          else if (w->gather_unr == 16)
            k_gather_t<1, 16><<<ggrid, 256, 0, gs>>>(ga);
          else
            k_gather_t<1, 8><<<ggrid, 256, 0, gs>>>(ga);
        }
        else if (D < 768)
          k_gather_t<2, 8><<<ggrid, 256, 0, gs>>>(ga);
        else
          k_gather_t<3, 8><<<ggrid, 256, 0, gs>>>(ga);
        if (cgrid) switch (w->NCH) {  // second level over the partials: layout-independent
          case 2: k_combine<T, A, 2><<<cgrid, 256, 0, gs>>>(ga); break;
          case 3: k_combine<T, A, 3><<<cgrid, 256, 0, gs>>>(ga); break;
          default: k_combine<T, A, 4><<<cgrid, 256, 0, gs>>>(ga); break;
        }
        goto gather_done;
      }
    }
    switch (w->NCH) {
      case 1: launch_gather<1, T, A>(ga, ggrid, cgrid, s); break;
      case 2: launch_gather<2, T, A>(ga, ggrid, cgrid, s); break;
      case 3: launch_gather<3, T, A>(ga, ggrid, cgrid, s); break;
      default: launch_gather<4, T, A>(ga, ggrid, cgrid, s); break;
    }
  gather_done:
    SWPS_HIP(hipGetLastError());
    tm.end(KT_GATHER, eg, gs);
    if (split) SWPS_HIP(hipEventRecord(w->ev_gat, gs));
    w->st_pairs += pb.M;
    w->st_sums++;
    w->st_fused += fused_ip;
    w->st_fused_g += fused_g;
  }
  if (U > 0) {
    // ---- push: mean + AdaGrad (also clears the local index map) ----
    PushArgs<T, A> pa{K, U, w->d_vid_row.as<uint32_t>(), w->d_seg.as<uint32_t>(), w->d_ioff.as<uint32_t>(),
                      w->d_partial.as<A>(), w->t->rows.as<T>(), w->d_local.as<int32_t>(), D,
                      (double)w->t->cfg.learning_rate, (double)w->t->cfg.fudge, d_grads,
                      d_vals ? nullptr : w->d_cache_h.as<T>(), d_vals ? nullptr : w->d_cache_v.as<T>(), w->cs,
                      w->d_pvals_s.as<uint32_t>(), w->d_pg.as<float>(), w->d_neu1.as<A>(), w->d_neu1e.as<A>(),
                      pb.HOFF, (uint32_t)P, sp ? bfp_ld(D, w->bfp_rb) : row_ld(D, sizeof(A), w->row_pad), w->d_krow.as<uint32_t>(),
                      (uint32_t)(N + 1), (uint32_t)(2 * W), w->full_lines,
                      use_combine(w, pb.M) ? kGroup : 0xFFFFFFFFu};
    hipEvent_t ep = tm.begin(s);
    if constexpr (std::is_same<T, float>::value && std::is_same<A, float>::value) {
      const unsigned pgrid = (unsigned)std::min<uint64_t>(nblk((uint64_t)U * 128),
                                                          w->push_grid ? w->push_grid : (U < 65536 ? 2048 : ~0u));
      if (sp) {
        const double *part = w->d_partial.as<double>();
        double *g64 = (double *)d_grads;  // BFP mode: the fp64 push payload
        if (!d_grads) {
          // D = 257..320, bfp32: 134 -> 128 VGPRs (2 spilled) for 4 waves per SIMD; small batches only
          // (same-box A/B: B = 100 2.87e8 -> 3.06e8 words/s, B = 5000 -0.1 %); SWPS_PUSH_WPE=1 / 4 forces
          const bool wpe4 = w->push_wpe == 4 || (w->push_wpe == 0 && U < 65536);
          hipEvent_t pb = tm.ext(), pe = tm.ext();  // profiled: the kernel's own start / end stamps
          if (wpe4 && w->push_unr == 4 && U < 65536 && w->bfp_rb == 0 && bfp_shape(D) == 11) {
            // D = 257..320, bfp32, small batches: 4 record rows in flight, 114 VGPRs, 4 waves per SIMD
            // without spills (same-box A/B, round 4: B = 100 3.01e8 -> 3.09e8 words/s; 5 / 6 / 8 rows:
            // 3.07 / 3.03 / 3.01e8; 5 waves per SIMD (13 spills) 2.85e8).  Not above 64k keys: B = 5000
            // +0.1 %, the config-4 shape's push 4.78 -> 5.00 ms.  SWPS_PUSH_WPE=1 turns it off too
            hipExtLaunchKernelGGL(k_push_b<1, 1, 0, 4, false, 4>, dim3(pgrid), dim3(256), 0, s, pb, pe, 0, pa, part,
                                  (double *)nullptr);
          } else if (wpe4 && w->bfp_rb == 0 && bfp_shape(D) == 11) {
            hipExtLaunchKernelGGL(k_push_b<1, 1, 0, 8, false, 4>, dim3(pgrid), dim3(256), 0, s, pb, pe, 0, pa, part,
                                  (double *)nullptr);
          } else {
#define SWPS_F(a_, b_, r_)                                                                                    \
  hipExtLaunchKernelGGL(k_push_b<a_, b_, r_, 8, false>, dim3(pgrid), dim3(256), 0, s, pb, pe, 0, pa, part, \
                        (double *)nullptr)
            SWPS_BFP_DISPATCH(w, SWPS_F);
#undef SWPS_F
          }
          if (pb) {
            tm.ext_end(KT_PUSH, pb, pe);
            tm.drop(ep);
            ep = nullptr;
          }
          goto push_done;
        }
        // (4 record rows in flight here: 94 VGPRs, 5 waves per SIMD, but the sharded world-1 push
        // 2.487 -> 2.506 ms, same-box A/B, round 4: kept at 8)
#define SWPS_F(a_, b_, r_) k_push_b<a_, b_, r_, 8, true><<<pgrid, 256, 0, s>>>(pa, part, g64)
        const int world = w->world;
        if (w->split_grads && world > 1 && world <= kMaxSplitOwners) {  // two owner-half passes (below)
          if (!w->ev_half) SWPS_HIP(hipEventCreateWithFlags(&w->ev_half, hipEventDisableTiming));
          pa.nown = (uint32_t)world;
          uint32_t acc = 0;
          for (int r = 0; r < world; r++) {
            const uint64_t c = w->bcounts[pb.bi * world + r];
            pa.obnd[r] = acc;
            pa.ohalf[r] = (uint32_t)(c / 2);
            acc += (uint32_t)c;
          }
          pa.obnd[world] = acc;
          pa.gpass = 1;
          SWPS_BFP_DISPATCH(w, SWPS_F);
          SWPS_HIP(hipEventRecord(w->ev_half, s));
          pa.gpass = 2;
          SWPS_BFP_DISPATCH(w, SWPS_F);
          w->half_ready = true;
        } else {
          SWPS_BFP_DISPATCH(w, SWPS_F);
        }
#undef SWPS_F
        goto push_done;
      }
      if (split) {  // every other (key, half) beside the gather, then the multi-chunk halves
        if (fused_g)
          k_push_thp<1, 8, true, 1><<<pgrid, 256, 0, s>>>(pa);
        else
          k_push_thp<1, 8, false, 1><<<pgrid, 256, 0, s>>>(pa);
        SWPS_HIP(hipStreamWaitEvent(s, w->ev_gat, 0));
        if (fused_g)
          k_push_thp<1, 8, true, 2><<<pgrid, 256, 0, s>>>(pa);
        else
          k_push_thp<1, 8, false, 2><<<pgrid, 256, 0, s>>>(pa);
        w->st_split++;
        goto push_done;
      }
      if (fused_g) {
        const int world = w->world;
        if (w->split_grads && world > 1 && world <= kMaxSplitOwners) {
          // two passes, each owner's first half of keys first: the driver sends those gradients
          // (ev_half) while the second pass runs
          if (!w->ev_half) SWPS_HIP(hipEventCreateWithFlags(&w->ev_half, hipEventDisableTiming));
          pa.nown = (uint32_t)world;
          uint32_t acc = 0;
          for (int r = 0; r < world; r++) {
            const uint64_t c = w->bcounts[pb.bi * world + r];
            pa.obnd[r] = acc;
            pa.ohalf[r] = (uint32_t)(c / 2);
            acc += (uint32_t)c;
          }
          pa.obnd[world] = acc;
          pa.gpass = 1;
          k_push_thp<1, 8, true><<<pgrid, 256, 0, s>>>(pa);
          SWPS_HIP(hipEventRecord(w->ev_half, s));
          pa.gpass = 2;
          k_push_thp<1, 8, true><<<pgrid, 256, 0, s>>>(pa);
          w->half_ready = true;
        } else {
          k_push_thp<1, 8, true><<<pgrid, 256, 0, s>>>(pa);
        }
        goto push_done;
      }
      if (fused) {
        if (w->push_tg_var == 5)
          // small batches are latency-bound: several items per wave, and the idle CUs run the prep stream
          // (A/B at B = 100 lines: 2048 blocks 0.317 ms/step, 4096 0.323, one item per wave 0.331); large ones want every item in flight
          k_push_thp<1, 8><<<(unsigned)std::min<uint64_t>(nblk((uint64_t)U * 128),
                                                          w->push_grid ? w->push_grid : (U < 65536 ? 2048 : ~0u)),
                             256, 0, s>>>(pa);
        else if (w->push_tg_var == 3)
          k_push_th<1, 8><<<nblk((uint64_t)U * 128), 256, 0, s>>>(pa);
        else if (w->push_tg_var == 4)
          k_push_th<1, 16><<<nblk((uint64_t)U * 128), 256, 0, s>>>(pa);
        else if (w->push_tg_var == 1)
          k_push_tg<1, 8, 4><<<nblk((uint64_t)U * 64), 256, 0, s>>>(pa);  // occupancy 4, 5 VGPRs spilled
        else if (w->push_tg_var == 2)
          k_push_tg<1, 4, 1><<<nblk((uint64_t)U * 64), 256, 0, s>>>(pa);
        else
          k_push_tg<1, 8, 1><<<nblk((uint64_t)U * 64), 256, 0, s>>>(pa);  // 135 VGPRs, occupancy 3
        goto push_done;
      }
      if (w->tail && !d_grads && w->push_t) {
        if (D < 512)
          k_push_t<1><<<nblk((uint64_t)U * 64), 256, 0, s>>>(pa);
        else if (D < 768)
          k_push_t<2><<<nblk((uint64_t)U * 64), 256, 0, s>>>(pa);
        else
          k_push_t<3><<<nblk((uint64_t)U * 64), 256, 0, s>>>(pa);
        goto push_done;
      }
    }
    switch (w->NCH) {
      case 1: launch_push<1>(pa, s); break;
      case 2: launch_push<2>(pa, s); break;
      case 3: launch_push<3>(pa, s); break;
      default: launch_push<4>(pa, s); break;
    }
  push_done:
    SWPS_HIP(hipGetLastError());
    tm.end(KT_PUSH, ep, s);
    w->st_pushed += U;
  }
  w->pb.valid = false;
  w->cursor++;
  return SWPS_OK;
}

template <typename T, typename A> int run_batch(swps_w2v *w, const void *d_vals = nullptr, A *d_grads = nullptr) {
  return learn_batch<T, A>(w, d_vals, d_grads);
}

}  // namespace

void swap_prep_set(swps_w2v *w) {
  for (int k = 0; k < swps_w2v::kPrepBufs; k++) {
    std::swap(w->prep_set[k]->p, w->alt[k].p);
    std::swap(w->prep_set[k]->bytes, w->alt[k].bytes);
  }
}

// Single-GPU minibatch loop with prep(i+1) (epoch plan, local key map,
// records, radix sort, chunk index — parameter-independent, SURVEY.md §3.2's
// draws) on s_prep into the second buffer set while learn(i) (pull, forward,
// gather, push) runs on s.  prep(i+1) waits for learn(i-1), the last user of
// that set (its push also clears that set's local-key map); learn(i+1) waits
// for prep(i+1).  Every kernel sees the same inputs as in the sequential
// loop, so results are bit-identical (tests: SWPS_OVERLAP=0 vs 1).  Nothing
// is left prepared when the call returns.
template <typename T, typename A> int train_overlapped(swps_w2v *w, uint64_t count) {
  if (!w->s_prep) {
    int lo = 0, hi = 0;
    SWPS_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // the prep chain is short latency-bound launches: at the highest priority they take CUs as
    // soon as they are issued instead of queueing behind the learn kernels (same-box A/B at
    // B = 100 lines: highest 0.317 ms/step, lowest 0.321); SWPS_PREP_PRIO=0 default, 1 lowest
    const char *pe = getenv("SWPS_PREP_PRIO");
    if (pe && atoi(pe) == 0)
      SWPS_HIP(hipStreamCreateWithFlags(&w->s_prep, hipStreamNonBlocking));
    else if (pe && atoi(pe) == 1)
      SWPS_HIP(hipStreamCreateWithPriority(&w->s_prep, hipStreamNonBlocking, lo));
    else
      SWPS_HIP(hipStreamCreateWithPriority(&w->s_prep, hipStreamNonBlocking, hi));
    SWPS_HIP(hipEventCreateWithFlags(&w->ev_learn, hipEventDisableTiming));
    SWPS_HIP(hipEventCreateWithFlags(&w->ev_prep, hipEventDisableTiming));
  }
  const uint64_t V = w->vocab_keys.size();
  if (!w->alt_local_ready) {
    DevMem &al = w->alt[swps_w2v::kPrepBufs - 1];
    SWPS_TRY(al.ensure(V * 4));
    SWPS_HIP(hipMemsetAsync(al.p, 0xFF, V * 4, w->s));
    w->alt_local_ready = true;
  }
  const hipStream_t s = w->s;
  bool prep_pending = false;  // batch i's prep ran on s_prep (ev_prep)
  if (w->overlap == 2) {
    // prep(i+1) issued after learn(i), waiting for forward(i): it runs beside the gather and the
    // push (latency-bound) instead of beside the forward (bandwidth-bound).  It writes the other
    // buffer set, whose last user learn(i-1) finished before forward(i) did.
    for (uint64_t i = 0; i < count; i++) {
      if (!w->pb.valid) SWPS_TRY(prep_batch(w));  // inline on s (first batch of the call)
      if (prep_pending) SWPS_HIP(hipStreamWaitEvent(s, w->ev_prep, 0));
      w->fwd_event = i + 1 < count ? w->ev_learn : nullptr;
      const int lrc = learn_batch<T, A>(w);  // cursor -> i + 1
      w->fwd_event = nullptr;
      SWPS_TRY(lrc);
      prep_pending = false;
      if (i + 1 < count) {
        SWPS_HIP(hipStreamWaitEvent(w->s_prep, w->ev_learn, 0));
        swap_prep_set(w);  // the other set becomes the current one: prep(i+1) fills it, learn(i+1) reads it
        w->s = w->s_prep;
        w->pb = swps_w2v::Prepped();
        const int rc = prep_batch(w);
        w->s = s;
        SWPS_TRY(rc);
        SWPS_HIP(hipEventRecord(w->ev_prep, w->s_prep));
        prep_pending = true;
      }
    }
    if (prep_pending) SWPS_HIP(hipStreamWaitEvent(s, w->ev_prep, 0));
    return SWPS_OK;
  }
  for (uint64_t i = 0; i < count; i++) {
    if (!w->pb.valid) SWPS_TRY(prep_batch(w));  // inline on s (first batch of the call)
    const swps_w2v::Prepped cur = w->pb;
    swps_w2v::Prepped next;
    if (i + 1 < count) {
      SWPS_HIP(hipEventRecord(w->ev_learn, s));  // learn(i-1) done -> the other set is free
      SWPS_HIP(hipStreamWaitEvent(w->s_prep, w->ev_learn, 0));
      swap_prep_set(w);
      w->s = w->s_prep;
      w->cursor++;
      w->pb = swps_w2v::Prepped();
      const int rc = prep_batch(w);
      next = w->pb;
      w->cursor--;
      w->s = s;
      swap_prep_set(w);
      SWPS_TRY(rc);
    }
    if (prep_pending) SWPS_HIP(hipStreamWaitEvent(s, w->ev_prep, 0));
    if (i + 1 < count) SWPS_HIP(hipEventRecord(w->ev_prep, w->s_prep));
    prep_pending = i + 1 < count;
    w->pb = cur;
    SWPS_TRY((learn_batch<T, A>(w)));
    if (prep_pending) {
      swap_prep_set(w);
      w->pb = next;
    }
  }
  return SWPS_OK;
}

extern "C" {

int swps_w2v_create(swps_table *t, const swps_w2v_cfg *cfg, swps_w2v **out) {
  if (!t || !cfg || !out) return fail(SWPS_E_CFG, "null argument");
  *out = nullptr;
  if (t->cfg.layout != SWPS_LAYOUT_W2V) return fail(SWPS_E_CFG, "table layout must be SWPS_LAYOUT_W2V");
  SWPS_TRY(check_app_table(t));
  SWPS_HIP(hipSetDevice(t->cfg.device));
  swps_w2v *w = new swps_w2v();
  w->t = t;
  w->cfg = *cfg;
  w->D = t->cfg.dim;
  w->W = cfg->window;
  w->N = cfg->negative;
  w->f64 = t->cfg.dtype == SWPS_F64;
  w->s = t->stream;
  w->timer.on = cfg->profile != 0;
  if (const char *e = getenv("SWPS_XCD_ORDER")) w->xcd_order = atoi(e) != 0;
  if (const char *e = getenv("SWPS_PUSH_T")) w->push_t = atoi(e) != 0;  // A/B timing
  if (const char *e = getenv("SWPS_FUSED_PUSH")) w->fused_push = atoi(e) != 0;  // A/B timing
  if (const char *e = getenv("SWPS_PUSH_TG")) w->push_tg_var = atoi(e);          // A/B timing
  if (const char *e = getenv("SWPS_FWD_G")) w->fwd_g = atoi(e);
  if (const char *e = getenv("SWPS_COMBINE")) w->combine = atoi(e);
  if (const char *e = getenv("SWPS_COMBINE_MIN")) w->combine_min = strtoull(e, nullptr, 10);
  if (const char *e = getenv("SWPS_FULL_LINES")) w->full_lines = atoi(e) != 0;
  if (const char *e = getenv("SWPS_SPLIT_PUSH")) w->split_push = atoi(e);
  if (const char *e = getenv("SWPS_SPLIT_GRADS")) w->split_grads = atoi(e) != 0;
  if (const char *e = getenv("SWPS_PUSH_GRID")) w->push_grid = (uint32_t)std::max(0, atoi(e));
  if (const char *e = getenv("SWPS_MULTI_SORT")) w->multi_sort = atoi(e);        // A/B timing
  if (const char *e = getenv("SWPS_MULTI_CHUNK")) w->multi_chunk = (uint32_t)std::min(128, std::max(0, atoi(e)));
  if (const char *e = getenv("SWPS_MULTI_SORT_MIN")) w->multi_sort_min = strtoull(e, nullptr, 10);
  if (const char *e = getenv("SWPS_ROW_PAD")) w->row_pad = atoi(e) != 0;  // A/B timing
  if (const char *e = getenv("SWPS_UNI_INDEX")) w->uni_index = atoi(e) != 0;  // A/B timing
  if (const char *e = getenv("SWPS_SEG4")) w->seg4 = atoi(e) != 0;            // A/B timing
  if (const char *e = getenv("SWPS_TOK_LOCAL")) w->tok_local = atoi(e) != 0;  // A/B timing
  if (const char *e = getenv("SWPS_ITEM_HEADS")) w->item_heads = atoi(e) != 0;  // A/B timing
  if (const char *e = getenv("SWPS_CACHE_PAD")) w->cache_pad = atoi(e) != 0;  // A/B timing
  if (const char *e = getenv("SWPS_OVERLAP")) w->overlap = atoi(e);  // A/B timing
  if (const char *e = getenv("SWPS_GATHER_UNR")) w->gather_unr = atoi(e);
  if (const char *e = getenv("SWPS_REC_GENERIC")) w->rec_generic = atoi(e) != 0;
  if (const char *e = getenv("SWPS_GATHER_GRID")) w->gather_grid = std::max(64, atoi(e));
  if (const char *e = getenv("SWPS_PUSH_WPE")) w->push_wpe = atoi(e);  // A/B: push occupancy
  if (const char *e = getenv("SWPS_PUSH_UNR8")) w->push_unr = atoi(e) ? 8 : 4;  // A/B, tests
  int rc = check_cfg(w);
  if (!rc && hipHostMalloc((void **)&w->h_small, 64) != hipSuccess) rc = fail(SWPS_E_OOM, "pinned alloc");
  if (!rc) rc = w->d_rows_touched.ensure(16);
  if (!rc && hipMemset(w->d_rows_touched.p, 0, 16) != hipSuccess) rc = fail(SWPS_E_HIP, "memset");
  if (!rc) rc = w->d_gstats.ensure(32);
  if (!rc && hipMemset(w->d_gstats.p, 0, 32) != hipSuccess) rc = fail(SWPS_E_HIP, "memset");
  if (!rc) {
    uint64_t A[kMaxJump + 1], C[kMaxJump + 1];
    for (int k = 0; k <= kMaxJump; k++) {
      A[k] = lcg_jump(1, k, kLcgA, kLcgC) - lcg_jump(0, k, kLcgA, kLcgC);
      C[k] = lcg_jump(0, k, kLcgA, kLcgC);
    }
    uint64_t PA[64], PC[64];  // jumps by 2^i draws
    for (int i = 0; i < 64; i++) {
      PA[i] = lcg_jump(1, 1ULL << i, kLcgA, kLcgC) - lcg_jump(0, 1ULL << i, kLcgA, kLcgC);
      PC[i] = lcg_jump(0, 1ULL << i, kLcgA, kLcgC);
    }
    uint64_t FA[64], FC[64];  // the subsampling float LCG's jumps by 2^i draws
    for (int i = 0; i < 64; i++) {
      FA[i] = lcg_jump(1, 1ULL << i, kFlcgA, kLcgC) - lcg_jump(0, 1ULL << i, kFlcgA, kLcgC);
      FC[i] = lcg_jump(0, 1ULL << i, kFlcgA, kLcgC);
    }
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_f2A), FA, sizeof(FA)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_f2C), FC, sizeof(FC)) != hipSuccess)
      rc = fail(SWPS_E_HIP, "constant upload");
    if (!rc && (hipMemcpyToSymbol(HIP_SYMBOL(c_jumpA), A, sizeof(A)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_jumpC), C, sizeof(C)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_p2A), PA, sizeof(PA)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_p2C), PC, sizeof(PC)) != hipSuccess))
      rc = fail(SWPS_E_HIP, "constant upload");
  }
  if (rc) {
    if (w->h_small) (void)hipHostFree(w->h_small);
    delete w;
    return rc;
  }
  *out = w;
  return SWPS_OK;
}

int swps_w2v_destroy(swps_w2v *w) {
  if (!w) return SWPS_OK;
  (void)hipSetDevice(w->t->cfg.device);
  (void)hipStreamSynchronize(w->s);
  if (w->s_prep) {
    (void)hipStreamSynchronize(w->s_prep);
    (void)hipStreamDestroy(w->s_prep);
  }
  if (w->s_side) {
    (void)hipStreamSynchronize(w->s_side);
    (void)hipStreamDestroy(w->s_side);
  }
  if (w->ev_learn) (void)hipEventDestroy(w->ev_learn);
  if (w->ev_prep) (void)hipEventDestroy(w->ev_prep);
  if (w->ev_fwd) (void)hipEventDestroy(w->ev_fwd);
  if (w->ev_half) (void)hipEventDestroy(w->ev_half);
  if (w->ev_gat) (void)hipEventDestroy(w->ev_gat);
  if (w->h_small) (void)hipHostFree(w->h_small);
  delete w->drv;
  delete w;
  (void)hipGetLastError();  // leave no sticky error from the calls above
  return SWPS_OK;
}

// LineFileReader + split(" ") + BKDRHash / atoi (word2vec_global.h:215-227)
int swps_w2v_load_text(swps_w2v *w, const char *path) {
  if (!w->cfg.minibatch_vocab && !w->cfg.host_ingest) {  // the GPU ingest (no NUL bytes in the file)
    FILE *f = fopen(path, "rb");
    if (!f) return fail(SWPS_E_IO, std::string("no such file or directory: ") + path);
    std::vector<char> text;
    char chunk[1 << 16];
    size_t k;
    while ((k = fread(chunk, 1, sizeof(chunk), f)) > 0) text.insert(text.end(), chunk, chunk + k);
    fclose(f);
    if (!memchr(text.data(), 0, text.size())) {
      SWPS_HIP(hipSetDevice(w->t->cfg.device));
      DevMem d_keys;
      uint64_t nt = 0;
      std::vector<int64_t> off;
      SWPS_TRY(tokenize_gpu(w, text, d_keys, nt, off));
      std::vector<char>().swap(text);
      SWPS_TRY(ingest_gpu(w, d_keys, nt, std::move(off)));
      SWPS_TRY(schedule_gpu(w));
      return upload_corpus(w);
    }
  }
  FILE *f = fopen(path, "rb");
  if (!f) return fail(SWPS_E_IO, std::string("no such file or directory: ") + path);
  std::vector<uint64_t> keys;
  std::vector<int64_t> off{0};
  char *buf = nullptr;
  size_t cap = 0;
  ssize_t n;
  std::string word;
  while ((n = getdelim(&buf, &cap, '\n', f)) >= 0) {
    if (n >= 1 && buf[n - 1] == '\n') buf[--n] = 0;
    const size_t len = strlen(buf);  // std::string(cline) stops at a NUL
    size_t i = 0;
    while (i < len) {
      while (i < len && buf[i] == ' ') i++;
      if (i >= len) break;
      size_t j = i;
      while (j < len && buf[j] != ' ') j++;
      word.assign(buf + i, j - i);
      keys.push_back(w->cfg.key_mode == SWPS_KEY_ATOI ? (uint64_t)(int64_t)atoi(word.c_str()) : bkdr(word.c_str()));
      i = j;
    }
    off.push_back((int64_t)keys.size());
  }
  free(buf);
  fclose(f);
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  SWPS_TRY(ingest(w, keys, std::move(off)));
  if (w->cfg.minibatch_vocab)
    SWPS_TRY(build_schedule_mb(w));
  else
    build_schedule(w);
  return upload_corpus(w);
}

int swps_w2v_load_tokens(swps_w2v *w, const uint32_t *word_ids, uint64_t ntok, const uint64_t *line_off,
                         uint64_t nlines, const uint64_t *word_keys, uint64_t nwords) {
  if (line_off[0] != 0 || line_off[nlines] != ntok) return fail(SWPS_E_CFG, "line_off must span [0, ntok]");
  std::vector<int64_t> off(line_off, line_off + nlines + 1);
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  if (!w->cfg.minibatch_vocab && !w->cfg.host_ingest) {  // the GPU ingest
    DevMem d_ids, d_wk, d_keys, d_bad;
    SWPS_TRY(d_ids.ensure(std::max<uint64_t>(ntok, 1) * 4));
    SWPS_TRY(d_wk.ensure(std::max<uint64_t>(nwords, 1) * 8));
    SWPS_TRY(d_keys.ensure(std::max<uint64_t>(ntok, 1) * 8));
    SWPS_TRY(d_bad.ensure(4));
    if (ntok) SWPS_HIP(hipMemcpyAsync(d_ids.p, word_ids, ntok * 4, hipMemcpyHostToDevice, w->s));
    if (nwords) SWPS_HIP(hipMemcpyAsync(d_wk.p, word_keys, nwords * 8, hipMemcpyHostToDevice, w->s));
    SWPS_HIP(hipMemsetAsync(d_bad.p, 0, 4, w->s));
    if (ntok)
      k_gather_keys<<<nblk(ntok), 256, 0, w->s>>>(d_ids.as<uint32_t>(), ntok, d_wk.as<uint64_t>(), nwords,
                                                   d_keys.as<uint64_t>(), d_bad.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    uint32_t bad = 0;
    SWPS_HIP(hipMemcpyAsync(&bad, d_bad.p, 4, hipMemcpyDeviceToHost, w->s));
    SWPS_HIP(hipStreamSynchronize(w->s));
    if (bad) return fail(SWPS_E_CFG, "word id out of range");
    d_ids.release();
    d_wk.release();
    SWPS_TRY(ingest_gpu(w, d_keys, ntok, std::move(off)));
    SWPS_TRY(schedule_gpu(w));
    return upload_corpus(w);
  }
  std::vector<uint64_t> keys(ntok);
  for (uint64_t i = 0; i < ntok; i++) {
    if (word_ids[i] >= nwords) return fail(SWPS_E_CFG, "word id out of range");
    keys[i] = word_keys[word_ids[i]];
  }
  SWPS_TRY(ingest(w, keys, std::move(off)));
  if (w->cfg.minibatch_vocab)
    SWPS_TRY(build_schedule_mb(w));
  else
    build_schedule(w);
  return upload_corpus(w);
}

int swps_w2v_corpus(swps_w2v *w, int32_t *vid, int32_t *line, uint64_t cap) {
  if (!w->loaded) return fail(SWPS_E_STATE, "load a corpus first");
  if (cap < w->ntok) return fail(SWPS_E_CFG, "buffer too small");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  if (w->ntok) {
    SWPS_HIP(hipMemcpyAsync(vid, w->d_tok.p, w->ntok * 4, hipMemcpyDeviceToHost, w->s));
    SWPS_HIP(hipMemcpyAsync(line, w->d_tok_line.p, w->ntok * 4, hipMemcpyDeviceToHost, w->s));
  }
  SWPS_HIP(hipStreamSynchronize(w->s));
  return SWPS_OK;
}

int swps_w2v_batch_keys(swps_w2v *w, uint64_t b, int32_t *out, uint64_t cap, uint64_t *n, uint64_t *lines2) {
  if (!w->loaded) return fail(SWPS_E_STATE, "load a corpus first");
  if (b >= w->batches.size()) return fail(SWPS_E_CFG, "no such batch");
  const auto &bt = w->batches[b];
  *n = bt.U;
  if (lines2) {
    lines2[0] = bt.l0;
    lines2[1] = bt.l1;
  }
  if (cap < bt.U) return fail(SWPS_E_CFG, "buffer too small");
  std::copy(w->allK.begin() + bt.kofs, w->allK.begin() + bt.kofs + bt.U, out);
  return SWPS_OK;
}

int swps_w2v_vocab(swps_w2v *w, uint64_t *keys, int32_t *counts, uint64_t cap, uint64_t *n) {
  *n = w->vocab_keys.size();
  if (cap < *n) return fail(SWPS_E_CFG, "buffer too small");
  for (size_t i = 0; i < w->vocab_keys.size(); i++) {
    if (keys) keys[i] = w->vocab_keys[i];
    if (counts) counts[i] = w->counts[i];
  }
  return SWPS_OK;
}

int swps_w2v_info(swps_w2v *w, uint64_t *o) {
  o[0] = w->vocab_keys.size();
  o[1] = w->train_words;
  o[2] = w->line_off.empty() ? 0 : w->line_off.size() - 1;
  o[3] = w->ntok;
  o[4] = w->batches.size();
  o[5] = w->max_tok;
  o[6] = w->lstate;
  o[7] = w->fstate;
  return SWPS_OK;
}

// The first full pull (word2vec_global.h:557-562 -> accessmethod.h:63-70):
// every vocab key misses and gets a fresh WParam.
int swps_w2v_init(swps_w2v *w) {
  if (!w->loaded) return fail(SWPS_E_STATE, "load a corpus first");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  if (w->drv) return w->drv->full_pull();  // the first full pull, over the communicator
  if (w->t->comm)
    return fail(SWPS_E_UNSUPPORTED, "the table is key-sharded (swps_table_route): drive the context with "
                                    "swps_w2v_shard_comm");
  const uint64_t V = w->vocab_keys.size();
  DevMem dk;
  SWPS_TRY(upload(dk, w->vocab_keys, w->s));
  SWPS_TRY(table_find_or_insert(w->t, dk.as<uint64_t>(), V, w->d_vid_row.as<uint32_t>(), w->s));
  if (w->cfg.init_mode == SWPS_W2V_INIT_REF) {
    // Vec::randInit (vec1.h:229-232): (rand()/(float)RAND_MAX - 0.5)/D, h then
    // v per key, keys in _local_keys order, after rand_offset earlier calls —
    // generated on the GPU by jump-ahead (rand_init_gpu)
    SWPS_TRY(w->f64 ? rand_init_gpu<double>(w) : rand_init_gpu<float>(w));
  } else {
    SWPS_TRY(w->f64 ? pull_all<double>(w) : pull_all<float>(w));
  }
  w->inited = true;
  return SWPS_OK;
}

int swps_w2v_train_batches(swps_w2v *w, uint64_t count) {
  if (!w->inited) return fail(SWPS_E_STATE, "call swps_w2v_init first");
  if (w->drv) {
    SWPS_HIP(hipSetDevice(w->t->cfg.device));
    return w->drv->steps(count);  // collective: `count` lockstep steps on every rank
  }
  if (w->sharded) return fail(SWPS_E_STATE, "sharded context: drive it with request / serve_pull / step / serve_push");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  const bool ov = w->overlap > 0 || (w->overlap < 0 && w->max_tok <= kOverlapTok);
  if (ov && count > 1 && !w->cfg.minibatch_vocab && w->trace.size() >= w->trace_cap && !w->pb.valid) {
    if (w->f64) return train_overlapped<double, double>(w, count);
    if (inter64(w->cfg)) return train_overlapped<float, double>(w, count);
    return train_overlapped<float, float>(w, count);
  }
  for (uint64_t i = 0; i < count; i++) {
    if (w->f64)
      SWPS_TRY((run_batch<double, double>(w)));
    else if (inter64(w->cfg))
      SWPS_TRY((run_batch<float, double>(w)));
    else
      SWPS_TRY((run_batch<float, float>(w)));
  }
  return SWPS_OK;
}

int swps_w2v_train_epochs(swps_w2v *w, int32_t niters) {
  if (w->drv) {
    if (w->drv->spe && w->drv->cursor % w->drv->spe) return fail(SWPS_E_STATE, "not at an epoch boundary");
    SWPS_TRY(swps_w2v_train_batches(w, (uint64_t)niters * w->drv->spe));
    return swps_w2v_sync(w);
  }
  if (w->cursor % std::max<size_t>(1, w->batches.size()) != 0) return fail(SWPS_E_STATE, "not at an epoch boundary");
  SWPS_TRY(swps_w2v_train_batches(w, (uint64_t)niters * w->batches.size()));
  return swps_w2v_sync(w);
}

int swps_w2v_sync(swps_w2v *w) {
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  if (w->drv) SWPS_TRY(w->drv->sync());
  SWPS_HIP(hipStreamSynchronize(w->s));
  if (w->ss) SWPS_HIP(hipStreamSynchronize(w->ss));
  w->timer.resolve();
  return SWPS_OK;
}

int swps_w2v_stats(swps_w2v *w, uint64_t *o) {
  o[0] = w->st_batches;
  o[1] = w->st_kept;
  o[2] = w->st_words;
  o[3] = w->st_pairs;
  o[4] = w->lstate;
  o[5] = w->fstate;
  o[6] = w->st_pulled;
  o[7] = w->st_pushed;
  uint64_t rt[2] = {0, 0};
  SWPS_HIP(hipStreamSynchronize(w->s));
  SWPS_HIP(hipMemcpy(rt, w->d_rows_touched.p, 16, hipMemcpyDeviceToHost));
  o[8] = rt[0];
  o[9] = rt[1];
  return SWPS_OK;
}

int swps_w2v_gather_stats(swps_w2v *w, uint64_t *out2) {
  SWPS_HIP(hipStreamSynchronize(w->s));
  SWPS_HIP(hipMemcpy(out2, w->d_gstats.p, 16, hipMemcpyDeviceToHost));
  return SWPS_OK;
}

int swps_w2v_sum_stats(swps_w2v *w, uint64_t *out8) {
  SWPS_HIP(hipStreamSynchronize(w->s));
  SWPS_HIP(hipMemcpy(out8, w->d_gstats.p, 32, hipMemcpyDeviceToHost));
  out8[4] = w->st_fused;
  out8[5] = w->st_sums;
  out8[6] = w->st_fused_g;
  out8[7] = w->st_split;
  return SWPS_OK;
}

int swps_w2v_get_params(swps_w2v *w, double *out) {
  SWPS_TRY(swps_w2v_sync(w));
  const uint64_t V = w->vocab_keys.size();
  const int R = 4 * w->D;
  DevMem d;
  const size_t es = w->f64 ? 8 : 4;
  SWPS_TRY(d.ensure(V * R * es));
  SWPS_TRY(table_get_rows(w->t, w->d_vid_row.as<uint32_t>(), V, d.p, w->s));
  std::vector<char> h(V * R * es);
  SWPS_HIP(hipMemcpyAsync(h.data(), d.p, h.size(), hipMemcpyDeviceToHost, w->s));
  SWPS_HIP(hipStreamSynchronize(w->s));
  for (uint64_t i = 0; i < V * R; i++) out[i] = w->f64 ? ((double *)h.data())[i] : (double)((float *)h.data())[i];
  return SWPS_OK;
}

int swps_w2v_set_params(swps_w2v *w, const double *hv) {
  if (!w->inited) SWPS_TRY(swps_w2v_init(w));
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  return w->f64 ? set_hv<double>(w, hv) : set_hv<float>(w, hv);
}

int swps_w2v_unigram_at(swps_w2v *w, const uint64_t *idx, uint64_t n, uint32_t *out) {
  if (w->cfg.minibatch_vocab) return fail(SWPS_E_STATE, "minibatch-vocab mode has one table per minibatch");
  if (w->cfg.sampler == SWPS_SAMPLER_ALIAS) return fail(SWPS_E_STATE, "the alias sampler has no slot table");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  SWPS_HIP(hipStreamSynchronize(w->s));
  for (uint64_t i = 0; i < n; i++) {
    if (idx[i] >= w->cfg.unigram_size) return fail(SWPS_E_CFG, "slot out of range");
    SWPS_HIP(hipMemcpy(out + i, w->d_unigram.as<int32_t>() + idx[i], 4, hipMemcpyDeviceToHost));
  }
  return SWPS_OK;
}

int swps_w2v_trace_negatives(swps_w2v *w, uint64_t cap) {
  w->trace_cap = cap;
  w->trace.clear();
  return SWPS_OK;
}

int swps_w2v_negatives(swps_w2v *w, int64_t *out, uint64_t cap, uint64_t *n) {
  *n = std::min<uint64_t>(cap, w->trace.size());
  std::copy(w->trace.begin(), w->trace.begin() + *n, out);
  return SWPS_OK;
}

int swps_w2v_set_profile(swps_w2v *w, int32_t on) {
  SWPS_TRY(swps_w2v_sync(w));
  w->timer.on = on != 0;
  return SWPS_OK;
}

int swps_w2v_kernel_times(swps_w2v *w, double *out, int32_t reset) {
  SWPS_TRY(swps_w2v_sync(w));
  for (int k = 0; k < KT_N; k++) {
    out[2 * k] = w->timer.ms[k];
    out[2 * k + 1] = (double)w->timer.cnt[k];
    if (reset) {
      w->timer.ms[k] = 0;
      w->timer.cnt[k] = 0;
    }
  }
  return SWPS_OK;
}

void *swps_w2v_stream(swps_w2v *w) { return (void *)w->s; }

int swps_unigram_starts(const uint64_t *keys, const int32_t *counts, uint64_t V, uint64_t table_size,
                        uint64_t *starts) {
  if (V == 0 || table_size == 0) return fail(SWPS_E_CFG, "empty vocab or table");
  std::vector<uint64_t> st;
  unigram_starts(keys, counts, V, table_size, st);
  std::copy(st.begin(), st.end(), starts);
  return SWPS_OK;
}

int swps_glibc_rand(uint32_t seed, uint64_t skip, uint64_t n, int32_t *out) {
  GlibcRand r(seed);
  r.discard(skip);
  for (uint64_t i = 0; i < n; i++) out[i] = r.next();
  return SWPS_OK;
}

}  // extern "C"

// ============================================================================
// Sharded mode: every rank is a worker (its own corpus,
// vocab, RNG streams and full-vocab cache, like a reference MPI rank) and a
// server for the keys BasicHashFrag assigns to node rank+1.  The caller moves
// bytes between ranks (RCCL all-to-all-v through torch.distributed; see
// swiftmpi_amd/dist.py); this library produces and consumes the payloads:
//   request    keys of the next batch grouped by owner      (pull request)
//   serve_pull owner: rows of the received keys  [n][h|v]    (pull response)
//   step       install the pulled rows, learn the batch, emit the mean
//              gradients [U][h|v] fp64 in request order        (push request)
//   serve_push owner: AdaGrad per source rank, in rank order (server.h:156-176)
// ============================================================================
extern "C" {

int swps_w2v_shard(swps_w2v *w, int32_t rank, int32_t world, int32_t frag_num) {
  if (!w->loaded) return fail(SWPS_E_STATE, "load a corpus first");
  if (w->inited) return fail(SWPS_E_STATE, "shard before swps_w2v_init / the first pull");
  if (world < 1 || rank < 0 || rank >= world) return fail(SWPS_E_CFG, "bad rank/world");
  if (w->cfg.init_mode == SWPS_W2V_INIT_REF)
    return fail(SWPS_E_UNSUPPORTED, "sharded mode initialises on the owners (SWPS_W2V_INIT_TABLE + SWPS_INIT_HASH): "
                                    "the reference's rand() order depends on message arrival");
  std::vector<uint32_t> map(frag_num);
  SWPS_TRY(swps_hashfrag_table(frag_num, world, map.data()));
  const uint64_t V = w->vocab_keys.size(), nb = w->batches.size();
  std::vector<int32_t> owner(V);
  for (uint64_t i = 0; i < V; i++) owner[i] = (int32_t)map[fmix64(w->vocab_keys[i]) % (uint64_t)frag_num] - 1;
  auto by_owner = [&](int32_t a, int32_t b) { return owner[a] != owner[b] ? owner[a] < owner[b] : a < b; };
  w->bcounts.assign(nb * world, 0);
  for (uint64_t bi = 0; bi < nb; bi++) {
    auto &b = w->batches[bi];
    std::sort(w->allK.begin() + b.kofs, w->allK.begin() + b.kofs + b.U, by_owner);
    for (uint32_t u = 0; u < b.U; u++) w->bcounts[bi * world + owner[w->allK[b.kofs + u]]]++;
  }
  w->init_order.resize(V);
  for (uint64_t i = 0; i < V; i++) w->init_order[i] = (int32_t)i;
  std::sort(w->init_order.begin(), w->init_order.end(), by_owner);
  w->icounts.assign(world, 0);
  for (uint64_t i = 0; i < V; i++) w->icounts[owner[i]]++;
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  SWPS_TRY(upload(w->d_K, w->allK, w->s));
  SWPS_TRY(upload(w->d_vkeys, w->vocab_keys, w->s));
  SWPS_TRY(upload(w->d_init_order, w->init_order, w->s));
  SWPS_HIP(hipStreamSynchronize(w->s));
  w->rank = rank;
  w->world = world;
  w->frag_num = frag_num;
  w->sharded = true;
  return SWPS_OK;
}

int swps_w2v_batch_counts(swps_w2v *w, uint64_t *out, uint64_t cap, uint64_t *nb) {
  if (!w->sharded) return fail(SWPS_E_STATE, "not sharded");
  *nb = w->batches.size();
  if (cap < w->bcounts.size()) return fail(SWPS_E_CFG, "buffer too small");
  std::copy(w->bcounts.begin(), w->bcounts.end(), out);
  return SWPS_OK;
}

// Server-side work (request, serve_pull, serve_push) is issued on the serve
// stream when one is set — the pipelined driver overlaps it, and the RCCL
// exchanges ordered on it, with the compute stream's minibatch.
int swps_w2v_set_serve_stream(swps_w2v *w, void *stream) {
  w->ss = (hipStream_t)stream;
  return SWPS_OK;
}

int swps_w2v_request(swps_w2v *w, int32_t init, uint64_t *counts, uint64_t *d_keys, uint64_t *n) {
  if (!w->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  hipStream_t ss = w->ss ? w->ss : w->s;
  if (init) {
    std::copy(w->icounts.begin(), w->icounts.end(), counts);
    *n = w->vocab_keys.size();
    if (d_keys) k_vid_keys<<<nblk(*n), 256, 0, ss>>>(w->d_init_order.as<int32_t>(), *n, w->d_vkeys.as<uint64_t>(), d_keys);
  } else {
    const uint64_t bi = w->cursor % w->batches.size();
    const auto &b = w->batches[bi];
    std::copy(w->bcounts.begin() + bi * w->world, w->bcounts.begin() + (bi + 1) * w->world, counts);
    *n = b.U;
    if (d_keys && b.U)
      k_vid_keys<<<nblk(b.U), 256, 0, ss>>>(w->d_K.as<int32_t>() + b.kofs, b.U, w->d_vkeys.as<uint64_t>(), d_keys);
  }
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

int swps_w2v_serve_pull(swps_w2v *w, const uint64_t *d_keys, const uint64_t *src_counts, int32_t insert,
                        void *d_vals) {
  if (!w->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  hipStream_t ss = w->ss ? w->ss : w->s;
  uint64_t n = 0;
  for (int r = 0; r < w->world; r++) n += src_counts[r];
  SWPS_TRY(w->d_serve_rows.ensure(std::max<uint64_t>(n, 1) * 4));
  uint32_t *rows = w->d_serve_rows.as<uint32_t>();
  if (!insert && w->slot >= 0) {  // a driver step slot: the same keys every epoch
    while ((uint64_t)w->slot >= w->slot_rows.size()) w->slot_rows.emplace_back(new swps_w2v::SlotRows());
    auto &e = *w->slot_rows[w->slot];
    if (e.n != n || !e.rows.p) {
      SWPS_TRY(e.rows.ensure(std::max<uint64_t>(n, 1) * 4));
      SWPS_TRY(table_lookup(w->t, d_keys, n, e.rows.as<uint32_t>(), ss));
      e.n = n;
      e.sorted_valid = false;
    }
    if (!d_vals && n) {  // the driver's in-place pull (AppOps::pull_in_place): the step's install reads
      if (w->world != 1) return fail(SWPS_E_STATE, "an in-place pull needs world 1");
      w->pull_rows = e.rows.as<uint32_t>();  // these rows of the shard itself
      return SWPS_OK;
    }
    return table_copy_pull(w->t, e.rows.as<uint32_t>(), n, d_vals, ss);
  }
  if (!d_vals && n) return fail(SWPS_E_STATE, "serve_pull without a value buffer needs a world-1 driver step slot");
  if (insert) {  // keys are distinct within a source, not across sources
    uint64_t off = 0;
    for (int r = 0; r < w->world; r++) {
      SWPS_TRY(table_find_or_insert(w->t, d_keys + off, src_counts[r], rows + off, ss));
      off += src_counts[r];
    }
  } else {
    SWPS_TRY(table_lookup(w->t, d_keys, n, rows, ss));
  }
  SWPS_TRY(table_copy_pull(w->t, rows, n, d_vals, ss));
  return SWPS_OK;
}

int swps_w2v_install_init(swps_w2v *w, const void *d_vals) {
  if (!w->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  const uint64_t V = w->vocab_keys.size();
  if (w->f64)
    k_install<double><<<nblk(V * 64), 256, 0, w->s>>>(w->d_init_order.as<int32_t>(), (uint32_t)V,
                                                      (const double *)d_vals, w->D, w->d_cache_h.as<double>(),
                                                      w->d_cache_v.as<double>(), w->d_local.as<int32_t>(), 0, w->cs);
  else
    k_install<float><<<nblk(V * 64), 256, 0, w->s>>>(w->d_init_order.as<int32_t>(), (uint32_t)V,
                                                     (const float *)d_vals, w->D, w->d_cache_h.as<float>(),
                                                     w->d_cache_v.as<float>(), w->d_local.as<int32_t>(), 0, w->cs);
  SWPS_HIP(hipGetLastError());
  w->inited = true;
  return SWPS_OK;
}

int swps_w2v_prep(swps_w2v *w) {
  if (!w->inited) return fail(SWPS_E_STATE, "init first");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  return prep_batch(w);
}

int swps_w2v_step(swps_w2v *w, const void *d_vals, void *d_grads) {
  if (!w->sharded) return fail(SWPS_E_STATE, "not sharded");
  if (!w->inited) return fail(SWPS_E_STATE, "init first");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  if (w->f64) return run_batch<double, double>(w, d_vals, (double *)d_grads);
  if (inter64(w->cfg)) return run_batch<float, double>(w, d_vals, (double *)d_grads);
  return run_batch<float, float>(w, d_vals, (float *)d_grads);  // fast, or BFP (d_grads: the fp64 payload)
}

// d_keys: the keys of the matching serve_pull (the push request carries its
// keys, as the reference's push Request does, global_push_access.h:48-67).
int swps_w2v_serve_push(swps_w2v *w, const uint64_t *d_keys, const void *d_grads, const uint64_t *src_counts) {
  if (!w->sharded) return fail(SWPS_E_STATE, "not sharded");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  hipStream_t ss = w->ss ? w->ss : w->s;
  uint64_t n = 0;
  for (int r = 0; r < w->world; r++) n += src_counts[r];
  const bool g32 = !w->f64 && !w->cfg.fp64_intermediates;  // fast mode: fp32 push payload
  int nsrc = 0;
  for (int r = 0; r < w->world; r++) nsrc += src_counts[r] > 0;
  if (w->slot >= 0 && (uint64_t)w->slot < w->slot_rows.size() && w->slot_rows[w->slot]->n == n &&
      w->slot_rows[w->slot]->rows.p) {  // this slot's pull looked the same keys up
    auto &e = *w->slot_rows[w->slot];
    return table_push_sources(w->t, e.rows.as<uint32_t>(), n, d_grads, ss, g32, nsrc <= 1, &e.sorted,
                              &e.sorted_valid);
  }
  SWPS_TRY(w->d_push_rows.ensure(std::max<uint64_t>(n, 1) * 4));
  SWPS_TRY(table_lookup(w->t, d_keys, n, w->d_push_rows.as<uint32_t>(), ss));
  // one AdaGrad step per source, in rank order, all sources in one pass
  return table_push_sources(w->t, w->d_push_rows.as<uint32_t>(), n, d_grads, ss, g32, nsrc <= 1);
}

// flags[j] = 1 when the j-th key served at slot `cur` (its cached row lookups) was served at slot
// `prev` too: a push of slot prev may change its row, so its pull must follow that push
static int w2v_late_mask(swps_w2v *w, int64_t cur, int64_t prev, uint8_t *d_flags, uint64_t n) {
  if (cur < 0 || prev < 0 || (uint64_t)cur >= w->slot_rows.size() || (uint64_t)prev >= w->slot_rows.size())
    return fail(SWPS_E_STATE, "late_mask: slot rows not cached");
  auto &ec = *w->slot_rows[cur], &ep = *w->slot_rows[prev];
  if (ec.n != n || (n && !ec.rows.p) || (ep.n && !ep.rows.p)) return fail(SWPS_E_STATE, "late_mask: slot rows not cached");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  hipStream_t ss = w->ss ? w->ss : w->s;
  const uint32_t cap = (uint32_t)w->t->cfg.capacity;
  if (!w->d_mark.p) {
    SWPS_TRY(w->d_mark.ensure((uint64_t)cap * 4));
    SWPS_HIP(hipMemsetAsync(w->d_mark.p, 0, (uint64_t)cap * 4, ss));
  }
  const uint32_t stamp = ++w->mark_stamp;
  if (ep.n) k_stamp_rows<<<nblk(ep.n), 256, 0, ss>>>(ep.rows.as<uint32_t>(), ep.n, cap, stamp, w->d_mark.as<uint32_t>());
  if (n)
    k_flag_rows<<<nblk(n), 256, 0, ss>>>(ec.rows.as<uint32_t>(), n, cap, stamp, w->d_mark.as<uint32_t>(), d_flags);
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

int swps_w2v_shard_comm(swps_w2v *w, swps_comm *c, int32_t frag_num) {
  if (!c) return fail(SWPS_E_CFG, "null communicator");
  if (comm_device(c) != w->t->cfg.device) return fail(SWPS_E_CFG, "communicator and table are on different devices");
  if (w->t->comm && w->t->comm != c) return fail(SWPS_E_CFG, "the table is routed over another communicator");
  if (w->drv) return fail(SWPS_E_STATE, "swps_w2v_shard_comm was already called on this context");
  SWPS_TRY(swps_w2v_shard(w, comm_rank(c), comm_world(c), frag_num));
  ShardDriver *d = new ShardDriver();
  d->c = c;
  AppOps &o = d->ops;
  o.h = w;
  o.cs = w->s;
  o.width = 2 * (uint64_t)w->D;
  o.val_bytes = w->f64 ? 8 : 4;
  o.grad_bytes = (w->f64 || w->cfg.fp64_intermediates) ? 8 : 4;
  o.batch_counts = [](void *h, uint64_t *out, uint64_t cap, uint64_t *nb) {
    return swps_w2v_batch_counts((swps_w2v *)h, out, cap, nb);
  };
  o.request = [](void *h, int32_t init, uint64_t *cnt, uint64_t *k, uint64_t *n) {
    return swps_w2v_request((swps_w2v *)h, init, cnt, k, n);
  };
  o.serve_pull = [](void *h, const uint64_t *k, const uint64_t *sc, int32_t ins, void *v) {
    return swps_w2v_serve_pull((swps_w2v *)h, k, sc, ins, v);
  };
  o.install = [](void *h, const void *v) { return swps_w2v_install_init((swps_w2v *)h, v); };
  // world 1: the step installs from the shard (serve_pull with no value buffer); SWPS_PULL_IN_PLACE=0: off (A/B)
  const char *pip = getenv("SWPS_PULL_IN_PLACE");
  o.pull_in_place = !(pip && atoi(pip) == 0);
  o.step = [](void *h, const void *v, void *g) { return swps_w2v_step((swps_w2v *)h, v, g); };
  o.serve_push = [](void *h, const uint64_t *k, const void *g, const uint64_t *sc) {
    return swps_w2v_serve_push((swps_w2v *)h, k, g, sc);
  };
  o.prep = [](void *h) { return swps_w2v_prep((swps_w2v *)h); };
  o.set_serve_stream = [](void *h, void *s) { return swps_w2v_set_serve_stream((swps_w2v *)h, s); };
  o.half_event = [](void *h) -> void * {
    swps_w2v *x = (swps_w2v *)h;
    const bool r = x->half_ready;
    x->half_ready = false;
    return r ? (void *)x->ev_half : nullptr;
  };
  o.set_slot = [](void *h, int64_t slot) {
    ((swps_w2v *)h)->slot = slot;
    return (int)SWPS_OK;
  };
  o.late_mask = [](void *h, int64_t cur, int64_t prev, uint8_t *f, uint64_t n) {
    return w2v_late_mask((swps_w2v *)h, cur, prev, f, n);
  };
  o.install_parts = [](void *h, const void *v0, const uint32_t *p0, uint64_t n0, const void *v1, const uint32_t *p1,
                       uint64_t n1) {
    auto &q = ((swps_w2v *)h)->parts;
    q.vals[0] = v0;
    q.pos[0] = p0;
    q.n[0] = n0;
    q.vals[1] = v1;
    q.pos[1] = p1;
    q.n[1] = n1;
    return (int)SWPS_OK;
  };
  const int rc = d->setup();
  if (rc) {
    delete d;
    return rc;
  }
  w->drv = d;
  return SWPS_OK;
}

int swps_w2v_exchange_stats(swps_w2v *w, int32_t on, double *out4) {
  if (!w->drv) return fail(SWPS_E_STATE, "not driven by swps_w2v_shard_comm");
  SWPS_TRY(w->drv->sync());
  if (out4) {
    out4[0] = (double)w->drv->bytes_remote;
    out4[1] = (double)w->drv->bytes_total;
    out4[2] = (double)w->drv->calls;
    out4[3] = w->drv->xms;
  }
  if (on >= 0) {
    w->drv->xprof = on != 0;
    w->drv->bytes_remote = w->drv->bytes_total = w->drv->calls = 0;
    w->drv->xms = 0;
  }
  return SWPS_OK;
}

}  // extern "C"

// ============================================================================
// Worker checkpoint (swps_w2v_save_state / swps_w2v_restore_state).  With the
// table snapshot (swps_save) it is an exact resume point at any batch
// boundary: the epoch plan is a function of the two LCG states at the epoch
// start, so those are stored instead of the plan, and the worker cache is
// stored because negatives outside a batch's key set read its stale rows.
//   "SWPSW2V2" | u64 config fp | u64 corpus fp | u64 V | u32 D | u32 esize |
//   u64 table snapshot checksum (swps_table::snap_sum of the swps_save that
//   goes with this state; restore_state requires the table to have been
//   swps_restore-d from exactly that file) |
//   u64 cursor, lstate0, fstate0, 6 counters, 2 row counters |
//   cache_h [V][D] | cache_v [V][D] (table dtype) | u64 checksum
// ============================================================================
namespace {

const char kW2VMagic[8] = {'S', 'W', 'P', 'S', 'W', '2', 'V', '2'};

uint64_t w2v_config_fp(const swps_w2v *w) {
  const auto &c = w->cfg;
  const uint64_t f[] = {(uint64_t)c.window,   (uint64_t)c.negative,         (uint64_t)c.min_sentence_length,
                        (uint64_t)c.minibatch, __float_as_uint_host(c.sample), __float_as_uint_host(c.alpha),
                        c.unigram_size,        (uint64_t)c.key_mode,         (uint64_t)c.fp64_intermediates,
                        (uint64_t)c.minibatch_vocab, (uint64_t)c.sampler,    (uint64_t)w->D,
                        (uint64_t)w->f64,      (uint64_t)w->sharded,         (uint64_t)w->rank,
                        (uint64_t)w->world,    (uint64_t)w->frag_num,
                        __float_as_uint_host(w->t->cfg.learning_rate), __float_as_uint_host(w->t->cfg.fudge)};
  return checksum64(1, f, sizeof(f));
}

uint64_t w2v_corpus_fp(const swps_w2v *w) {
  uint64_t h = checksum64(2, &w->train_words, 8);
  h = checksum64(h, w->vocab_keys.data(), w->vocab_keys.size() * 8);
  h = checksum64(h, w->counts.data(), w->counts.size() * 4);
  h = checksum64(h, w->line_off.data(), w->line_off.size() * 8);
  return checksum64(h, &w->tok_fp, 8);
}

}  // namespace

extern "C" {

int swps_w2v_save_state(swps_w2v *w, const char *path) {
  if (!w->inited) return fail(SWPS_E_STATE, "nothing to save: the context is not initialised");
  if (w->drv && w->drv->spe && w->drv->cursor % w->drv->spe != 0)
    return fail(SWPS_E_STATE, "a library-driven sharded context saves at epoch boundaries (swps_w2v_train_epochs)");
  SWPS_TRY(swps_w2v_sync(w));
  const uint64_t nb = std::max<uint64_t>(1, w->batches.size());
  // the current epoch is planned once its first batch was prepared
  const bool planned = w->cursor % nb != 0 || w->pb.valid;
  const uint64_t V = w->vocab_keys.size();
  const uint32_t es = w->f64 ? 8 : 4;
  uint64_t rt[2] = {0, 0};
  SWPS_HIP(hipMemcpy(rt, w->d_rows_touched.p, 16, hipMemcpyDeviceToHost));
  if (!w->t->snap_sum)
    return fail(SWPS_E_STATE, "save the table first (swps_save): the worker state is tied to that table snapshot");
  const uint64_t head[] = {w2v_config_fp(w), w2v_corpus_fp(w), V, (uint64_t)w->D | ((uint64_t)es << 32),
                           w->t->snap_sum};
  const uint64_t st[] = {w->cursor,       planned ? w->lstate_epoch : w->lstate,
                         planned ? w->fstate_epoch : w->fstate,
                         w->st_batches,   w->st_kept, w->st_words, w->st_pairs, w->st_pulled, w->st_pushed, rt[0], rt[1]};
  std::vector<char> cache(V * w->D * es);
  SnapFile f;
  SWPS_TRY(f.open(path, true));
  SWPS_TRY(f.put(kW2VMagic, 8));
  SWPS_TRY(f.put(head, sizeof(head)));
  SWPS_TRY(f.put(st, sizeof(st)));
  for (DevMem *m : {&w->d_cache_h, &w->d_cache_v}) {
    if (!cache.empty())  // unpadded [V][D] in the file whatever the device row stride
      SWPS_HIP(hipMemcpy2D(cache.data(), w->D * es, m->p, (size_t)w->cs * es, w->D * es, V, hipMemcpyDeviceToHost));
    SWPS_TRY(f.put(cache.data(), cache.size()));
  }
  return f.finish_write();
}

int swps_w2v_restore_state(swps_w2v *w, const char *path) {
  if (!w->loaded) return fail(SWPS_E_STATE, "load the corpus first");
  if (w->inited) return fail(SWPS_E_STATE, "restore_state needs a fresh context (corpus loaded, not initialised)");
  SWPS_HIP(hipSetDevice(w->t->cfg.device));
  const uint64_t V = w->vocab_keys.size();
  const uint32_t es = w->f64 ? 8 : 4;
  SnapFile f;
  SWPS_TRY(f.open(path, false));
  char magic[8];
  uint64_t head[5], st[11];
  if (f.get(magic, 8) != SWPS_OK || memcmp(magic, kW2VMagic, 8) != 0)
    return fail(SWPS_E_IO, std::string("not a swps word2vec state snapshot: ") + path);
  SWPS_TRY(f.get(head, sizeof(head)));
  SWPS_TRY(f.get(st, sizeof(st)));
  if (head[0] != w2v_config_fp(w))
    return fail(SWPS_E_CFG, "snapshot was taken with a different word2vec config (window, negative, minibatch, "
                            "sample, alpha, dim, dtype, precision mode, sampler or sharding)");
  if (head[1] != w2v_corpus_fp(w) || head[2] != V || head[3] != ((uint64_t)w->D | ((uint64_t)es << 32)))
    return fail(SWPS_E_CFG, "snapshot was taken on a different corpus");
  if (head[4] != w->t->snap_sum)
    return fail(SWPS_E_STATE, "the table was not restored from the table snapshot saved with this worker state "
                              "(swps_restore <prefix>.table of the same save first)");
  std::vector<char> ch(V * w->D * es), cv(ch.size());
  SWPS_TRY(f.get(ch.data(), ch.size()));
  SWPS_TRY(f.get(cv.data(), cv.size()));
  SWPS_TRY(f.finish_read());
  if (!w->sharded) {  // the vocab rows must be in the table already (swps_restore)
    DevMem dk;
    SWPS_TRY(upload(dk, w->vocab_keys, w->s));
    SWPS_TRY(table_lookup(w->t, dk.as<uint64_t>(), V, w->d_vid_row.as<uint32_t>(), w->s));
    if (table_check_error(w->t, w->s) != SWPS_OK)
      return fail(SWPS_E_STATE, "the table lacks the worker's vocab rows: swps_restore its table snapshot first");
  }
  if (!ch.empty()) {
    SWPS_HIP(hipMemcpy2D(w->d_cache_h.p, (size_t)w->cs * es, ch.data(), w->D * es, w->D * es, V,
                         hipMemcpyHostToDevice));
    SWPS_HIP(hipMemcpy2D(w->d_cache_v.p, (size_t)w->cs * es, cv.data(), w->D * es, w->D * es, V,
                         hipMemcpyHostToDevice));
  }
  SWPS_HIP(hipMemcpy(w->d_rows_touched.p, st + 9, 16, hipMemcpyHostToDevice));
  w->cursor = st[0];
  w->lstate = st[1];
  w->fstate = st[2];
  w->st_batches = st[3];
  w->st_kept = st[4];
  w->st_words = st[5];
  w->st_pairs = st[6];
  w->st_pulled = st[7];
  w->st_pushed = st[8];
  w->pb = swps_w2v::Prepped();
  const uint64_t nb = std::max<uint64_t>(1, w->batches.size());
  if (w->cursor % nb != 0) SWPS_TRY(plan_epoch(w));  // mid-epoch: re-plan from the epoch-start states
  if (w->drv) {
    // the library driver's lockstep step count is not this rank's batch count (ranks with fewer
    // batches idle to the epoch's end), so its saves are at epoch boundaries (save_state), where
    // it is epochs * spe; its server work then goes to the serve stream, as after full_pull
    if (w->cursor % nb != 0) return fail(SWPS_E_STATE, "library-driven sharded state not at an epoch boundary");
    w->drv->cursor = w->cursor / nb * w->drv->spe;
    if (w->drv->ops.set_serve_stream) SWPS_TRY(w->drv->ops.set_serve_stream(w, w->drv->S));
  }
  w->inited = true;
  return SWPS_OK;
}

}  // extern "C"
