// sent2vec on one MI355X: the reference's Sent2Vec::train
// (apps/sent2vec/sent2vec.cpp:37-181, on apps/word2vec/word2vec.h's MiniBatch,
// nthreads = 1 semantics) as HIP kernels over the HBM word table.
//
// The word table is an swps_table (W2V layout) filled by swps_load — the
// reference's ClusterServer::load (cluster/server.h:49-62) — or by a word2vec
// run on the same GPU.  WordMiniBatch never pushes, so the table is read-only
// here apart from the keys a minibatch pull misses, which the server inserts
// with a fresh WParam (accessmethod.h:63-70).  Everything that depends only
// on the corpus and the two RNG streams is fixed on the host at load time:
//   * minibatch windows (word2vec.h:323-377: next B+1 valid lines), their key
//     sets in `_local_keys` iteration order (pull order), their std::map-
//     ordered vocab and unigram^0.75 table in run-length form (word2vec.h:
//     398-425);
//   * the glibc rand() stream: 2·D per pulled key (the WParam the pull handler
//     constructs, server.h:143-150), `rand_insert_extra` more per inserted key,
//     D per sentence (Vec::random, utils/vec1.h:229-232);
//   * the main-LCG state of every sentence: niters·(1 + L·(1+negative)) draws
//     each (sent2vec.cpp:112,123,142-146; sent2vec has no subsampling).
// Per minibatch on the device:
//   k_s2v_records  one wave per sentence, lanes over its (iter, position)
//                  pairs: jump the LCG, draw b and the negatives (binary
//                  search in the minibatch's unigram run starts), write the
//                  word-table rows the position reads (context v, target h)
//   k_s2v_docs     one wave per sentence, positions in order: the sentence
//                  vector lives in registers (fp64), neu1 = sent + sum of the
//                  context v rows, fp64 dots with the target h rows, exp-table
//                  sigmoid, neu1e += g*h, sent += alpha*neu1e; written once to
//                  the HBM doc table with the sentence's error g*g.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <limits>
#include <unordered_map>
#include <atomic>
#include <chrono>
#include <thread>
#include <unordered_set>

#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "swps_internal.h"
#include "swps_rand.h"
#include "swps_sort.h"
#include "swps_wave.h"

using namespace swps;

namespace {

template <typename T> struct RowVec;
template <> struct RowVec<float> {
  using V = float4;
  static constexpr int E = 4;
};
template <> struct RowVec<double> {
  using V = double2;
  static constexpr int E = 2;
};


__device__ __forceinline__ uint64_t mod_magic(uint64_t x, uint64_t d, uint64_t m) {
  const uint64_t q = __umul64hi(x, m);  // underestimates x/d by at most 2
  uint64_t r = x - q * d;
  if (r >= d) r -= d;
  if (r >= d) r -= d;
  return r;
}

struct S2VRecArgs {
  const uint32_t *tok_row;    // word-table row of every token of the sentences
  const uint64_t *doc_tok;    // [ndocs+1] token offsets
  const uint64_t *doc_rec;    // [ndocs+1] record offsets (niters * tokens)
  const uint64_t *doc_lcg;    // [ndocs] main-LCG state before the sentence
  uint64_t d0, nd;            // sentences of this launch (one or several consecutive minibatches)
  const uint32_t *vocab_row;  // concatenated minibatch vocabs (std::map order) -> word-table row
  const uint64_t *starts;     // concatenated unigram run starts of the minibatch vocabs
  const uint32_t *doc_batch;  // minibatch of every sentence
  const uint64_t *bv0, *bs0;  // per minibatch: offset of its vocab / its run starts
  const uint32_t *bU;         // per minibatch: vocab size
  uint64_t T, mT;  // unigram table size, floor((2^64-1)/T)
  int W, N, niters;
  uint64_t mW;
  int32_t *rec;  // [records][2W + N + 1] rows, -1 = none
};

// learn_instance's draws for every (iter, pos) of one sentence
// (sent2vec.cpp:112 initial b, :123 b per position, :142-146 negatives; a
// target equal to the word is skipped, :147-148).
__global__ __launch_bounds__(256) void k_s2v_records(S2VRecArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t j = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= a.nd) return;
  const uint64_t doc = a.d0 + j;
  const uint64_t t0 = a.doc_tok[doc];
  const int L = (int)(a.doc_tok[doc + 1] - t0);
  const int W = a.W, N = a.N, S = 2 * W + N + 1;
  const uint64_t per_iter = 1 + (uint64_t)L * (N + 1);
  const uint64_t r0 = a.doc_rec[doc] - a.doc_rec[a.d0];
  const uint32_t bi = a.doc_batch[doc];  // the sentence's minibatch: its vocab and unigram table
  const uint32_t *vocab_row = a.vocab_row + a.bv0[bi];
  const uint64_t *starts = a.starts + a.bs0[bi];
  const uint32_t U = a.bU[bi];
  for (int q = lane; q < L * a.niters; q += 64) {
    const int it = q / L, p = q - it * L;
    uint64_t x = lcg_jump(a.doc_lcg[doc], (uint64_t)it * per_iter + 1 + (uint64_t)p * (N + 1), kLcgA, kLcgC);
    x = x * kLcgA + kLcgC;
    const int b = (int)mod_magic(x, (uint64_t)W, a.mW);
    const uint32_t word = a.tok_row[t0 + p];
    int32_t *r = a.rec + (r0 + q) * (uint64_t)S;
    for (int s = 0; s < 2 * W; s++) {
      int32_t cv = -1;
      if (s < 2 * (W - b)) {
        int aa = b + s;
        if (aa >= W) aa++;
        const int c = p - W + aa;
        if (c >= 0 && c < L) cv = (int32_t)a.tok_row[t0 + c];
      }
      r[s] = cv;
    }
    r[2 * W] = (int32_t)word;
    for (int d = 1; d <= N; d++) {
      x = x * kLcgA + kLcgC;
      const uint64_t slot = mod_magic(x >> 16, a.T, a.mT);
      uint32_t lo = 0, hi = U;  // largest i with starts[i] <= slot
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= slot)
          lo = mid;
        else
          hi = mid;
      }
      const uint32_t row = vocab_row[lo];
      r[2 * W + d] = row == word ? -1 : (int32_t)row;
    }
  }
}

template <typename T> struct S2VDocArgs {
  const int32_t *rec;
  const uint64_t *doc_tok, *doc_rec;
  uint64_t d0, nd;
  const int32_t *init;  // [ndocs][D] glibc rand() outputs (Vec::random)
  const T *rows;        // word table rows [h | v | h2 | v2]
  const float *exptab;
  int D, W, N, niters;
  float alpha;
  T *out;      // doc table [ndocs][D]
  float *err;  // [ndocs] learn_instance's return value of the last pass
  unsigned long long *rows_read;
};

// A word-table row slice held by one lane: NCH 16-byte chunks (elements
// [E*ci, E*ci+E) for ci = lane + 64*c) plus, when TAIL, one scalar at element
// 64*E*NCH + lane.  D = 300 fp32 is one float4 chunk + a 44-lane float tail
// (5 registers per row instead of the 8 two whole chunks take), which leaves
// room to keep two positions' rows in flight.
template <typename T, int NCH, bool TAIL> struct Slice {
  using V = typename RowVec<T>::V;
  static constexpr int E = RowVec<T>::E;
  V v[NCH];
  T t;
  __device__ __forceinline__ void load(const T *row, int lane, int D) {
#pragma unroll
    for (int c = 0; c < NCH; c++)
      if ((lane + c * 64) * E < D) v[c] = ((const V *)row)[lane + c * 64];
    if (TAIL && 64 * E * NCH + lane < D) t = row[64 * E * NCH + lane];
  }
  __device__ __forceinline__ double at(int c, int k) const { return (double)((const T *)&v[c])[k]; }
};

// per-lane fp64 accumulator of the same shape
template <typename T, int NCH, bool TAIL> struct Acc {
  static constexpr int E = RowVec<T>::E;
  double v[NCH][E];
  double t;
};

template <typename T, int NCH, bool TAIL, int G> struct DocCtx {
  using SL = Slice<T, NCH, TAIL>;
  using AC = Acc<T, NCH, TAIL>;
  static constexpr int E = RowVec<T>::E;
  const S2VDocArgs<T> &a;
  const int32_t *rec;
  int lane, D, W, N, S;

  // rows of slots [s0, s0+G) of record q: context slots read v, target slots h
  __device__ __forceinline__ void load(int q, int s0, SL (&rv)[G], int32_t (&id)[G]) const {
    const int32_t *r = rec + (uint64_t)q * S;
#pragma unroll
    for (int u = 0; u < G; u++) {
      const int slot = s0 + u;
      id[u] = slot < S ? r[slot] : -1;
      if (id[u] >= 0) rv[u].load(a.rows + (uint64_t)id[u] * 4 * D + (slot < 2 * W ? D : 0), lane, D);
    }
  }

  // learn_instance's work for slots [s0, s0+G): context slots add into neu1
  // in window order (sent2vec.cpp:125-135); target slots (positive, then the
  // negatives, :136-163) get their fp64 dots with the finished neu1 reduced
  // together (wave_sum8), g from the exp table, and neu1e += g*h
  __device__ __forceinline__ void work(int s0, const SL (&rv)[G], const int32_t (&id)[G], AC &neu1, AC &ne,
                                       float &g, unsigned long long &nctx, unsigned long long &ntgt) const {
    const bool tl = TAIL && 64 * E * NCH + lane < D;
#pragma unroll
    for (int u = 0; u < G; u++) {
      if (s0 + u >= 2 * W || id[u] < 0) continue;
      nctx++;
#pragma unroll
      for (int c = 0; c < NCH; c++)
        if ((lane + c * 64) * E < D)
#pragma unroll
          for (int k = 0; k < E; k++) neu1.v[c][k] += rv[u].at(c, k);
      if (tl) neu1.t += (double)rv[u].t;
    }
    if (s0 + G <= 2 * W) return;  // no target in this group
    double part[G];
    uint32_t tmask = 0;  // wave-uniform: present targets
#pragma unroll
    for (int u = 0; u < G; u++) {
      double pq = 0.0;
      if (s0 + u >= 2 * W && id[u] >= 0) {
        tmask |= 1u << u;
#pragma unroll
        for (int c = 0; c < NCH; c++)
          if ((lane + c * 64) * E < D)
#pragma unroll
            for (int k = 0; k < E; k++) {
              const double prod = neu1.v[c][k] * rv[u].at(c, k);
              pq += prod;
            }
        if (tl) {
          const double prod = neu1.t * (double)rv[u].t;
          pq += prod;
        }
      }
      part[u] = pq;
    }
    const double tot = wave_sum8(part, lane);
    // lanes 8u..8u+7 hold slot s0+u's dot
    const int d = s0 + (lane >> 3) - 2 * W;
    const int label = d == 0 ? 1 : 0;
    float f = 0;
    f += tot;
    float gl;
    if (f > 6)
      gl = (label - 1) * a.alpha;
    else if (f < -6)
      gl = (label - 0) * a.alpha;
    else
      gl = (label - a.exptab[(int)((f + 6) * (1000 / 6 / 2))]) * a.alpha;
#pragma unroll
    for (int u = 0; u < G; u++) {
      if (!((tmask >> u) & 1)) continue;
      ntgt++;
      g = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gl), 8 * u));
      // neu1e += g * h  (Vec operator*(double, Vec): h[i] * (double)g)
#pragma unroll
      for (int c = 0; c < NCH; c++)
        if ((lane + c * 64) * E < D)
#pragma unroll
          for (int k = 0; k < E; k++) {
            const double prod = rv[u].at(c, k) * (double)g;
            ne.v[c][k] += prod;
          }
      if (tl) {
        const double prod = (double)rv[u].t * (double)g;
        ne.t += prod;
      }
    }
  }
};

// One wave per sentence: learn_instance (sent2vec.cpp:109-181) for every
// position of every pass, in order.  All arithmetic is fp64 like the
// reference's Vec, products rounded before their adds (-ffp-contract=off).
// The sentence vector is the only loop-carried value, and no row address
// depends on it, so the rows are software-pipelined across positions: slot
// group 0 (the first G context rows) of position q+1 is in flight while
// position q's targets are reduced, and group 1 of q while group 0 is summed —
// one exposed memory latency per position at most, instead of one per group.
template <typename T, int NCH, bool TAIL, int G, int WPE = 1>  // WPE: occupancy floor (1 = none)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_s2v_docs(S2VDocArgs<T> a) {
  using C = DocCtx<T, NCH, TAIL, G>;
  using SL = typename C::SL;
  using AC = typename C::AC;
  constexpr int E = RowVec<T>::E;
  static_assert(G == 8, "wave_sum8 reduces eight targets");
  const int lane = threadIdx.x & 63;
  const uint64_t j = (uint32_t)__builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (j >= a.nd) return;
  const uint64_t doc = a.d0 + j;
  const int L = (int)(a.doc_tok[doc + 1] - a.doc_tok[doc]);
  const int D = a.D, W = a.W, N = a.N, S = 2 * W + N + 1;
  const C cx{a, a.rec + (a.doc_rec[doc] - a.doc_rec[a.d0]) * (uint64_t)S, lane, D, W, N, S};
  const bool tl = TAIL && 64 * E * NCH + lane < D;
  AC sent;
  // Vec::random: (rand()/(float)RAND_MAX - 0.5)/D
  auto init = [&](int e) {
    const float u = (float)a.init[doc * D + e] / (float)2147483647;
    return ((double)u - 0.5) / (double)D;
  };
#pragma unroll
  for (int c = 0; c < NCH; c++)
#pragma unroll
    for (int k = 0; k < E; k++) sent.v[c][k] = (lane + c * 64) * E < D ? init((lane + c * 64) * E + k) : 0.0;
  sent.t = tl ? init(64 * E * NCH + lane) : 0.0;
  float g = 0.f;
  unsigned long long nctx = 0, ntgt = 0;
  const int Q = L * a.niters;
  SL ra[G], rb[G];
  int32_t ia[G], ib[G];
  if (Q > 0) cx.load(0, 0, ra, ia);
  for (int q = 0; q < Q; q++) {
    AC neu1 = sent, ne;
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
      for (int k = 0; k < E; k++) ne.v[c][k] = 0.0;
    ne.t = 0.0;
    if (S > G) cx.load(q, G, rb, ib);
    cx.work(0, ra, ia, neu1, ne, g, nctx, ntgt);
    if (q + 1 < Q) cx.load(q + 1, 0, ra, ia);  // prefetch: group 0 of the next position
    for (int s0 = G; s0 < S; s0 += G) {
      if (s0 > G) cx.load(q, s0, rb, ib);
      cx.work(s0, rb, ib, neu1, ne, g, nctx, ntgt);
    }
    // sent_vec += alpha * neu1e (sent2vec.cpp:164)
#pragma unroll
    for (int c = 0; c < NCH; c++)
#pragma unroll
      for (int k = 0; k < E; k++) {
        const double prod = ne.v[c][k] * (double)a.alpha;
        sent.v[c][k] += prod;
      }
    if (tl) {
      const double prod = ne.t * (double)a.alpha;
      sent.t += prod;
    }
  }
#pragma unroll
  for (int c = 0; c < NCH; c++) {
    const int ci = lane + c * 64;
    if (ci * E < D)
#pragma unroll
      for (int k = 0; k < E; k++) a.out[doc * D + ci * E + k] = (T)sent.v[c][k];
  }
  if (tl) a.out[doc * D + 64 * E * NCH + lane] = (T)sent.t;
  if (lane == 0) {
    a.err[doc] = g * g;
    atomicAdd(&a.rows_read[0], nctx);
    atomicAdd(&a.rows_read[1], ntgt);
  }
}

inline unsigned nblk(uint64_t threads, unsigned bs = 256) {
  return (unsigned)std::max<uint64_t>(1, (threads + bs - 1) / bs);
}

enum { ST_REC = 0, ST_DOC, ST_N };

}  // namespace

// the sentences' Vec::random draws (utils/vec1.h:229-232: D rand() outputs per sentence, one
// contiguous run of the stream per minibatch) on the device: a thread per chunk {first output's
// destination, its stream index, count <= kRandRun} jumps there (swps_rand.h) and steps
__global__ __launch_bounds__(64) void k_s2v_rand(const uint32_t *__restrict__ base, const uint64_t *__restrict__ ch,
                                                 uint64_t nch, int32_t *__restrict__ out) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nch) return;
  const uint64_t dst = ch[3 * q], o = ch[3 * q + 1], cnt = ch[3 * q + 2];
  uint32_t ring[31];
  glibc_ring_at(base, o - 31, ring);  // o[o-31 .. o-1]
  int h = 0;  // ring[h] = o[i-31], ring[(h+28)%31] = o[i-3]
  for (uint64_t k = 0; k < cnt; k++) {
    const int h28 = h + 28 >= 31 ? h + 28 - 31 : h + 28;
    const uint32_t v = ring[h] + ring[h28];
    ring[h] = v;
    h = h + 1 == 31 ? 0 : h + 1;
    out[dst + k] = (int32_t)(v >> 1);
  }
}

struct swps_s2v {
  swps_table *t = nullptr;
  swps_s2v_cfg cfg{};
  int D = 0, W = 0, N = 0, NCH = 1;
  bool tail = false;  // row slices: NCH 16-B chunks + a scalar tail (k_s2v_docs)
  bool f64 = false;
  hipStream_t s = nullptr;
  // host schedule (fixed at load)
  struct Batch {
    uint64_t d0, d1;  // sentences
    uint64_t v0, s0;  // offsets into the concatenated minibatch vocabs / run starts
    uint32_t U;
    uint64_t recs;  // (iter, position) records of the minibatch
  };
  std::vector<Batch> batches;
  std::vector<uint64_t> doc_id, doc_tok, doc_rec, doc_lcg;
  uint64_t nlines = 0, ntok = 0, misses = 0, rand_calls = 0, max_recs = 0, max_docs = 0;
  uint64_t lstate_end = 2008;
  bool loaded = false;
  // doc sharding (swps_s2v_shard): keep the lines whose sentence id this rank owns
  int32_t shard_rank = 0, shard_world = 1, shard_frag = 0;
  uint64_t cursor = 0;
  // device
  DevMem d_tok_row, d_doc_tok, d_doc_rec, d_doc_lcg, d_vocab_row, d_starts, d_init, d_exptab, d_rec, d_out, d_err,
      d_rows_read;
  DevMem d_rec2;                // the single pass: the second records buffer (groups alternate)
  hipEvent_t ev_rec = nullptr;  // the single pass: a group's records built on the load stream
  hipEvent_t ev_docs[2] = {nullptr, nullptr};  // ... and the last documents launch that read each buffer
  DevMem d_doc_batch, d_bv0, d_bs0, d_bU;  // sentence -> minibatch; per minibatch vocab / run-start offsets, size
  // consecutive minibatches per launch, up to this many sentences (SWPS_S2V_GROUP; 0 = one minibatch):
  // the word table is read-only while training and every miss was inserted at load, so the
  // minibatches are independent and one launch over several fills the GPU (no per-minibatch tail)
  uint64_t group_docs = 262144;  // A/B on the config-5 shape: per minibatch 2.62e8 words/s, 65,536 3.02e8, 262,144 3.06e8
  // stats and HIP-event kernel timing
  uint64_t st_batches = 0, st_docs = 0, st_pos = 0;
  bool timing = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  double ms[ST_N] = {0};
  uint64_t cnt[ST_N] = {0};
};

namespace {

hipEvent_t ev_begin(swps_s2v *m, hipStream_t st = nullptr) {
  if (!m->timing) return nullptr;
  hipEvent_t e;
  (void)hipEventCreate(&e);
  (void)hipEventRecord(e, st ? st : m->s);
  return e;
}
void ev_end(swps_s2v *m, int k, hipEvent_t b, hipStream_t st = nullptr) {
  if (!b) return;
  hipEvent_t e;
  (void)hipEventCreate(&e);
  (void)hipEventRecord(e, st ? st : m->s);
  m->pending.push_back({k, {b, e}});
}
void ev_resolve(swps_s2v *m) {
  for (auto &p : m->pending) {
    float t = 0;
    (void)hipEventElapsedTime(&t, p.second.first, p.second.second);
    m->ms[p.first] += t;
    m->cnt[p.first]++;
    (void)hipEventDestroy(p.second.first);
    (void)hipEventDestroy(p.second.second);
  }
  m->pending.clear();
}

// run-length unigram^0.75 table of word2vec.h:398-425 over a vocab in std::map
// (ascending key) order: word i owns slots [st[i], st[i+1]).  The literal walk
// moves to word i+1 after the first slot a with a/T > d1_i.
// pow(c, 0.75) of the small counts most words have, computed once (the same std::pow call: the same bits)
struct Pow75 {
  double t[4096];
  Pow75() {
    for (int c = 0; c < 4096; c++) t[c] = std::pow(c, 0.75);
  }
  double operator()(int32_t c) const { return c >= 0 && c < 4096 ? t[c] : std::pow(c, 0.75); }
};
const Pow75 &pow75() {
  static const Pow75 p;
  return p;
}

// (key, count) by key, ascending — std::sort's order for distinct keys — as an LSD radix sort of
// 8-bit digits that skips the digits every key shares
void s2v_sort_by_key(std::vector<std::pair<uint64_t, int32_t>> &a, std::vector<std::pair<uint64_t, int32_t>> &tmp) {
  const size_t n = a.size();
  tmp.resize(n);
  for (int sh = 0; sh < 64; sh += 8) {
    size_t h[256] = {0};
    for (auto &x : a) h[(x.first >> sh) & 255]++;
    if (h[(a.empty() ? 0 : a[0].first >> sh) & 255] == n) continue;
    size_t o = 0;
    for (int b = 0; b < 256; b++) {
      const size_t c = h[b];
      h[b] = o;
      o += c;
    }
    for (auto &x : a) tmp[h[(x.first >> sh) & 255]++] = x;
    a.swap(tmp);
  }
}

void s2v_unigram_starts(const std::vector<std::pair<uint64_t, int32_t>> &vc, uint64_t T, std::vector<uint64_t> &st) {
  const size_t V = vc.size();
  const Pow75 &P = pow75();
  double pw = 0;
  for (auto &kc : vc) pw += P(kc.second);
  st.assign(V + 1, T);
  st[0] = 0;
  double d1 = P(vc[0].second) / (double)pw;
  for (size_t i = 0; i + 1 < V; i++) {
    const uint64_t lo = st[i];
    auto pred = [&](uint64_t a) { return (int64_t)a / (double)T > d1; };
    uint64_t a = (uint64_t)std::max<double>((double)lo, std::floor(d1 * (double)T));
    if (a > T) a = T;
    while (a > lo && pred(a - 1)) a--;
    while (a < T && !pred(a)) a++;
    if (a >= T) break;  // word i runs to the end; later words get no slots
    st[i + 1] = a + 1;
    d1 += P(vc[i + 1].second) / (double)pw;
  }
}

// The corpus as the caller holds it (read in place during the load, never copied on the host):
// tok_keys[line_off[l] .. line_off[l + 1]) are line l's word keys, sent_ids[l] the BKDR hash of
// the line (sent2vec.cpp:75)
struct S2VCorpus {
  const uint64_t *tok_keys, *line_off, *sent_ids;
  uint64_t nl;
  bool train;  // the single pass (swps_s2v_run_tokens): each group trains as soon as it is loaded
};

// The host schedule: Sent2Vec::train's loop (sent2vec.cpp:95-103) replayed over the parsed corpus.
int s2v_ingest_all(swps_s2v *m, const S2VCorpus &c);
template <typename T>
int s2v_group(swps_s2v *m, uint64_t c0, uint64_t c1, hipStream_t rs = nullptr, DevMem *rec = nullptr);

// Documents are independent and the word table is read-only:
// a rank trains exactly the lines whose sentence id BasicHashFrag assigns to
// it (hashfrag.h:33-56), with no exchange.
int s2v_ingest(swps_s2v *m, const S2VCorpus &c) {
  if (m->shard_world <= 1) return s2v_ingest_all(m, c);
  std::vector<uint32_t> map(m->shard_frag);
  SWPS_TRY(swps_hashfrag_table(m->shard_frag, m->shard_world, map.data()));
  std::vector<uint64_t> k2, off2{0}, id2;
  for (uint64_t l = 0; l < c.nl; l++) {
    if ((int32_t)map[fmix64(c.sent_ids[l]) % (uint64_t)m->shard_frag] - 1 != m->shard_rank) continue;
    k2.insert(k2.end(), c.tok_keys + c.line_off[l], c.tok_keys + c.line_off[l + 1]);
    off2.push_back(k2.size());
    id2.push_back(c.sent_ids[l]);
  }
  return s2v_ingest_all(m, S2VCorpus{k2.data(), off2.data(), id2.data(), id2.size(), c.train});
}

// the table's rows by key rank: rank_of_row[srow[q]] = q (srow: the rows sorted by key)
__global__ void k_s2v_rank_scatter(const uint32_t *__restrict__ srow, uint64_t n, uint32_t *__restrict__ rank_of_row) {
  const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) rank_of_row[srow[q]] = (uint32_t)q;
}
// every token's key rank among the table's keys at load (kNoRow: a key the table lacks)
__global__ void k_s2v_rank_map(const uint32_t *__restrict__ row, uint64_t n, const uint32_t *__restrict__ rank_of_row,
                               uint64_t got, uint32_t *__restrict__ rank) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = row[i];
  rank[i] = r != kNoRow && r < got ? rank_of_row[r] : kNoRow;
}

// every document's token rows from the rows of every corpus token (a wave per document): the
// documents are the valid lines of the minibatches trained, in order
__global__ __launch_bounds__(256) void k_s2v_doc_rows(const uint32_t *__restrict__ all_row,
                                                      const uint64_t *__restrict__ line_off,
                                                      const uint32_t *__restrict__ doc_line,
                                                      const uint64_t *__restrict__ doc_tok, uint64_t nd,
                                                      uint32_t *__restrict__ tok_row) {
  const uint64_t d = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (d >= nd) return;
  const uint64_t a = line_off[doc_line[d]], n = doc_tok[d + 1] - doc_tok[d], o = doc_tok[d];
  for (uint64_t i = lane; i < n; i += 64) tok_row[o + i] = all_row[a + i];
}

int s2v_ingest_all(swps_s2v *m, const S2VCorpus &c) {
  const uint64_t *tok_keys = c.tok_keys, *line_off = c.line_off, *sent_ids = c.sent_ids;
  const uint64_t nl = c.nl;
  const int D = m->D, B = m->cfg.minibatch, N = m->N, S = 2 * m->W + m->N + 1;
  const uint64_t T = m->cfg.unigram_size;
  hipStream_t s = m->s;
  const bool tm = getenv("SWPS_S2V_LOAD_TIMES") != nullptr;  // phase times on stderr
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double tph = now();
  auto phase = [&](const char *what) {
    if (!tm) return;
    const double t = now();
    fprintf(stderr, "[s2v load] %-28s %8.3f s\n", what, t - tph);
    tph = t;
  };
  SWPS_HIP(hipSetDevice(m->t->cfg.device));
  std::vector<uint8_t> valid(nl);
  for (uint64_t l = 0; l < nl; l++)
    valid[l] = (int64_t)(line_off[l + 1] - line_off[l]) >= (int64_t)m->cfg.min_sentence_length;
  // keys the server already holds (the loaded word vectors): the map is filled by a thread beside
  // the plan workers (they need it only for their last step, the keys the table lacks)
  uint64_t have = 0, got = 0;
  SWPS_TRY(swps_table_size(m->t, &have));
  std::vector<uint64_t> tk(std::max<uint64_t>(have, 1));
  SWPS_TRY(swps_table_keys(m->t, tk.data(), tk.size(), &got));
  phase("table keys");
  std::unique_ptr<FlatMap64> present;
  // built on the first minibatch with misses only (a corpus whose words the table holds never
  // needs it, and its 1M inserts would take a core from the plan workers at the start)
  auto wait_present = [&] {
    if (present) return;
    present.reset(new FlatMap64(got + 1024));
    for (uint64_t i = 0; i < got; i++) present->at(tk[i]) = 1;
  };
  // the rand() stream: the draws nobody reads (the WParam a pull constructs for a key the server
  // already holds, server.h:143-150) are counted and skipped in one jump before the next read
  GlibcRand rnd(m->cfg.rand_seed);
  rnd.discard(m->cfg.rand_offset);
  uint64_t skip = 0;
  auto draw = [&]() {
    if (skip) {
      rnd.discard(skip);
      skip = 0;
    }
    return rnd.next();
  };
  auto rand_val = [&](int32_t r) { return ((double)(r / (float)2147483647) - 0.5) / (double)(size_t)D; };
  std::vector<uint64_t> miss_keys;
  std::vector<double> miss_rows;     // [h | v | h2 = 0 | v2 = 0] per miss
  std::unordered_set<uint64_t> lk;   // MiniBatch::_local_keys: one object, cleared per minibatch
  uint64_t nvocab = 0, nstarts = 0;  // the minibatch vocabs (std::map order) and run starts so far (on the device)
  std::vector<uint64_t> rand_chunks;  // the sentences' rand() outputs: {destination, stream index, count}
  std::vector<uint32_t> doc_line;   // sentence -> its line
  uint64_t doc_ntok = 0;
  std::vector<uint32_t> doc_batch;  // sentence -> minibatch
  m->batches.clear();
  m->doc_id.clear();
  m->doc_tok.assign(1, 0);
  m->doc_rec.assign(1, 0);
  m->doc_lcg.clear();
  m->misses = m->max_recs = m->max_docs = 0;
  uint64_t lstate = 2008ULL;  // utils/random.h:44-47
  // Per minibatch k, everything that depends on its own lines only — gather_keys' window (the next
  // B + 1 valid lines from line k (B + 1), word2vec.h:323-377), its vocab in first-occurrence and in
  // std::map order, the unigram run starts, the keys the table did not hold at load — is built by
  // worker threads; the pass after them carries what runs through the minibatches in order (the
  // rand() stream, the table's inserts, `_local_keys`' bucket count, the LCG, the documents).
  struct Plan {
    std::vector<uint64_t> first;  // the gather's vocab, first-occurrence order
    std::vector<uint64_t> vkeys;  // std::map order
    std::vector<uint64_t> st;     // unigram run starts
    std::vector<uint64_t> cand;   // first-occurrence keys absent from the table at load
    bool zero = false;
  };
  const uint64_t K = nl ? (nl + (uint64_t)B) / (uint64_t)(B + 1) : 0;  // handler windows of B + 1 lines
  std::vector<Plan> plan(K);
  // the workers take the minibatches in order and flag each plan when it is done; the pass below
  // (this thread) follows them minibatch by minibatch instead of waiting for all of them
  std::unique_ptr<std::atomic<int>[]> ready(new std::atomic<int>[std::max<uint64_t>(K, 1)]);
  for (uint64_t k = 0; k < K; k++) ready[k].store(0, std::memory_order_relaxed);
  std::atomic<uint64_t> next{0};
  std::atomic<bool> quit{false};
  std::vector<std::thread> workers;
  // every token's table row at load (kNoRow: a key the table lacks), fetched by a thread in chunks
  // of whole lines — the caller's keys to the device (they stay there for the documents' rows), a
  // probe, the rows back — so the plans count by row in dense arrays and wait only for their lines
  // — and, first, the table's keys sorted on the device: every token's key rank (its position in
  // std::map order among the table's keys) comes back instead of its row, and a plan counts by rank
  // and reads its vocabulary off a bitmap of ranks in key order (tks_h: the keys by rank)
  const uint64_t ntok_all = line_off[nl];
  DevMem d_keys_all, d_all_row, d_all_rank, d_rank_of_row;
  SWPS_TRY(d_keys_all.ensure(std::max<uint64_t>(ntok_all, 1) * 8));
  SWPS_TRY(d_all_row.ensure(std::max<uint64_t>(ntok_all, 1) * 4));
  SWPS_TRY(d_all_rank.ensure(std::max<uint64_t>(ntok_all, 1) * 4));
  SWPS_TRY(d_rank_of_row.ensure(std::max<uint64_t>(got, 1) * 4));
  // the tokens' key ranks (not zero-filled: a plan reads a line's only after the fetch stored them)
  std::unique_ptr<uint32_t[]> rows_h(new uint32_t[std::max<uint64_t>(ntok_all, 1)]);
  std::vector<uint64_t> tks_h(std::max<uint64_t>(got, 1));
  std::atomic<int> tks_ready{0};
  std::atomic<uint64_t> rows_upto{0};
  std::atomic<int> fetch_rc{SWPS_OK};
  std::atomic<bool> fetch_stop{false};  // set only on the way out (the groups need every line's rows)
  std::thread fetch_th([&] {
    hipStream_t fs = nullptr;
    int rc = hipSetDevice(m->t->cfg.device) == hipSuccess && hipStreamCreateWithFlags(&fs, hipStreamNonBlocking) == hipSuccess
                 ? SWPS_OK : SWPS_E_HIP;
    DevMem skeys, srows, tmp;
    if (rc == SWPS_OK && got) {  // the table's keys by rank (rows sorted by key, rocPRIM onesweep)
      size_t sb = 0;
      if (skeys.ensure(got * 8) || srows.ensure(got * 4) ||
          sort_pairs_iota(nullptr, sb, m->t->row_key.as<uint64_t>(), skeys.as<uint64_t>(), srows.as<uint32_t>(), got,
                          64, fs) != hipSuccess ||
          tmp.ensure(std::max<size_t>(sb, 1)))
        rc = SWPS_E_HIP;
      sb = tmp.bytes;
      if (rc == SWPS_OK &&
          (sort_pairs_iota(tmp.p, sb, m->t->row_key.as<uint64_t>(), skeys.as<uint64_t>(), srows.as<uint32_t>(), got, 64,
                           fs) != hipSuccess ||
           (k_s2v_rank_scatter<<<(unsigned)((got + 255) / 256), 256, 0, fs>>>(srows.as<uint32_t>(), got,
                                                                              d_rank_of_row.as<uint32_t>()),
            hipGetLastError() != hipSuccess)))
        rc = SWPS_E_HIP;
    }
    // the keys by rank come back after the first chunk's ranks (the plans need them only to order
    // their vocabularies, after counting)
    bool tks_done = false;
    auto fetch_tks = [&] {
      if (tks_done) return;
      if (rc == SWPS_OK && got &&
          (hipMemcpyAsync(tks_h.data(), skeys.p, got * 8, hipMemcpyDeviceToHost, fs) != hipSuccess ||
           hipStreamSynchronize(fs) != hipSuccess))
        rc = SWPS_E_HIP;
      tks_done = true;
      tks_ready.store(1, std::memory_order_release);
    };
    uint64_t l0 = 0, chunk = 1 << 20;  // the first chunks small: the first plans start early
    while (rc == SWPS_OK && l0 < nl && !fetch_stop.load(std::memory_order_relaxed)) {
      uint64_t l1 = l0 + 1;
      while (l1 < nl && line_off[l1] - line_off[l0] < chunk) l1++;
      const uint64_t t0 = line_off[l0], t1 = line_off[l1];
      if (t1 > t0 && (hipMemcpyAsync(d_keys_all.as<uint64_t>() + t0, tok_keys + t0, (t1 - t0) * 8,
                                     hipMemcpyHostToDevice, fs) != hipSuccess ||
                      table_probe(m->t, d_keys_all.as<uint64_t>() + t0, t1 - t0, d_all_row.as<uint32_t>() + t0, fs) ||
                      (k_s2v_rank_map<<<(unsigned)((t1 - t0 + 255) / 256), 256, 0, fs>>>(
                           d_all_row.as<uint32_t>() + t0, t1 - t0, d_rank_of_row.as<uint32_t>(), got,
                           d_all_rank.as<uint32_t>() + t0),
                       hipGetLastError() != hipSuccess) ||
                      hipMemcpyAsync(rows_h.get() + t0, d_all_rank.as<uint32_t>() + t0, (t1 - t0) * 4,
                                     hipMemcpyDeviceToHost, fs) != hipSuccess ||
                      hipStreamSynchronize(fs) != hipSuccess))
        rc = SWPS_E_HIP;
      rows_upto.store(t1, std::memory_order_release);
      fetch_tks();
      l0 = l1;
      chunk = std::min<uint64_t>(chunk * 2, 8u << 20);
    }
    fetch_tks();  // (no lines, or a failed fetch: the plans must not wait for it)
    if (fs) (void)hipStreamDestroy(fs);
    if (rc != SWPS_OK) {
      fetch_rc.store(rc);
      rows_upto.store(~0ull, std::memory_order_release);  // nobody waits forever
    }
  });
  struct JoinFetch {
    std::thread &t;
    std::atomic<bool> &q;
    ~JoinFetch() {
      q.store(true);
      if (t.joinable()) t.join();
    }
  } join_fetch{fetch_th, fetch_stop};
  auto wait_rows = [&](uint64_t t) {
    for (unsigned it = 0; rows_upto.load(std::memory_order_acquire) < t; it++)
      if (it < 64)
        std::this_thread::yield();
      else
        std::this_thread::sleep_for(std::chrono::microseconds(20));
  };
  // SWPS_S2V_LOAD_TIMES: when the first plans were ready, from the workers' start
  const double t_sched0 = now();
  double t_plan[16] = {0};
  {
    // 12 plan workers (16 on the GPU boxes' CPU share measured 1.8e8 words/s single-pass, 12 2.0e8,
    // 8 1.9e8: the pass below, the group uploads and the runtime's threads need cores too)
    int nth = (int)std::min<unsigned>(12u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char *e = getenv("SWPS_S2V_THREADS")) nth = std::max(1, atoi(e));
    nth = (int)std::min<uint64_t>((uint64_t)nth, std::max<uint64_t>(K, 1));
    // the workers below the pass's priority (SWPS_S2V_NICE, default 10; 0: same): the pass, the
    // fetch thread and the group uploads are the pipeline's sequential part and must not wait for a
    // core behind the plan workers
    static const int nice_w = [] {
      const char *e = getenv("SWPS_S2V_NICE");
      return e ? atoi(e) : 10;
    }();
    auto work = [&]() {
      if (nice_w > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice_w);
      // counts by key rank in one dense array ({generation stamp, count} per rank: one line per
      // token), the ranks seen marked in a bitmap as they come; keys the table lacks (rank kNoRow:
      // the minibatch's pull inserts them) in a hash map
      struct RankCount {
        uint32_t gen;
        int32_t cnt;
      };
      FlatMap64 fq(1 << 10);
      std::vector<RankCount> rc(std::max<uint64_t>(got, 1), RankCount{0u, 0});
      std::vector<uint32_t> bits((got + 31) / 32 + 1, 0);
      std::vector<std::pair<uint64_t, int32_t>> vc, va, vtmp;
      uint32_t gen = 0;
      const uint32_t rmax = got ? (uint32_t)(got - 1) : 0u;
      for (uint64_t k; !quit.load(std::memory_order_relaxed) && (k = next.fetch_add(1)) < K;) {
        Plan &pl = plan[k];
        fq.clear();
        if (++gen == 0) {
          for (auto &e : rc) e.gen = 0u;
          gen = 1;
        }
        bool zero = false;
        int cnt = 0;
        uint64_t npres = 0, lo = ~0ull, hi = 0;
        for (uint64_t j = k * (uint64_t)(B + 1); j < nl;) {
          const uint64_t l = j++;
          if (!valid[l]) continue;
          wait_rows(line_off[l + 1]);
          const uint64_t e1 = line_off[l + 1];
          for (uint64_t i = line_off[l]; i < e1; i++) {
            // the rank 24 tokens ahead (this line's, or a stale value: a prefetch only)
            if (i + 24 < e1) __builtin_prefetch(&rc[std::min(rows_h[i + 24], rmax)], 1);
            const uint32_t q = rows_h[i];
            const uint64_t key = tok_keys[i];
            zero |= key == 0;
            if (q < got) {  // (kNoRow: absent; after a failed fetch, anything: the load fails anyway)
              RankCount &e = rc[q];
              if (e.gen != gen) {
                e.gen = gen;
                e.cnt = 1;
                pl.first.push_back(key);
                bits[q >> 5] |= 1u << (q & 31);
                lo = std::min<uint64_t>(lo, q >> 5);
                hi = std::max<uint64_t>(hi, q >> 5);
                npres++;
              } else {
                e.cnt++;
              }
            } else {
              bool fresh = false;
              fq.at(key, &fresh)++;
              if (fresh) {
                pl.first.push_back(key);
                pl.cand.push_back(key);  // absent from the table at load, first-occurrence order
              }
            }
          }
          if (++cnt > B) break;
        }
        if (pl.first.size() < 5) {  // the loop ends here (sent2vec.cpp:97)
          for (uint64_t w = lo; npres && w <= hi; w++) bits[w] = 0;
          ready[k].store(1, std::memory_order_release);
          continue;
        }
        pl.zero = zero;
        // std::map order: the present keys by rank (the bitmap), merged with the absent ones (few;
        // sorted) — the same (key, count) sequence as sorting every pair by key
        while (!tks_ready.load(std::memory_order_acquire)) std::this_thread::yield();
        vc.clear();
        va.clear();
        for (uint64_t key : pl.cand) va.emplace_back(key, fq.at(key));
        s2v_sort_by_key(va, vtmp);
        vc.reserve(pl.first.size());
        {
          size_t ia = 0;
          for (uint64_t w = lo; npres && w <= hi; w++) {
            uint32_t b = bits[w];
            bits[w] = 0;
            while (b) {
              const uint32_t q = (uint32_t)(w << 5) + (uint32_t)__builtin_ctz(b);
              b &= b - 1;
              const uint64_t key = tks_h[q];
              while (ia < va.size() && va[ia].first < key) vc.push_back(va[ia++]);
              vc.emplace_back(key, rc[q].cnt);
            }
          }
          while (ia < va.size()) vc.push_back(va[ia++]);
        }
        s2v_unigram_starts(vc, T, pl.st);
        if (tm && k < 16) t_plan[k] = now() - t_sched0;
        pl.vkeys.resize(vc.size());
        for (size_t q = 0; q < vc.size(); q++) pl.vkeys[q] = vc[q].first;
        ready[k].store(1, std::memory_order_release);
      }
    };
    for (int q = 0; q < nth; q++) workers.emplace_back(work);
  }
  struct Join {  // the workers end with this scope, on every return path
    std::vector<std::thread> &w;
    std::atomic<bool> &q;
    ~Join() {
      q.store(true);
      for (auto &t : w)
        if (t.joinable()) t.join();
    }
  } join{workers, quit};
  FlatMap64 inserted(1024);  // keys the minibatches so far inserted (the server's inserts persist)
  // Bounds for the device arrays, from the line lengths alone, so everything the pass below makes
  // can go to the device group by group (never reallocated while a group trains): the gather
  // windows' tokens bound the minibatch vocabularies, the valid lines the documents, each
  // pipeline group's records the record buffer
  uint64_t wtok = 0, ndmax = 0;
  std::vector<uint64_t> krec(K, 0), kdoc(K, 0);
  for (uint64_t k = 0; k < K; k++) {
    int cnt = 0;
    for (uint64_t l = k * (uint64_t)(B + 1); l < nl;) {
      const uint64_t q = l++;
      if (!valid[q]) continue;
      wtok += line_off[q + 1] - line_off[q];
      if (++cnt > B) break;
    }
    for (uint64_t l = k * (uint64_t)(B + 1); l < std::min<uint64_t>(nl, (k + 1) * (uint64_t)(B + 1)); l++)
      if (valid[l]) {
        kdoc[k]++;
        krec[k] += (line_off[l + 1] - line_off[l]) * (uint64_t)m->cfg.niters;
      }
    ndmax += kdoc[k];
  }
  // pipeline groups: consecutive minibatches, at most kGroupMax and group_docs documents; the pass
  // sends a group up when it is full or when the GPU has nothing left to train (the first groups
  // are small, so training starts after the first plan, and the GPU never waits for a full group
  // while plans are late).  The records buffers hold the largest group any such rule can make.
  constexpr uint64_t kGroupMax = 8;
  uint64_t grec_max = 0;
  for (uint64_t k0 = 0; k0 < K; k0++) {
    uint64_t k1 = k0 + 1, docs = kdoc[k0], recs = krec[k0];
    while (k1 < K && k1 - k0 < kGroupMax && docs + kdoc[k1] <= m->group_docs) {
      docs += kdoc[k1];
      recs += krec[k1];
      k1++;
    }
    grec_max = std::max(grec_max, recs);
  }
  const uint64_t nchunk_max = ndmax * (uint64_t)D / kRandRun + K + 1;

  rand_chunks.reserve(3 * nchunk_max);
  // The documents (the training handler's sentences, sent2vec.cpp:48-93) depend only on the lines:
  // minibatch k's are the valid lines of its B + 1, at dbase[k] .. dbase[k + 1).  A thread fills
  // every array for all minibatches in order (the LCG state runs through them) and flags each
  // minibatch; the pass reads them once flagged.  Arrays past the last minibatch trained are cut
  // after the pass.
  std::vector<uint64_t> dbase(K + 1, 0), lst_end(K, 0);
  for (uint64_t k = 0; k < K; k++) dbase[k + 1] = dbase[k] + kdoc[k];
  std::unique_ptr<std::atomic<int>[]> dready(new std::atomic<int>[std::max<uint64_t>(K, 1)]);
  for (uint64_t k = 0; k < K; k++) dready[k].store(0, std::memory_order_relaxed);
  std::atomic<bool> docs_quit{false};
  std::thread docs_th([&] {
    m->doc_id.resize(ndmax);
    m->doc_tok.resize(ndmax + 1);
    m->doc_rec.resize(ndmax + 1);
    m->doc_lcg.resize(ndmax);
    doc_line.resize(ndmax);
    doc_batch.resize(ndmax);
    m->doc_tok[0] = m->doc_rec[0] = 0;
    uint64_t ls_ = lstate, ntok = 0, nrec = 0, d = 0;
    std::vector<std::pair<uint64_t, uint64_t>> jmp;  // per document length: (A^k, c (A^k - 1) / (A - 1))
    for (uint64_t k = 0; k < K && !docs_quit.load(std::memory_order_relaxed); k++) {
      const uint64_t li = k * (uint64_t)(B + 1);
      for (uint64_t l = li; l < std::min<uint64_t>(nl, li + (uint64_t)(B + 1)); l++) {
        if (!valid[l]) continue;
        const uint64_t L = line_off[l + 1] - line_off[l];
        m->doc_id[d] = sent_ids[l];
        doc_line[d] = (uint32_t)l;
        doc_batch[d] = (uint32_t)k;
        ntok += L;
        nrec += L * (uint64_t)m->cfg.niters;
        m->doc_tok[d + 1] = ntok;
        m->doc_rec[d + 1] = nrec;
        m->doc_lcg[d] = ls_;
        // the LCG's jump over a document: the same multiplier and increment for every length L
        // (lcg_jump(x, k) = A^k x + c(A^k - 1)/(A - 1)), cached per L
        if (L >= jmp.size()) jmp.resize(L + 1, {0, 0});
        if (!jmp[L].first) {
          const uint64_t kk = (uint64_t)m->cfg.niters * (1 + L * (uint64_t)(N + 1));
          jmp[L] = {lcg_jump(1, kk, kLcgA, kLcgC) - lcg_jump(0, kk, kLcgA, kLcgC), lcg_jump(0, kk, kLcgA, kLcgC)};
        }
        ls_ = jmp[L].first * ls_ + jmp[L].second;
        d++;
      }
      lst_end[k] = ls_;
      dready[k].store(1, std::memory_order_release);
    }
  });
  struct JoinDocs {
    std::thread &t;
    std::atomic<bool> &q;
    ~JoinDocs() {
      q.store(true);
      if (t.joinable()) t.join();
    }
  } join_docs{docs_th, docs_quit};
  auto wait_docs = [&](uint64_t k) {
    for (unsigned it = 0; !dready[k].load(std::memory_order_acquire); it++)
      if (it < 64)
        std::this_thread::yield();
      else
        std::this_thread::sleep_for(std::chrono::microseconds(20));
  };
  std::vector<uint64_t> bv0(K), bs0(K), plan_st_n(K, 0);
  std::vector<uint32_t> bU(K);
  DevMem d_vkeys, d_line_off, d_doc_line, d_chunks, d_base;
  SWPS_TRY(d_vkeys.ensure(std::max<uint64_t>(wtok, 1) * 8));
  SWPS_TRY(m->d_vocab_row.ensure(std::max<uint64_t>(wtok, 1) * 4));
  SWPS_TRY(m->d_starts.ensure((wtok + K + 1) * 8));
  SWPS_TRY(m->d_doc_tok.ensure((ndmax + 1) * 8));
  SWPS_TRY(m->d_doc_rec.ensure((ndmax + 1) * 8));
  SWPS_TRY(m->d_doc_lcg.ensure(std::max<uint64_t>(ndmax, 1) * 8));
  SWPS_TRY(m->d_doc_batch.ensure(std::max<uint64_t>(ndmax, 1) * 4));
  SWPS_TRY(d_doc_line.ensure(std::max<uint64_t>(ndmax, 1) * 4));
  SWPS_TRY(m->d_bv0.ensure(std::max<uint64_t>(K, 1) * 8));
  SWPS_TRY(m->d_bs0.ensure(std::max<uint64_t>(K, 1) * 8));
  SWPS_TRY(m->d_bU.ensure(std::max<uint64_t>(K, 1) * 4));
  SWPS_TRY(m->d_init.ensure(std::max<uint64_t>(ndmax, 1) * D * 4));
  SWPS_TRY(m->d_out.ensure(std::max<uint64_t>(ndmax, 1) * D * (m->f64 ? 8 : 4)));
  SWPS_TRY(m->d_err.ensure(std::max<uint64_t>(ndmax, 1) * 4));
  SWPS_TRY(m->d_rec.ensure(std::max<uint64_t>(grec_max, 1) * (uint64_t)S * 4));
  if (c.train) SWPS_TRY(m->d_rec2.ensure(std::max<uint64_t>(grec_max, 1) * (uint64_t)S * 4));
  SWPS_TRY(m->d_tok_row.ensure(std::max<uint64_t>(ntok_all, 1) * 4));
  SWPS_TRY(d_line_off.ensure((nl + 1) * 8));
  SWPS_TRY(d_chunks.ensure(3 * nchunk_max * 8));
  {
    std::vector<float> ex(1000);
    for (int i = 0; i < 1000; i++) {  // ExpTable (word2vec.h:241-253)
      float x = (i / (float)1000 * 2 - 1) * 6;
      float e = (float)std::exp((double)x);
      ex[i] = e / (e + 1);
    }
    SWPS_TRY(upload(m->d_exptab, ex, s));
    SWPS_TRY(upload(d_base, glibc_base(m->cfg.rand_seed), s));
    SWPS_HIP(hipStreamSynchronize(s));  // ex, the base vector: locals
  }
  // the groups' vocabularies and run starts go up from two pinned staging buffers in turn (one copy
  // each per group; a pageable copy per minibatch ran at ~2 GB/s and synchronised the load stream):
  // a buffer is refilled once the copy that last read it is done
  struct Pinned {
    void *p = nullptr;
    uint64_t bytes = 0;
    hipEvent_t done = nullptr;
    ~Pinned() {
      if (done) {
        (void)hipEventSynchronize(done);
        (void)hipEventDestroy(done);
      }
      if (p) (void)hipHostFree(p);
    }
    int ensure(uint64_t n) {
      if (done) SWPS_HIP(hipEventSynchronize(done));
      if (n <= bytes) return SWPS_OK;
      if (p) SWPS_HIP(hipHostFree(p));
      p = nullptr;
      bytes = 0;
      const uint64_t want = std::max<uint64_t>(n + n / 4, 4u << 20);
      if (hipHostMalloc(&p, want) != hipSuccess) return fail(SWPS_E_OOM, "pinned staging buffer");
      bytes = want;
      return SWPS_OK;
    }
  } pin[2];
  int pin_next = 0;
  // both buffers allocated by a thread at the start, sized for a full group at a guessed vocabulary
  // of a third of its window's tokens (a larger group grows them in ensure): pinning tens of MB in
  // the first flushes delayed the first full groups by ~10 ms each
  phase("plans started, bounds, device arrays");
  double t_pin = 0, t_first_flush = 0, t_pass0 = now();  // SWPS_S2V_LOAD_TIMES
  std::thread prepin([&] {
    if (!c.train || !K || hipSetDevice(m->t->cfg.device) != hipSuccess) return;
    const double a = now();
    const uint64_t est = std::min<uint64_t>(kGroupMax * (wtok / K + 1) * 16 / 3 + (4u << 20), 256u << 20);
    for (auto &b : pin) (void)b.ensure(est);
    t_pin = now() - a;
  });
  struct JoinPin {
    std::thread &t;
    ~JoinPin() {
      if (t.joinable()) t.join();
    }
  } join_pin{prepin};
  // the load stream: each group's uploads, lookups and rand() rows; the training of a group waits
  // for its event on the table's stream
  struct LoadStream {
    hipStream_t s = nullptr;
    std::vector<hipEvent_t> ev;
    ~LoadStream() {
      if (s) (void)hipStreamSynchronize(s);
      for (auto e : ev) (void)hipEventDestroy(e);
      if (s) (void)hipStreamDestroy(s);
    }
  } ls;
  {  // at the highest priority: its small kernels (doc rows, rand() rows, records) get CUs as the
     // training kernel's waves retire instead of after the whole kernel
    int lo = 0, hi = 0;
    SWPS_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    SWPS_HIP(hipStreamCreateWithPriority(&ls.s, hipStreamNonBlocking, hi));
  }
  if (nl) SWPS_HIP(hipMemcpyAsync(d_line_off.p, line_off, (nl + 1) * 8, hipMemcpyHostToDevice, ls.s));
  const uint64_t zero = 0;
  SWPS_HIP(hipMemcpyAsync(m->d_doc_tok.p, &zero, 8, hipMemcpyHostToDevice, ls.s));
  SWPS_HIP(hipMemcpyAsync(m->d_doc_rec.p, &zero, 8, hipMemcpyHostToDevice, ls.s));
  SWPS_HIP(hipStreamSynchronize(ls.s));  // `zero` is a local
  m->cursor = 0;
  m->loaded = false;
  size_t mk_done = 0;  // misses already in the table
  uint64_t kf = 0, rc_done = 0;  // minibatches / rand chunks already on the device
  // one group's device part: its misses into the table, its vocabularies' rows and run starts, its
  // documents' arrays, token rows and rand() rows; then (train) its records + docs launch
  double t_fv = 0, t_fm = 0;  // SWPS_S2V_LOAD_TIMES: the flushes' vocabulary copies, miss inserts
  struct OwnedEvent {
    hipEvent_t e = nullptr;
    ~OwnedEvent() {
      if (e) (void)hipEventDestroy(e);
    }
  } ev_gpu;
  // nothing left to train: no group sent yet, or the last one done
  auto gpu_idle = [&]() { return !ev_gpu.e || hipEventQuery(ev_gpu.e) == hipSuccess; };
  uint64_t nflush = 0;        // groups trained so far (their records buffers alternate)
  auto flush = [&](uint64_t k1) -> int {
    if (k1 == kf) return SWPS_OK;
    const double fa = tm ? now() : 0;
    if (miss_keys.size() > mk_done) {  // rows = [h | v | h2 = 0 | v2 = 0]; the table's own stream (syncs)
      const std::vector<uint64_t> mk(miss_keys.begin() + mk_done, miss_keys.end());
      DevMem dk, dv;
      SWPS_TRY(upload(dk, mk, s));
      if (m->f64) {
        const std::vector<double> fr(miss_rows.begin() + mk_done * 4 * D, miss_rows.end());
        SWPS_TRY(upload(dv, fr, s));
        SWPS_HIP(hipStreamSynchronize(s));
      } else {
        const std::vector<float> fr(miss_rows.begin() + mk_done * 4 * D, miss_rows.end());
        SWPS_TRY(upload(dv, fr, s));
        SWPS_HIP(hipStreamSynchronize(s));
      }
      SWPS_TRY(swps_assign(m->t, dk.as<uint64_t>(), mk.size(), dv.p));
      mk_done = miss_keys.size();
    }
    const double fb = tm ? now() : 0;
    if (tm) t_fm += fb - fa;
    hipStream_t q = ls.s;
    const swps_s2v::Batch &b0 = m->batches[kf], &b1 = m->batches[k1 - 1];
    const uint64_t v0 = b0.v0, v1 = b1.v0 + b1.U, d0 = b0.d0, d1 = b1.d1;
    // Everything the group sends up goes through one pinned staging buffer (two in turn): its
    // vocabularies and run starts (consecutive in d_vkeys / d_starts), the per-minibatch offsets, the
    // documents' arrays and the rand() chunks.  A pageable copy waits for the load stream's earlier
    // work, which queues behind the training kernels: the pass would wait for the GPU at every copy.
    const uint64_t sv0 = b0.s0, sv1 = b1.s0 + plan_st_n[k1 - 1], nk = k1 - kf, nd = d1 - d0;
    const uint64_t nch = rand_chunks.size() / 3, nc = nch - rc_done;
    auto al = [](uint64_t b) { return (b + 15) & ~15ull; };
    const uint64_t o_st = al((v1 - v0) * 8), o_bv = o_st + al((sv1 - sv0) * 8), o_bs = o_bv + al(nk * 8),
                   o_bu = o_bs + al(nk * 8), o_dt = o_bu + al(nk * 4), o_dr = o_dt + al(nd * 8), o_dl = o_dr + al(nd * 8),
                   o_db = o_dl + al(nd * 8), o_dn = o_db + al(nd * 4), o_rc = o_dn + al(nd * 4), o_end = o_rc + al(nc * 24);
    if (prepin.joinable()) prepin.join();
    if (tm && !t_first_flush) t_first_flush = now() - t_pass0;
    Pinned &pb = pin[pin_next];
    pin_next ^= 1;
    SWPS_TRY(pb.ensure(o_end));  // waits for the copies that last read this buffer
    char *h = (char *)pb.p;
    uint64_t *hv = (uint64_t *)h, *hs = (uint64_t *)(h + o_st);
    // each minibatch's plan into the staging buffer on a thread of its own (~3.5 MB each)
    auto stage = [&](uint64_t k) {
      Plan &pk = plan[k];
      std::copy(pk.vkeys.begin(), pk.vkeys.end(), hv + (m->batches[k].v0 - v0));
      std::copy(pk.st.begin(), pk.st.end(), hs + (m->batches[k].s0 - sv0));
      std::vector<uint64_t>().swap(pk.vkeys);
      std::vector<uint64_t>().swap(pk.st);
    };
    {
      std::vector<std::thread> cp;
      for (uint64_t k = kf + 1; k < k1; k++) cp.emplace_back(stage, k);
      stage(kf);
      for (auto &t : cp) t.join();
    }
    for (uint64_t k = kf; k < k1; k++) {
      bv0[k] = m->batches[k].v0;
      bs0[k] = m->batches[k].s0;
      bU[k] = m->batches[k].U;
    }
    std::copy(bv0.begin() + kf, bv0.begin() + k1, (uint64_t *)(h + o_bv));
    std::copy(bs0.begin() + kf, bs0.begin() + k1, (uint64_t *)(h + o_bs));
    std::copy(bU.begin() + kf, bU.begin() + k1, (uint32_t *)(h + o_bu));
    if (nd) {
      std::copy(m->doc_tok.begin() + d0 + 1, m->doc_tok.begin() + d1 + 1, (uint64_t *)(h + o_dt));
      std::copy(m->doc_rec.begin() + d0 + 1, m->doc_rec.begin() + d1 + 1, (uint64_t *)(h + o_dr));
      std::copy(m->doc_lcg.begin() + d0, m->doc_lcg.begin() + d1, (uint64_t *)(h + o_dl));
      std::copy(doc_batch.begin() + d0, doc_batch.begin() + d1, (uint32_t *)(h + o_db));
      std::copy(doc_line.begin() + d0, doc_line.begin() + d1, (uint32_t *)(h + o_dn));
    }
    if (nc) std::copy(rand_chunks.begin() + 3 * rc_done, rand_chunks.begin() + 3 * nch, (uint64_t *)(h + o_rc));
    auto up = [&](void *dst, uint64_t off, uint64_t bytes) -> int {
      if (bytes) SWPS_HIP(hipMemcpyAsync(dst, h + off, bytes, hipMemcpyHostToDevice, q));
      return SWPS_OK;
    };
    SWPS_TRY(up(d_vkeys.as<uint64_t>() + v0, 0, (v1 - v0) * 8));
    SWPS_TRY(up(m->d_starts.as<uint64_t>() + sv0, o_st, (sv1 - sv0) * 8));
    SWPS_TRY(up(m->d_bv0.as<uint64_t>() + kf, o_bv, nk * 8));
    SWPS_TRY(up(m->d_bs0.as<uint64_t>() + kf, o_bs, nk * 8));
    SWPS_TRY(up(m->d_bU.as<uint32_t>() + kf, o_bu, nk * 4));
    SWPS_TRY(up(m->d_doc_tok.as<uint64_t>() + d0 + 1, o_dt, nd * 8));
    SWPS_TRY(up(m->d_doc_rec.as<uint64_t>() + d0 + 1, o_dr, nd * 8));
    SWPS_TRY(up(m->d_doc_lcg.as<uint64_t>() + d0, o_dl, nd * 8));
    SWPS_TRY(up(m->d_doc_batch.as<uint32_t>() + d0, o_db, nd * 4));
    SWPS_TRY(up(d_doc_line.as<uint32_t>() + d0, o_dn, nd * 4));
    SWPS_TRY(up(d_chunks.as<uint64_t>() + 3 * rc_done, o_rc, nc * 24));
    if (!pb.done) SWPS_HIP(hipEventCreateWithFlags(&pb.done, hipEventDisableTiming));
    SWPS_HIP(hipEventRecord(pb.done, q));
    if (tm) t_fv += now() - fb;
    if (v1 > v0)
      SWPS_TRY(table_lookup(m->t, d_vkeys.as<uint64_t>() + v0, v1 - v0, m->d_vocab_row.as<uint32_t>() + v0, q));
    if (nd) {
      // the group's lines' token rows: probed by the fetch thread at load; again once the pulls
      // inserted keys (their rows exist only now).  Probed, not looked up: a short line's keys
      // (read, never gathered) may be absent; the documents' keys are all in their minibatches'
      // vocabularies, whose lookup above latches
      const uint64_t la = kf * (uint64_t)(B + 1), lb = std::min<uint64_t>(nl, k1 * (uint64_t)(B + 1));
      const uint64_t t0 = line_off[la], t1 = line_off[lb];
      wait_rows(t1);  // (the plans of these minibatches waited for them already)
      if (t1 > t0 && !miss_keys.empty())
        SWPS_TRY(table_probe(m->t, d_keys_all.as<uint64_t>() + t0, t1 - t0, d_all_row.as<uint32_t>() + t0, q));
      k_s2v_doc_rows<<<(unsigned)((nd * 64 + 255) / 256), 256, 0, q>>>(
          d_all_row.as<uint32_t>(), d_line_off.as<uint64_t>(), d_doc_line.as<uint32_t>() + d0,
          m->d_doc_tok.as<uint64_t>() + d0, nd, m->d_tok_row.as<uint32_t>());
      SWPS_HIP(hipGetLastError());
    }
    if (nc) {
      k_s2v_rand<<<(unsigned)((nc + 63) / 64), 64, 0, q>>>(d_base.as<uint32_t>(), d_chunks.as<uint64_t>() + 3 * rc_done, nc,
                                                          m->d_init.as<int32_t>());
      SWPS_HIP(hipGetLastError());
      rc_done = nch;
    }
    hipEvent_t ev;
    SWPS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ls.ev.push_back(ev);
    SWPS_HIP(hipEventRecord(ev, q));
    if (c.train) {  // the group trains on the table's stream as soon as its data is there
      // its records on the load stream (after its uploads) into the buffer the group before last
      // used: the documents of the previous group may still be reading the other one
      DevMem *rb = (nflush++ & 1) ? &m->d_rec2 : &m->d_rec;
      SWPS_TRY(m->f64 ? s2v_group<double>(m, kf, k1, q, rb) : s2v_group<float>(m, kf, k1, q, rb));
      m->cursor = k1;
      if (!ev_gpu.e) SWPS_HIP(hipEventCreateWithFlags(&ev_gpu.e, hipEventDisableTiming));
      SWPS_HIP(hipEventRecord(ev_gpu.e, s));  // the GPU's queue of training ends here
    }
    kf = k1;
    return SWPS_OK;
  };
  double t_wait = 0, t_flush = 0;  // SWPS_S2V_LOAD_TIMES: the pass's time waiting for plans, in flushes
  double t_lk = 0, t_vocab = 0, t_docs = 0;  // ... refilling _local_keys, appending vocabularies, documents
  for (uint64_t k = 0; k < K; k++) {
    {
      const double a = tm ? now() : 0;
      // waiting for plan k: the minibatches already passed go up as soon as the GPU runs dry
      for (unsigned it = 0; !ready[k].load(std::memory_order_acquire); it++) {
        if (c.train && m->batches.size() > kf && gpu_idle()) {
          SWPS_TRY(flush(m->batches.size()));
          continue;
        }
        if (it < 64)
          std::this_thread::yield();
        else
          std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
      if (tm) t_wait += now() - a;
    }
    Plan &pl = plan[k];
    const std::vector<uint64_t> &first_seen = pl.first;
    if (first_seen.size() < 5) break;  // sent2vec.cpp:97
    if (pl.zero)
      return fail(SWPS_E_UNSUPPORTED, "a minibatch vocab holds key 0 (atoi of a non-numeric word): the reference "
                                      "redraws negatives that hit it, a data-dependent draw count");
    // MiniBatch::pull: one WParam (2·D rand()) per pulled key in `_local_keys`
    // order; a miss is inserted with it (server.h:143-150, accessmethod.h:63-70).  Only the misses'
    // draws are read, so a minibatch without misses skips 2·D per key in one jump.  `_local_keys`
    // is one std::unordered_set cleared per minibatch: its iteration order depends on its bucket
    // count, which depends only on the key counts inserted so far (clear() keeps the buckets;
    // libstdc++'s prime rehash policy grows them only when an insert takes the element count past
    // the bucket count, at max_load_factor 1) — so the set is filled, in the reference's insertion
    // order, only for a minibatch with misses (its iteration is read) or one whose key count would
    // grow the buckets
    bool miss = false;
    for (uint64_t key : pl.cand)
      if (!inserted.contains(key)) {
        miss = true;
        break;
      }
    // without misses the set is only kept for its bucket count: refilled after this minibatch's
    // group decision (the first minibatch's 200k inserts are not on the way to the first launch)
    const bool lk_refill = miss || lk.bucket_count() <= 1 || first_seen.size() > lk.bucket_count();  // (a new set grows at once)
    auto refill_lk = [&] {
      const double tb0 = tm ? now() : 0;
      lk.clear();
      for (uint64_t key : first_seen) lk.insert(key);
      if (tm) t_lk += now() - tb0;
    };
    if (lk_refill && miss) refill_lk();
    if (!miss) skip += 2 * (uint64_t)D * first_seen.size();
    if (miss) wait_present();  // the table's keys at load (the map thread), read only for misses
    for (uint64_t key : lk) {
      if (!miss) break;
      if (present->contains(key) || inserted.contains(key)) {
        skip += 2 * (uint64_t)D;
        continue;
      }
      const size_t o = miss_rows.size();
      miss_rows.resize(o + 4 * (size_t)D, 0.0);
      for (int i = 0; i < 2 * D; i++) miss_rows[o + i] = rand_val(draw());
      skip += m->cfg.rand_insert_extra;
      miss_keys.push_back(key);
      inserted.at(key) = 1;
      m->misses++;
    }
    const double tb1 = tm ? now() : 0;
    swps_s2v::Batch b{dbase[k], 0, nvocab, nstarts, (uint32_t)pl.vkeys.size(), 0};
    nvocab += pl.vkeys.size();
    nstarts += pl.st.size();
    plan_st_n[k] = pl.st.size();
    if (tm) t_vocab += now() - tb1;
    const double tb2 = tm ? now() : 0;
    // the training handler (sent2vec.cpp:48-93): B+1 lines, valid or not; the sentences' Vec::random
    // draws are this minibatch's next run of the stream (drawn on the device, k_s2v_rand)
    wait_docs(k);  // the documents' arrays (the docs thread)
    const uint64_t run_o = 344 + rnd.produced + skip, run_d0 = dbase[k];
    skip += (uint64_t)D * kdoc[k];  // each sentence's Vec::random: D draws
    b.d1 = dbase[k + 1];
    for (uint64_t q = 0, tot = (b.d1 - run_d0) * (uint64_t)D; q < tot; q += kRandRun)
      rand_chunks.insert(rand_chunks.end(), {run_d0 * (uint64_t)D + q, run_o + q, std::min<uint64_t>(kRandRun, tot - q)});
    b.recs = m->doc_rec[b.d1] - m->doc_rec[b.d0];
    m->max_recs = std::max(m->max_recs, b.recs);
    m->max_docs = std::max(m->max_docs, b.d1 - b.d0);
    m->batches.push_back(b);
    if (tm) t_docs += now() - tb2;
    {  // the group goes up when full (the next minibatch would not fit) or the GPU has run dry
      const uint64_t pend = k + 1 - kf, docs = dbase[k + 1] - dbase[kf];
      const bool full = pend >= kGroupMax || (k + 1 < K && docs + kdoc[k + 1] > m->group_docs);
      if (full || (c.train && gpu_idle())) {
        const double a = tm ? now() : 0;
        SWPS_TRY(flush(k + 1));
        if (tm) t_flush += now() - a;
      }
    }
    if (lk_refill && !miss) refill_lk();
    std::vector<uint64_t>().swap(pl.first);
  }
  quit.store(true);  // plans past the corpus end (sent2vec.cpp:97) are not needed
  if (fetch_rc.load() != SWPS_OK) return fail(fetch_rc.load(), "sent2vec load: token rows (HIP)");
  SWPS_TRY(flush(m->batches.size()));
  if (tm)
    fprintf(stderr, "[s2v load]   of which waiting for plans %.3f s, group uploads + launches %.3f s (vocabulary copies %.3f, "
                    "miss inserts %.3f), _local_keys %.3f s, vocabularies %.3f s, documents %.3f s; first flush %.3f s "
                    "after the schedule, pinned staging %.3f s\n", t_wait, t_flush,
            t_fv, t_fm, t_lk, t_vocab, t_docs, t_first_flush, t_pin);
  if (tm) {
    fprintf(stderr, "[s2v load]   plans 0..15 ready at (ms from the workers' start):");
    for (int q = 0; q < 16; q++) fprintf(stderr, " %.1f", t_plan[q] * 1e3);
    fprintf(stderr, "; first flush at %.1f\n", (t_first_flush + t_pass0 - t_sched0) * 1e3);
  }
  phase("minibatch vocabs + schedule + groups (host)");
  {  // the documents of the minibatches trained (the pass may stop early: sent2vec.cpp:97)
    docs_quit.store(true);
    if (docs_th.joinable()) docs_th.join();
    const uint64_t nb = m->batches.size(), ndt = nb ? m->batches.back().d1 : 0;
    m->doc_id.resize(ndt);
    m->doc_tok.resize(ndt + 1);
    m->doc_rec.resize(ndt + 1);
    m->doc_lcg.resize(ndt);
    doc_ntok = m->doc_tok[ndt];
    if (nb) lstate = lst_end[nb - 1];
  }
  m->lstate_end = lstate;
  rnd.discard(skip);
  m->rand_calls = rnd.produced;  // includes the rand_offset skipped above
  m->nlines = nl;
  m->ntok = doc_ntok;
  SWPS_HIP(hipStreamSynchronize(ls.s));
  SWPS_TRY(table_check_error(m->t, s));  // syncs (a training pass too); every key was present
  phase("last uploads + lookups");
  m->loaded = true;
  if (!c.train) m->cursor = 0;
  return SWPS_OK;
}

template <typename T, int NCH, bool TAIL> void launch_docs(const S2VDocArgs<T> &a, hipStream_t s, int wpe) {
  // one sentence per wave is a serial chain (one exposed latency per position): 4 waves per SIMD
  // (143 -> 128 VGPRs, 38 spilled) beat 3 by 8 % at D = 300; 5 (180 spilled) lose 26 %.
  // SWPS_S2V_WPE=1: the unconstrained allocation (A/B)
  if (NCH == 1 && wpe == 4)
    k_s2v_docs<T, NCH, TAIL, 8, 4><<<nblk(a.nd * 64), 256, 0, s>>>(a);
  else
    k_s2v_docs<T, NCH, TAIL, 8><<<nblk(a.nd * 64), 256, 0, s>>>(a);
}

// minibatches [c0, c1) (consecutive, no wrap) in one records + docs launch
// rs / rec (the single pass): the group's records are built on the load stream rs into rec (one of
// two buffers in turn) while the previous group trains; the documents wait for them
template <typename T> int s2v_group(swps_s2v *m, uint64_t c0, uint64_t c1, hipStream_t rs, DevMem *rec) {
  hipStream_t s = m->s;
  DevMem &drec = rec ? *rec : m->d_rec;
  hipStream_t qs = rs ? rs : s;
  const uint64_t d0 = m->batches[c0].d0, d1 = m->batches[c1 - 1].d1, nd = d1 - d0;
  uint64_t recs = 0;
  for (uint64_t c = c0; c < c1; c++) recs += m->batches[c].recs;
  m->st_batches += c1 - c0;
  if (nd == 0) return SWPS_OK;
  const int S = 2 * m->W + m->N + 1;
  if (!rec) SWPS_TRY(m->d_rec.ensure(std::max<uint64_t>(recs, 1) * (uint64_t)S * 4));
  S2VRecArgs ra{m->d_tok_row.as<uint32_t>(),
                m->d_doc_tok.as<uint64_t>(),
                m->d_doc_rec.as<uint64_t>(),
                m->d_doc_lcg.as<uint64_t>(),
                d0,
                nd,
                m->d_vocab_row.as<uint32_t>(),
                m->d_starts.as<uint64_t>(),
                m->d_doc_batch.as<uint32_t>(),
                m->d_bv0.as<uint64_t>(),
                m->d_bs0.as<uint64_t>(),
                m->d_bU.as<uint32_t>(),
                m->cfg.unigram_size,
                ~0ULL / m->cfg.unigram_size,
                m->W,
                m->N,
                m->cfg.niters,
                ~0ULL / (uint64_t)m->W,
                drec.as<int32_t>()};
  const int rb = rec == &m->d_rec2 ? 1 : 0;
  if (rs && m->ev_docs[rb]) SWPS_HIP(hipStreamWaitEvent(rs, m->ev_docs[rb], 0));  // its last reader is done
  hipEvent_t e0 = ev_begin(m, qs);
  k_s2v_records<<<nblk(nd * 64), 256, 0, qs>>>(ra);
  SWPS_HIP(hipGetLastError());
  ev_end(m, ST_REC, e0, qs);
  if (rs) {  // the documents wait for the records (and everything earlier on the load stream)
    if (!m->ev_rec) SWPS_HIP(hipEventCreateWithFlags(&m->ev_rec, hipEventDisableTiming));
    SWPS_HIP(hipEventRecord(m->ev_rec, rs));
    SWPS_HIP(hipStreamWaitEvent(s, m->ev_rec, 0));
  }
  S2VDocArgs<T> da{drec.as<int32_t>(), m->d_doc_tok.as<uint64_t>(), m->d_doc_rec.as<uint64_t>(), d0, nd,
                   m->d_init.as<int32_t>(), m->t->rows.as<T>(), m->d_exptab.as<float>(), m->D, m->W, m->N,
                   m->cfg.niters, m->cfg.alpha, m->d_out.as<T>(), m->d_err.as<float>(),
                   m->d_rows_read.as<unsigned long long>()};
  hipEvent_t e1 = ev_begin(m);
  static const int wpe = [] {
    const char *e = getenv("SWPS_S2V_WPE");
    return e ? atoi(e) : 4;
  }();
  switch (m->NCH * 2 + (m->tail ? 1 : 0)) {
    case 2: launch_docs<T, 1, false>(da, s, wpe); break;
    case 3: launch_docs<T, 1, true>(da, s, wpe); break;
    case 4: launch_docs<T, 2, false>(da, s, wpe); break;
    case 5: launch_docs<T, 2, true>(da, s, wpe); break;
    case 6: launch_docs<T, 3, false>(da, s, wpe); break;
    case 7: launch_docs<T, 3, true>(da, s, wpe); break;
    default: launch_docs<T, 4, false>(da, s, wpe); break;
  }
  SWPS_HIP(hipGetLastError());
  if (rs) {
    if (!m->ev_docs[rb]) SWPS_HIP(hipEventCreateWithFlags(&m->ev_docs[rb], hipEventDisableTiming));
    SWPS_HIP(hipEventRecord(m->ev_docs[rb], s));
  }
  ev_end(m, ST_DOC, e1);
  m->st_docs += nd;
  m->st_pos += recs;
  return SWPS_OK;
}

}  // namespace

extern "C" {

int swps_s2v_create(swps_table *t, const swps_s2v_cfg *cfg, swps_s2v **out) {
  if (!t || !cfg || !out) return fail(SWPS_E_CFG, "null argument");
  *out = nullptr;
  if (t->cfg.layout != SWPS_LAYOUT_W2V) return fail(SWPS_E_CFG, "word table layout must be SWPS_LAYOUT_W2V");
  if (t->comm) return fail(SWPS_E_UNSUPPORTED, "sent2vec reads a local (replicated) word table, not a routed one");
  if (cfg->window <= 0 || 2 * cfg->window > 64) return fail(SWPS_E_CFG, "window must be in [1, 32]");
  if (cfg->negative < 0 || cfg->negative > 62) return fail(SWPS_E_CFG, "negative must be in [0, 62]");
  if (cfg->minibatch <= 0) return fail(SWPS_E_CFG, "minibatch must be positive");
  if (cfg->niters <= 0) return fail(SWPS_E_CFG, "niters must be positive (sent2vec.cpp:28)");
  if (cfg->unigram_size == 0 || cfg->unigram_size > (1ULL << 40)) return fail(SWPS_E_CFG, "unigram_size out of range");
  const int D = t->cfg.dim;
  const int E = t->cfg.dtype == SWPS_F64 ? 2 : 4;
  if (D % E) return fail(SWPS_E_UNSUPPORTED, "dim must be a multiple of 16 bytes (4 fp32 / 2 fp64)");
  const int nch = (D / E + 63) / 64;
  if (nch > 4) return fail(SWPS_E_UNSUPPORTED, "dim too large (max 1024 fp32 / 512 fp64)");
  SWPS_HIP(hipSetDevice(t->cfg.device));
  swps_s2v *m = new swps_s2v();
  m->t = t;
  m->cfg = *cfg;
  m->D = D;
  m->W = cfg->window;
  m->N = cfg->negative;
  // whole 64-lane chunks, and the remainder as a one-scalar-per-lane tail when it fits in 64 lanes
  const int full = D / (64 * E), rem = D - full * 64 * E;
  m->NCH = nch;
  if (full >= 1 && rem > 0 && rem <= 64) {
    m->NCH = full;
    m->tail = true;
  }
  m->f64 = t->cfg.dtype == SWPS_F64;
  m->s = t->stream;
  m->timing = cfg->profile != 0;
  if (const char *e = getenv("SWPS_S2V_GROUP")) m->group_docs = strtoull(e, nullptr, 10);  // A/B timing
  int rc = m->d_rows_read.ensure(16);
  if (!rc && hipMemset(m->d_rows_read.p, 0, 16) != hipSuccess) rc = fail(SWPS_E_HIP, "memset");
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return SWPS_OK;
}

int swps_s2v_destroy(swps_s2v *m) {
  if (!m) return SWPS_OK;
  (void)hipSetDevice(m->t->cfg.device);
  (void)hipStreamSynchronize(m->s);
  ev_resolve(m);
  if (m->ev_rec) (void)hipEventDestroy(m->ev_rec);
  for (auto e : m->ev_docs)
    if (e) (void)hipEventDestroy(e);
  delete m;
  (void)hipGetLastError();  // leave no sticky error from the calls above
  return SWPS_OK;
}

// LineFileReader + split(" ") + atoi keys (word2vec.h:206,212-224); the
// sentence id is BKDR of the whole line (sent2vec.cpp:75).
int swps_s2v_load_text(swps_s2v *m, const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return fail(SWPS_E_IO, std::string("no such file or directory: ") + path);
  std::vector<uint64_t> keys, off{0}, ids;
  char *buf = nullptr;
  size_t cap = 0;
  ssize_t n;
  std::string word;
  while ((n = getdelim(&buf, &cap, '\n', f)) >= 0) {
    if (n >= 1 && buf[n - 1] == '\n') buf[--n] = 0;
    const size_t len = strlen(buf);  // std::string(cline) stops at a NUL
    ids.push_back(bkdr(buf));
    size_t i = 0;
    while (i < len) {
      while (i < len && buf[i] == ' ') i++;
      if (i >= len) break;
      size_t j = i;
      while (j < len && buf[j] != ' ') j++;
      word.assign(buf + i, j - i);
      keys.push_back((uint64_t)(int64_t)atoi(word.c_str()));
      i = j;
    }
    off.push_back(keys.size());
  }
  free(buf);
  fclose(f);
  return s2v_ingest(m, S2VCorpus{keys.data(), off.data(), ids.data(), ids.size(), false});
}

int swps_s2v_shard(swps_s2v *m, int32_t rank, int32_t world, int32_t frag_num) {
  if (m->loaded) return fail(SWPS_E_STATE, "shard before loading the corpus");
  if (world < 1 || rank < 0 || rank >= world || frag_num < world) return fail(SWPS_E_CFG, "bad rank/world/frag_num");
  m->shard_rank = rank;
  m->shard_world = world;
  m->shard_frag = frag_num;
  return SWPS_OK;
}

int swps_s2v_load_tokens(swps_s2v *m, const uint64_t *tok_keys, uint64_t ntok, const uint64_t *line_off,
                         uint64_t nlines, const uint64_t *sent_ids) {
  if (line_off[0] != 0 || line_off[nlines] != ntok) return fail(SWPS_E_CFG, "line_off must span [0, ntok]");
  for (uint64_t l = 0; l < nlines; l++)
    if (line_off[l + 1] < line_off[l]) return fail(SWPS_E_CFG, "line_off must not decrease");
  // the caller's arrays are read in place (valid during this call)
  return s2v_ingest(m, S2VCorpus{tok_keys, line_off, sent_ids, nlines, false});
}

int swps_s2v_run_tokens(swps_s2v *m, const uint64_t *tok_keys, uint64_t ntok, const uint64_t *line_off,
                        uint64_t nlines, const uint64_t *sent_ids) {
  if (line_off[0] != 0 || line_off[nlines] != ntok) return fail(SWPS_E_CFG, "line_off must span [0, ntok]");
  for (uint64_t l = 0; l < nlines; l++)
    if (line_off[l + 1] < line_off[l]) return fail(SWPS_E_CFG, "line_off must not decrease");
  SWPS_TRY(s2v_ingest(m, S2VCorpus{tok_keys, line_off, sent_ids, nlines, true}));
  return swps_s2v_sync(m);
}

int swps_s2v_info(swps_s2v *m, uint64_t *o) {
  o[0] = m->nlines;
  o[1] = m->doc_id.size();
  o[2] = m->batches.size();
  o[3] = m->ntok;
  o[4] = m->misses;
  o[5] = m->max_docs;
  o[6] = m->max_recs;
  o[7] = m->rand_calls;
  o[8] = m->lstate_end;
  return SWPS_OK;
}

int swps_s2v_train_batches(swps_s2v *m, uint64_t count) {
  if (!m->loaded) return fail(SWPS_E_STATE, "load a corpus first");
  if (m->batches.empty()) return SWPS_OK;
  SWPS_HIP(hipSetDevice(m->t->cfg.device));
  const uint64_t nb = m->batches.size();
  for (uint64_t i = 0; i < count;) {
    if (m->cursor == nb) m->cursor = 0;  // another pass over the corpus
    // consecutive minibatches up to group_docs sentences, never across the corpus end
    const uint64_t c0 = m->cursor;
    uint64_t c1 = c0 + 1, docs = m->batches[c0].d1 - m->batches[c0].d0;
    while (c1 < nb && i + (c1 - c0) < count &&
           docs + (m->batches[c1].d1 - m->batches[c1].d0) <= m->group_docs) {
      docs += m->batches[c1].d1 - m->batches[c1].d0;
      c1++;
    }
    SWPS_TRY(m->f64 ? s2v_group<double>(m, c0, c1) : s2v_group<float>(m, c0, c1));
    m->cursor = c1;
    i += c1 - c0;
  }
  return SWPS_OK;
}

int swps_s2v_train(swps_s2v *m) {
  if (!m->loaded) return fail(SWPS_E_STATE, "load a corpus first");
  if (m->cursor != 0 && m->cursor != m->batches.size()) return fail(SWPS_E_STATE, "not at the corpus start");
  m->cursor = 0;
  SWPS_TRY(swps_s2v_train_batches(m, m->batches.size()));
  return swps_s2v_sync(m);
}

int swps_s2v_sync(swps_s2v *m) {
  SWPS_HIP(hipSetDevice(m->t->cfg.device));
  SWPS_HIP(hipStreamSynchronize(m->s));
  ev_resolve(m);
  return SWPS_OK;
}

int swps_s2v_docs(swps_s2v *m, uint64_t *ids, double *vecs, float *errs, uint64_t cap, uint64_t *n) {
  SWPS_TRY(swps_s2v_sync(m));
  const uint64_t nd = m->doc_id.size();
  *n = nd;
  if (cap < nd) return fail(SWPS_E_CFG, "buffer too small");
  if (ids) std::copy(m->doc_id.begin(), m->doc_id.end(), ids);
  if (nd && vecs) {
    const size_t cnt = nd * (size_t)m->D;
    if (m->f64) {
      SWPS_HIP(hipMemcpy(vecs, m->d_out.p, cnt * 8, hipMemcpyDeviceToHost));
    } else {
      std::vector<float> h(cnt);
      SWPS_HIP(hipMemcpy(h.data(), m->d_out.p, cnt * 4, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < cnt; i++) vecs[i] = h[i];
    }
  }
  if (nd && errs) SWPS_HIP(hipMemcpy(errs, m->d_err.p, nd * 4, hipMemcpyDeviceToHost));
  return SWPS_OK;
}

// the reference's output file (sent2vec.cpp:84): "sent_id\tVec:\tv0 v1 ... \n"
// (Vec::operator<<, utils/vec1.h:112-118) at ostream precision 6, for the
// sentences of the minibatches trained so far in this pass.
int swps_s2v_dump(swps_s2v *m, const char *path) {
  SWPS_TRY(swps_s2v_sync(m));
  const uint64_t nd = m->doc_id.size();
  const uint64_t done = m->cursor ? m->batches[m->cursor - 1].d1 : 0;
  const int D = m->D;
  std::vector<double> all(std::max<uint64_t>(nd, 1) * D);
  uint64_t n = 0;
  SWPS_TRY(swps_s2v_docs(m, nullptr, all.data(), nullptr, nd, &n));
  FILE *f = fopen(path, "w");
  if (!f) return fail(SWPS_E_IO, std::string("cannot write ") + path);
  for (uint64_t d = 0; d < done; d++) {
    fprintf(f, "%llu\tVec:\t", (unsigned long long)m->doc_id[d]);
    for (int i = 0; i < D; i++) fprintf(f, "%g ", all[d * D + i]);
    fputc('\n', f);
  }
  fclose(f);
  return SWPS_OK;
}

// [batches, sentences, positions, context rows read, target rows read]
int swps_s2v_stats(swps_s2v *m, uint64_t *o) {
  SWPS_TRY(swps_s2v_sync(m));
  uint64_t rr[2] = {0, 0};
  SWPS_HIP(hipMemcpy(rr, m->d_rows_read.p, 16, hipMemcpyDeviceToHost));
  o[0] = m->st_batches;
  o[1] = m->st_docs;
  o[2] = m->st_pos;
  o[3] = rr[0];
  o[4] = rr[1];
  return SWPS_OK;
}

int swps_s2v_set_profile(swps_s2v *m, int32_t on) {
  SWPS_TRY(swps_s2v_sync(m));
  m->timing = on != 0;
  return SWPS_OK;
}

// out[2k] = ms, out[2k+1] = launches for k in {records, docs}
int swps_s2v_kernel_times(swps_s2v *m, double *out, int32_t reset) {
  SWPS_TRY(swps_s2v_sync(m));
  for (int k = 0; k < ST_N; k++) {
    out[2 * k] = m->ms[k];
    out[2 * k + 1] = (double)m->cnt[k];
    if (reset) {
      m->ms[k] = 0;
      m->cnt[k] = 0;
    }
  }
  return SWPS_OK;
}

void *swps_s2v_stream(swps_s2v *m) { return (void *)m->s; }

}  // extern "C"
