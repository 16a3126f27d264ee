// HBM-resident parameter shard: an open-addressed (linear probing) u64-key
// hash index over a dense row store, with the reference's pull / push access
// methods as kernels.
//
// Replaces parameter/sparsetable.h:17-149 (google::dense_hash_map shards
// behind pthread RWLocks, 4 heap Vecs per key) and the server handlers of
// cluster/server.h:129-176 with their access methods
// (apps/word2vec/word2vec_global.h:158-191, apps/logistic/lr.cpp:45-81).
//
// HBM layout (row-major, one dense row per key, 16-B aligned for D % 4 == 0):
//   keys[nslots]      u64   slot -> key (EMPTY = ~0, the reference's empty key)
//   slot_row[nslots]  u32   slot -> dense row index
//   row_key[cap]      u64   row -> key (dump / key listing)
//   rows[cap][R]      T     W2V: [h | v | h2sum | v2sum] (R = 4D); LR: [w | g2] (R = 2)
#include <cmath>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <type_traits>

#include "swps_internal.h"
#include "swps_sort.h"

using namespace swps;

namespace {

constexpr uint32_t kFullRow = 0xFFFFFFFEu;  // slot claimed but the shard was full (no row)

__device__ __forceinline__ uint64_t slot_hash(uint64_t key) { return splitmix64(key ^ 0x5851f42d4c957f2dULL); }

__global__ void k_find_or_insert(const uint64_t *__restrict__ keys, uint64_t n, uint64_t *tkeys, uint32_t *slot_row,
                                 uint64_t *row_key, uint32_t *counters, uint64_t mask, uint64_t cap,
                                 uint32_t *out_rows, uint8_t *out_new) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t key = keys[i];
  uint32_t row = kNoRow;
  uint8_t isnew = 0;
  if (key == kEmptyKey) {
    atomicOr(&counters[1], 4u);  // the reference's empty key cannot be stored
  } else {
    uint64_t s = slot_hash(key) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      uint64_t k = __hip_atomic_load(&tkeys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == kEmptyKey) {
        unsigned long long old =
            atomicCAS((unsigned long long *)&tkeys[s], (unsigned long long)kEmptyKey, (unsigned long long)key);
        if (old == kEmptyKey) {
          uint32_t r = atomicAdd(&counters[0], 1u);
          if (r >= cap) {
            atomicOr(&counters[1], 1u);
            __hip_atomic_store(&slot_row[s], kFullRow, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            row_key[r] = key;
            row = r;
            isnew = 1;
            // published after the row's key: a thread that finds this key
            // (the same key twice in one call) waits for it below
            __hip_atomic_store(&slot_row[s], r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          }
          break;
        }
        k = old;
      }
      if (k == key) {
        uint32_t r;
        while ((r = __hip_atomic_load(&slot_row[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == kNoRow)
          __builtin_amdgcn_s_sleep(1);  // the inserting thread is between its CAS and the store above
        if (r != kFullRow) row = r;
        break;
      }
      s = (s + 1) & mask;
    }
    if (row == kNoRow && !isnew) atomicOr(&counters[1], 1u);
  }
  out_rows[i] = row;
  if (out_new) out_new[i] = isnew;
}

// table_find_or_insert_placed, step 1: a key the table holds gets its row; a new key claims its
// slot (out = the slot index, isnew = 1) and gets its row from step 2.  The keys of one call are
// distinct (the caller's contract): a key found claimed but unpublished is an error, never a wait.
__global__ void k_claim_slots(const uint64_t *__restrict__ keys, uint64_t n, uint64_t *tkeys, const uint32_t *slot_row,
                              uint32_t *counters, uint64_t mask, uint32_t *out, uint8_t *isnew) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t key = keys[i];
  uint32_t r = kNoRow;
  uint8_t nw = 0;
  if (key == kEmptyKey) {
    atomicOr(&counters[1], 4u);
  } else {
    uint64_t s = slot_hash(key) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      uint64_t k = __hip_atomic_load(&tkeys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (k == kEmptyKey) {
        const unsigned long long old =
            atomicCAS((unsigned long long *)&tkeys[s], (unsigned long long)kEmptyKey, (unsigned long long)key);
        if (old == kEmptyKey) {
          r = (uint32_t)s;
          nw = 1;
          break;
        }
        k = old;
      }
      if (k == key) {
        r = __hip_atomic_load(&slot_row[s], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (r == kNoRow) atomicOr(&counters[1], 2u);  // the same key twice in one call
        if (r == kFullRow || r == kNoRow) r = kNoRow;
        break;
      }
      s = (s + 1) & mask;
    }
    if (r == kNoRow && !nw) atomicOr(&counters[1], 1u);
  }
  out[i] = r;
  isnew[i] = nw;
}

// step 2: the new keys' rows (assigned on the host in placement order) published into their slots
__global__ void k_publish_rows(const uint64_t *__restrict__ keys, uint64_t n, const uint32_t *__restrict__ newrow,
                               uint32_t *slot_row, uint64_t *row_key, uint32_t *counters, uint64_t cap, uint32_t *out,
                               uint8_t *isnew) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !isnew[i]) return;
  const uint32_t s = out[i], r = newrow[i];
  if (r >= cap) {
    atomicOr(&counters[1], 1u);
    __hip_atomic_store(&slot_row[s], kFullRow, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    out[i] = kNoRow;
    isnew[i] = 0;
    return;
  }
  row_key[r] = keys[i];
  __hip_atomic_store(&slot_row[s], r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  out[i] = r;
}

__global__ void k_lookup(const uint64_t *__restrict__ keys, uint64_t n, const uint64_t *__restrict__ tkeys,
                         const uint32_t *__restrict__ slot_row, uint64_t mask, uint32_t *out_rows,
                         uint32_t *counters) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t key = keys[i];
  uint32_t row = kNoRow;
  uint64_t s = slot_hash(key) & mask;
  for (uint64_t probe = 0; probe <= mask; probe++) {
    uint64_t k = tkeys[s];
    if (k == key) {
      row = slot_row[s];
      // a key whose insert found the shard full owns its slot but no row: a miss (the
      // insert already latched the table-full error), never a row index
      if (row == kFullRow) row = kNoRow;
      break;
    }
    if (k == kEmptyKey) break;
    s = (s + 1) & mask;
  }
  if (row == kNoRow && counters) atomicOr(&counters[1], 2u);
  out_rows[i] = row;
}

__device__ __forceinline__ float unit_hash(uint64_t seed, uint64_t key, uint64_t i) {
  uint64_t z = splitmix64(seed ^ splitmix64(key + 0x632be59bd9b4e019ULL * (i + 1)));
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// PullAccessMethod::init_param on a miss (accessmethod.h:64-67), one wave per key.
template <typename T>
__global__ void k_init_rows(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ rows_idx,
                            const uint8_t *__restrict__ isnew, uint64_t n, T *rows, int R, int layout, int D,
                            int mode, uint64_t seed) {
  uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  int lane = threadIdx.x & 63;
  if (w >= n || !isnew[w]) return;
  T *row = rows + (uint64_t)rows_idx[w] * R;
  uint64_t key = keys[w];
  for (int e = lane; e < R; e += 64) {
    T val = 0;
    if (mode == SWPS_INIT_HASH) {
      if (layout == SWPS_LAYOUT_W2V) {
        if (e < 2 * D) val = (T)(((double)unit_hash(seed, key, e) - 0.5) / (double)D);
      } else if (e == 0) {
        val = (T)unit_hash(seed, key, 0);
      }
    }
    row[e] = val;
  }
}

// SWPS_INIT_FLCG (LRPullAccessMethod::init_param = global_random().gen_float(), lr.cpp:48-50): the
// new keys of one call take consecutive draws of the float LCG in the order the call lists them.
// Three passes: new keys per 256-key block, the blocks' exclusive offsets (one block), each new
// key's draw by jump-ahead from the call's start state.
__global__ __launch_bounds__(256) void k_flcg_counts(const uint8_t *__restrict__ isnew, uint64_t n,
                                                     uint32_t *__restrict__ blk) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = __syncthreads_count(i < n && isnew[i]);
  if (threadIdx.x == 0) blk[blockIdx.x] = (uint32_t)c;
}

__global__ __launch_bounds__(1024) void k_flcg_scan(uint32_t *__restrict__ blk, uint64_t nb,
                                                    uint64_t *__restrict__ st) {
  __shared__ uint32_t part[1024];
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {  // 1024 blocks at a time, in order
    const uint64_t b = b0 + threadIdx.x;
    const uint32_t v = b < nb ? blk[b] : 0u;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
      const uint32_t x = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0u;
      __syncthreads();
      part[threadIdx.x] += x;
      __syncthreads();
    }
    if (b < nb) blk[b] = (uint32_t)carry + part[threadIdx.x] - v;
    carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) st[1] = carry;
}

template <typename T>
__global__ __launch_bounds__(256) void k_flcg_init(const uint8_t *__restrict__ isnew,
                                                   const uint32_t *__restrict__ rows_idx, uint64_t n,
                                                   const uint32_t *__restrict__ blk, const uint64_t *__restrict__ st,
                                                   T *rows, int R) {
  __shared__ uint32_t wcnt[4];
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool nw = i < n && isnew[i];
  const uint64_t m = __ballot(nw);
  if (lane == 0) wcnt[wv] = (uint32_t)__popcll(m);
  __syncthreads();
  if (!nw) return;
  uint32_t r = blk[blockIdx.x] + (uint32_t)__popcll(m & ((1ULL << lane) - 1));
  for (int q = 0; q < wv; q++) r += wcnt[q];
  rows[(uint64_t)rows_idx[i] * R] = (T)flcg_value(lcg_jump(st[0], (uint64_t)r + 1, kFlcgA, kLcgC));
}

__global__ void k_flcg_advance(uint64_t *st) { st[0] = lcg_jump(st[0], st[1], kFlcgA, kLcgC); }

template <typename T>
__global__ void k_copy_rows_out(const uint32_t *__restrict__ rows_idx, uint64_t n, const T *__restrict__ rows, int R,
                                int ncopy, T *__restrict__ out) {
  uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  int lane = threadIdx.x & 63;
  if (w >= n) return;
  uint32_t r = rows_idx[w];
  for (int e = lane; e < ncopy; e += 64) out[w * ncopy + e] = r == kNoRow ? (T)0 : rows[(uint64_t)r * R + e];
}

// narrow rows (LR: one fp32 weight per key): one thread per row, ncopy <= 4 elements
template <typename T>
__global__ void k_copy_rows_out_t(const uint32_t *__restrict__ rows_idx, uint64_t n, const T *__restrict__ rows, int R,
                                  int ncopy, T *__restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = rows_idx[i];
  for (int e = 0; e < ncopy; e++) out[i * ncopy + e] = r == kNoRow ? (T)0 : rows[(uint64_t)r * R + e];
}

// the same with 16-B lanes (row stride and copy width multiples of 16 B)
__global__ void k_copy_rows_out16(const uint32_t *__restrict__ rows_idx, uint64_t n, const uint4 *__restrict__ rows,
                                  int R16, int ncopy16, uint4 *__restrict__ out) {
  uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  int lane = threadIdx.x & 63;
  if (w >= n) return;
  uint32_t r = rows_idx[w];
  for (int e = lane; e < ncopy16; e += 64)
    out[w * ncopy16 + e] = r == kNoRow ? make_uint4(0, 0, 0, 0) : rows[(uint64_t)r * R16 + e];
}

template <typename T>
__global__ void k_copy_rows_in(const uint32_t *__restrict__ rows_idx, uint64_t n, T *__restrict__ rows, int R,
                               const T *__restrict__ in) {
  uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  int lane = threadIdx.x & 63;
  if (w >= n) return;
  uint32_t r = rows_idx[w];
  if (r == kNoRow) return;
  for (int e = lane; e < R; e += 64) rows[(uint64_t)r * R + e] = in[w * R + e];
}

// WPushAccessMethod::apply_push_value (word2vec_global.h:176-185), fp64 math:
//   h2 += g_h*g_h; v2 += g_v*g_v; h += lr*g_h/sqrt(h2+fudge); v likewise.
// G = wire type of the mean gradients (fp64 = the reference's wire format;
// fp32 for fast-mode contexts).  E elements per lane per chunk (16-B row
// accesses when D % E == 0, else E = 1).
template <typename T, int E> struct alignas(sizeof(T) * E) Pack {
  T v[E];
};

template <typename T, typename G, int E>
__global__ void k_push_w2v(const uint32_t *__restrict__ rows_idx, uint64_t n, const G *__restrict__ grads,
                           T *__restrict__ rows, int D, double lr, double fudge, int rule) {
  uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  int lane = threadIdx.x & 63;
  if (w >= n) return;
  uint32_t r = rows_idx[w];
  if (r == kNoRow) return;
  using PT = Pack<T, E>;
  using PG = Pack<G, E>;
  T *row = rows + (uint64_t)r * 4 * D;
  const G *g = grads + w * 2 * D;
  for (int c = lane; c < D / E; c += 64) {
    const PG gh = ((const PG *)g)[c], gv = ((const PG *)(g + D))[c];
    PT h = ((PT *)row)[c], v = ((PT *)(row + D))[c];
    if (rule == SWPS_PUSH_SGD) {
#pragma unroll
      for (int k = 0; k < E; k++) {
        h.v[k] = (T)((double)h.v[k] + (double)gh.v[k] * lr);
        v.v[k] = (T)((double)v.v[k] + (double)gv.v[k] * lr);
      }
      ((PT *)row)[c] = h;
      ((PT *)(row + D))[c] = v;
      continue;
    }
    PT h2 = ((PT *)(row + 2 * D))[c], v2 = ((PT *)(row + 3 * D))[c];
#pragma unroll
    for (int k = 0; k < E; k++) {
      const double a = (double)gh.v[k], b = (double)gv.v[k];
      const double h2n = (double)h2.v[k] + a * a;
      const double v2n = (double)v2.v[k] + b * b;
      h.v[k] = (T)((double)h.v[k] + (a * lr) / sqrt(h2n + fudge));
      v.v[k] = (T)((double)v.v[k] + (b * lr) / sqrt(v2n + fudge));
      h2.v[k] = (T)h2n;
      v2.v[k] = (T)v2n;
    }
    ((PT *)(row + 2 * D))[c] = h2;
    ((PT *)(row + 3 * D))[c] = v2;
    ((PT *)row)[c] = h;
    ((PT *)(row + D))[c] = v;
  }
}

// LRPushAccessMethod::apply_push_value (lr.cpp:68-75), in the storage type
// (fp32 for SWPS_F32, exactly the reference's float arithmetic).
template <typename T>
__global__ void k_push_lr(const uint32_t *__restrict__ rows_idx, uint64_t n, const float *__restrict__ grads,
                          T *__restrict__ rows, T lr, T fudge, int rule) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t r = rows_idx[i];
  if (r == kNoRow) return;
  T m = (T)grads[i];
  T *row = rows + (uint64_t)r * 2;
  if (rule == SWPS_PUSH_SGD) {
    row[0] = row[0] + lr * m;
    return;
  }
  T g2 = row[1] + m * m;
  row[1] = g2;
  T step = lr * m;
  row[0] = row[0] + step / (T)sqrt(g2 + fudge);
}

inline unsigned blocks_for(uint64_t threads, unsigned bs = 256) { return (unsigned)((threads + bs - 1) / bs); }

// ---- several sources' pushes in one pass (sharded serve_push) -------------
// The owner receives the mean gradients of every source rank for its keys,
// concatenated in rank order; each source's keys are distinct, a key may come
// from several sources.  The reference applies each worker's push request as
// its own AdaGrad step, in arrival order (cluster/server.h:156-176); here the
// order is the rank order.  Instead of one launch per source re-reading and
// re-writing a hot row once per source, the (row, position) pairs are
// stable-sorted by row and one wave per distinct row applies its pushes in
// position (= rank) order with the row held in registers: the same
// arithmetic, element for element (every intermediate rounded to the table
// type, as the per-source form stores it), one read and one write per row.
__global__ void k_push_keys(const uint32_t *__restrict__ rows_idx, uint64_t n, uint32_t cap,
                            uint32_t *__restrict__ key, uint32_t *__restrict__ pos) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = rows_idx[i];
  key[i] = r == kNoRow ? cap : r;  // unknown keys (the lookup flagged them) sort last and are skipped
  pos[i] = (uint32_t)i;
}

template <typename T, typename G, int E>
__global__ void k_push_w2v_multi(const uint32_t *__restrict__ rows_s, const uint32_t *__restrict__ pos_s,
                                 uint64_t n, uint32_t cap, const G *__restrict__ grads, T *__restrict__ rows, int D,
                                 double lr, double fudge, int rule) {
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= n) return;
  const uint32_t r = rows_s[w];
  if (r >= cap || (w > 0 && rows_s[w - 1] == r)) return;  // only the head of each row's run works
  uint64_t e = w + 1;
  while (e < n && rows_s[e] == r) e++;
  using PT = Pack<T, E>;
  using PG = Pack<G, E>;
  T *row = rows + (uint64_t)r * 4 * D;
  for (int c = lane; c < D / E; c += 64) {
    PT h = ((PT *)row)[c], v = ((PT *)(row + D))[c], h2 = ((PT *)(row + 2 * D))[c], v2 = ((PT *)(row + 3 * D))[c];
    for (uint64_t j = w; j < e; j++) {
      const G *g = grads + (uint64_t)pos_s[j] * 2 * D;
      const PG gh = ((const PG *)g)[c], gv = ((const PG *)(g + D))[c];
      if (rule == SWPS_PUSH_SGD) {
#pragma unroll
        for (int k = 0; k < E; k++) {
          h.v[k] = (T)((double)h.v[k] + (double)gh.v[k] * lr);
          v.v[k] = (T)((double)v.v[k] + (double)gv.v[k] * lr);
        }
        continue;
      }
#pragma unroll
      for (int k = 0; k < E; k++) {
        const double a = (double)gh.v[k], b = (double)gv.v[k];
        const double h2n = (double)h2.v[k] + a * a;
        const double v2n = (double)v2.v[k] + b * b;
        h.v[k] = (T)((double)h.v[k] + (a * lr) / sqrt(h2n + fudge));
        v.v[k] = (T)((double)v.v[k] + (b * lr) / sqrt(v2n + fudge));
        h2.v[k] = (T)h2n;
        v2.v[k] = (T)v2n;
      }
    }
    ((PT *)(row + 2 * D))[c] = h2;
    ((PT *)(row + 3 * D))[c] = v2;
    ((PT *)row)[c] = h;
    ((PT *)(row + D))[c] = v;
  }
}

// k_push_w2v_multi for fp32 rows and fp32 mean gradients (the fast-mode push payload) when
// D = 256*NCH + tail, 0 < tail <= 64 (D = 300): a lane holds NCH float4 chunks plus one
// scalar of each quarter [h | v | h2 | v2], so the whole row is one register pass (the
// float4 form runs a second, 11-lane pass at D = 300).  pos_s == nullptr: the rows are
// distinct (one source), entry w's gradients are at w.  Same per-element arithmetic in
// the same source order: bit-identical.
template <int NCH>
__global__ __launch_bounds__(256) void k_push_w2v_multi_t(const uint32_t *__restrict__ rows_s,
                                                          const uint32_t *__restrict__ pos_s, uint64_t n, uint32_t cap,
                                                          const float *__restrict__ grads, float *__restrict__ rows,
                                                          int D, double lr, double fudge, int rule) {
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= n) return;
  const uint32_t r = rows_s[w];
  if (r >= cap) return;
  uint64_t e = w + 1;
  if (pos_s) {
    if (w > 0 && rows_s[w - 1] == r) return;  // only the head of each row's run works
    while (e < n && rows_s[e] == r) e++;
  }
  const bool tl = 256 * NCH + lane < D;
  const int ti = 256 * NCH + (tl ? lane : 0);  // lanes past the tail read a valid duplicate, never store it
  float *row = rows + (uint64_t)r * 4 * D;
  float4 q[4][NCH];
  float qt[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
#pragma unroll
    for (int c = 0; c < NCH; c++) q[k][c] = ((const float4 *)(row + k * D))[lane + c * 64];
    qt[k] = row[k * D + ti];
  }
  auto ada = [&](float &x, float &x2, float gv) {
    const double a = (double)gv;
    const double x2n = (double)x2 + a * a;
    x = (float)((double)x + (a * lr) / sqrt(x2n + fudge));
    x2 = (float)x2n;
  };
  auto sgd = [&](float &x, float gv) { x = (float)((double)x + (double)gv * lr); };
  for (uint64_t j = w; j < e; j++) {
    const float *g = grads + (pos_s ? (uint64_t)pos_s[j] : j) * 2 * D;
    float4 gh[NCH], gv[NCH];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      gh[c] = ((const float4 *)g)[lane + c * 64];
      gv[c] = ((const float4 *)(g + D))[lane + c * 64];
    }
    const float ght = g[ti], gvt = g[D + ti];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      if (rule == SWPS_PUSH_SGD) {
        sgd(q[0][c].x, gh[c].x); sgd(q[0][c].y, gh[c].y); sgd(q[0][c].z, gh[c].z); sgd(q[0][c].w, gh[c].w);
        sgd(q[1][c].x, gv[c].x); sgd(q[1][c].y, gv[c].y); sgd(q[1][c].z, gv[c].z); sgd(q[1][c].w, gv[c].w);
      } else {
        ada(q[0][c].x, q[2][c].x, gh[c].x); ada(q[0][c].y, q[2][c].y, gh[c].y);
        ada(q[0][c].z, q[2][c].z, gh[c].z); ada(q[0][c].w, q[2][c].w, gh[c].w);
        ada(q[1][c].x, q[3][c].x, gv[c].x); ada(q[1][c].y, q[3][c].y, gv[c].y);
        ada(q[1][c].z, q[3][c].z, gv[c].z); ada(q[1][c].w, q[3][c].w, gv[c].w);
      }
    }
    if (rule == SWPS_PUSH_SGD) {
      sgd(qt[0], ght);
      sgd(qt[1], gvt);
    } else {
      ada(qt[0], qt[2], ght);
      ada(qt[1], qt[3], gvt);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (rule == SWPS_PUSH_SGD && k >= 2) break;
#pragma unroll
    for (int c = 0; c < NCH; c++) ((float4 *)(row + k * D))[lane + c * 64] = q[k][c];
    if (tl) row[k * D + ti] = qt[k];
  }
}

template <typename T>
__global__ void k_push_lr_multi(const uint32_t *__restrict__ rows_s, const uint32_t *__restrict__ pos_s, uint64_t n,
                                uint32_t cap, const float *__restrict__ grads, T *__restrict__ rows, T lr, T fudge,
                                int rule) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = rows_s[i];
  if (r >= cap || (i > 0 && rows_s[i - 1] == r)) return;
  T *row = rows + (uint64_t)r * 2;
  T w = row[0], g2 = row[1];
  for (uint64_t j = i; j < n && rows_s[j] == r; j++) {  // k_push_lr's steps, in source order
    const T m = (T)grads[pos_s[j]];
    if (rule == SWPS_PUSH_SGD) {
      w = w + lr * m;
      continue;
    }
    g2 = g2 + m * m;
    const T step = lr * m;
    w = w + step / (T)sqrt(g2 + fudge);
  }
  row[1] = g2;
  row[0] = w;
}

}  // namespace

namespace swps {

int table_error_code(uint32_t flags) {
  if (flags & 1) return fail(SWPS_E_OOM, "table capacity exhausted");
  if (flags & 4) return fail(SWPS_E_BADKEY, "key ~0 is the table's empty key");
  return fail(SWPS_E_BADKEY, "new key should be inited before (push of an unknown key)");
}

int table_check_error(swps_table *t, hipStream_t s) {
  uint32_t h[2];
  SWPS_HIP(hipMemcpyAsync(h, t->counters.p, sizeof(h), hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  t->host_nrows = h[0] > t->cfg.capacity ? (uint32_t)t->cfg.capacity : h[0];
  if (h[1]) {
    uint32_t z = 0;
    SWPS_HIP(hipMemcpy((uint32_t *)t->counters.p + 1, &z, 4, hipMemcpyHostToDevice));
    return table_error_code(h[1]);
  }
  return SWPS_OK;
}

// init_param of a call's new keys (isnew), stream-ordered: the table's init mode; SWPS_INIT_FLCG
// draws in call order
static int init_new_rows(swps_table *t, const uint64_t *d_keys, uint64_t n, const uint32_t *d_rows_out,
                         const uint8_t *isnew, hipStream_t s) {
  if (t->cfg.dtype == SWPS_F64)
    k_init_rows<double><<<blocks_for(n * 64), 256, 0, s>>>(d_keys, d_rows_out, isnew, n, t->rows.as<double>(),
                                                           t->row_elems, t->cfg.layout, t->cfg.dim,
                                                           t->cfg.init_mode, t->cfg.seed);
  else
    k_init_rows<float><<<blocks_for(n * 64), 256, 0, s>>>(d_keys, d_rows_out, isnew, n, t->rows.as<float>(),
                                                          t->row_elems, t->cfg.layout, t->cfg.dim,
                                                          t->cfg.init_mode, t->cfg.seed);
  SWPS_HIP(hipGetLastError());
  if (t->cfg.init_mode == SWPS_INIT_FLCG) {  // the rows are zero: their w from the call-order draws
    const uint64_t nb = (n + 255) / 256;
    SWPS_TRY(t->flcg_blk.ensure(nb * 4));
    uint32_t *blk = t->flcg_blk.as<uint32_t>();
    uint64_t *st = t->flcg.as<uint64_t>();
    k_flcg_counts<<<nb, 256, 0, s>>>(isnew, n, blk);
    k_flcg_scan<<<1, 1024, 0, s>>>(blk, nb, st);
    if (t->cfg.dtype == SWPS_F64)
      k_flcg_init<double><<<nb, 256, 0, s>>>(isnew, d_rows_out, n, blk, st, t->rows.as<double>(), t->row_elems);
    else
      k_flcg_init<float><<<nb, 256, 0, s>>>(isnew, d_rows_out, n, blk, st, t->rows.as<float>(), t->row_elems);
    k_flcg_advance<<<1, 1, 0, s>>>(st);
    SWPS_HIP(hipGetLastError());
  }
  return SWPS_OK;
}

// find-or-insert + init_param of the new keys, stream-ordered (errors latched
// in counters[1]); `isnew` is the table's own scratch
static int find_or_insert_async(swps_table *t, const uint64_t *d_keys, uint64_t n, uint32_t *d_rows_out,
                                hipStream_t s, bool init = true) {
  if (n == 0) return SWPS_OK;
  SWPS_TRY(t->isnew.ensure(n));
  uint8_t *isnew = t->isnew.as<uint8_t>();
  k_find_or_insert<<<blocks_for(n), 256, 0, s>>>(d_keys, n, t->keys.as<uint64_t>(), t->slot_row.as<uint32_t>(),
                                                  t->row_key.as<uint64_t>(), t->counters.as<uint32_t>(), t->mask,
                                                  t->cfg.capacity, d_rows_out, isnew);
  SWPS_HIP(hipGetLastError());
  return init ? init_new_rows(t, d_keys, n, d_rows_out, isnew, s) : SWPS_OK;
}

int table_find_or_insert(swps_table *t, const uint64_t *d_keys, uint64_t n, uint32_t *d_rows_out, hipStream_t s,
                         bool init) {
  if (n == 0) return SWPS_OK;
  SWPS_TRY(find_or_insert_async(t, d_keys, n, d_rows_out, s, init));
  return table_check_error(t, s);
}

// find-or-insert of n DISTINCT keys whose new rows are laid out in placement order: the new key i
// gets the next free row after every new key j with place[j] < place[i] (place: a permutation of
// 0..n-1, host memory).  Found keys keep their rows; init_param runs in call order, as in
// table_find_or_insert (an SWPS_INIT_FLCG table draws in the order of d_keys, not of place).
int table_find_or_insert_placed(swps_table *t, const uint64_t *d_keys, uint64_t n, const uint32_t *place,
                                uint32_t *d_rows_out, hipStream_t s) {
  if (n == 0) return SWPS_OK;
  if (t->mask >= 0xFFFFFFFFull) return table_find_or_insert(t, d_keys, n, d_rows_out, s);
  // the placement must be a permutation: checked before any slot is claimed, so a bad one leaves
  // the table untouched
  std::vector<uint32_t> order(n, 0xFFFFFFFFu), newrow(n, 0);
  for (uint64_t i = 0; i < n; i++) {
    if (place[i] >= n || order[place[i]] != 0xFFFFFFFFu) return fail(SWPS_E_CFG, "placement is not a permutation");
    order[place[i]] = (uint32_t)i;
  }
  SWPS_TRY(t->isnew.ensure(n));
  uint8_t *isnew = t->isnew.as<uint8_t>();
  k_claim_slots<<<blocks_for(n), 256, 0, s>>>(d_keys, n, t->keys.as<uint64_t>(), t->slot_row.as<uint32_t>(),
                                               t->counters.as<uint32_t>(), t->mask, d_rows_out, isnew);
  SWPS_HIP(hipGetLastError());
  std::vector<uint8_t> nw(n);
  uint32_t base = 0;
  SWPS_HIP(hipMemcpyAsync(nw.data(), isnew, n, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipMemcpyAsync(&base, t->counters.p, 4, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  uint64_t next = base;
  for (uint64_t j = 0; j < n; j++)
    if (nw[order[j]]) newrow[order[j]] = (uint32_t)std::min<uint64_t>(next++, 0xFFFFFFFFull);
  DevMem dn;
  SWPS_TRY(upload(dn, newrow, s));
  k_publish_rows<<<blocks_for(n), 256, 0, s>>>(d_keys, n, dn.as<uint32_t>(), t->slot_row.as<uint32_t>(),
                                                t->row_key.as<uint64_t>(), t->counters.as<uint32_t>(),
                                                t->cfg.capacity, d_rows_out, isnew);
  SWPS_HIP(hipGetLastError());
  const uint32_t nrows = (uint32_t)std::min<uint64_t>(next, 0xFFFFFFFFull);
  SWPS_HIP(hipMemcpyAsync(t->counters.p, &nrows, 4, hipMemcpyHostToDevice, s));
  SWPS_TRY(init_new_rows(t, d_keys, n, d_rows_out, isnew, s));
  return table_check_error(t, s);  // synchronises: nrows and dn outlive their copies
}

int check_app_table(swps_table *t) {
  if (!t) return fail(SWPS_E_CFG, "null table");
  if (t->cfg.push_rule != SWPS_PUSH_ADAGRAD)
    return fail(SWPS_E_UNSUPPORTED, "app contexts apply the reference apps' AdaGrad rule: the table's push_rule "
                                    "must be SWPS_PUSH_ADAGRAD");
  return SWPS_OK;
}

int table_lookup(swps_table *t, const uint64_t *d_keys, uint64_t n, uint32_t *d_rows_out, hipStream_t s) {
  if (n == 0) return SWPS_OK;
  k_lookup<<<blocks_for(n), 256, 0, s>>>(d_keys, n, t->keys.as<uint64_t>(), t->slot_row.as<uint32_t>(), t->mask,
                                          d_rows_out, t->counters.as<uint32_t>());
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

// table_lookup that latches nothing: a key the table lacks is a kNoRow answer, not an error
int table_probe(swps_table *t, const uint64_t *d_keys, uint64_t n, uint32_t *d_rows_out, hipStream_t s) {
  if (n == 0) return SWPS_OK;
  k_lookup<<<blocks_for(n), 256, 0, s>>>(d_keys, n, t->keys.as<uint64_t>(), t->slot_row.as<uint32_t>(), t->mask,
                                          d_rows_out, nullptr);
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

int table_set_rows(swps_table *t, const uint32_t *d_rows, uint64_t n, const void *d_vals, hipStream_t s) {
  if (n == 0) return SWPS_OK;
  if (t->cfg.dtype == SWPS_F64)
    k_copy_rows_in<double><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, t->rows.as<double>(), t->row_elems,
                                                              (const double *)d_vals);
  else
    k_copy_rows_in<float><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, t->rows.as<float>(), t->row_elems,
                                                             (const float *)d_vals);
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

int table_get_rows(swps_table *t, const uint32_t *d_rows, uint64_t n, void *d_vals, hipStream_t s) {
  if (n == 0) return SWPS_OK;
  if (t->cfg.dtype == SWPS_F64)
    k_copy_rows_out<double><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, t->rows.as<double>(), t->row_elems,
                                                               t->row_elems, (double *)d_vals);
  else
    k_copy_rows_out<float><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, t->rows.as<float>(), t->row_elems,
                                                              t->row_elems, (float *)d_vals);
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

// pull values (first `ncopy` elements of each row) of known rows
int table_copy_pull(swps_table *t, const uint32_t *d_rows, uint64_t n, void *d_vals, hipStream_t s) {
  if (n == 0) return SWPS_OK;
  const size_t rb = (size_t)t->row_elems * t->esize, cb = (size_t)t->pull_elems * t->esize;
  if (t->pull_elems <= 4 && cb < 16) {  // a wave per row would leave 63 lanes idle
    if (t->cfg.dtype == SWPS_F64)
      k_copy_rows_out_t<double><<<blocks_for(n), 256, 0, s>>>(d_rows, n, t->rows.as<double>(), t->row_elems,
                                                              t->pull_elems, (double *)d_vals);
    else
      k_copy_rows_out_t<float><<<blocks_for(n), 256, 0, s>>>(d_rows, n, t->rows.as<float>(), t->row_elems,
                                                             t->pull_elems, (float *)d_vals);
  } else if (rb % 16 == 0 && cb % 16 == 0)
    k_copy_rows_out16<<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, t->rows.as<uint4>(), (int)(rb / 16),
                                                        (int)(cb / 16), (uint4 *)d_vals);
  else if (t->cfg.dtype == SWPS_F64)
    k_copy_rows_out<double><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, t->rows.as<double>(), t->row_elems,
                                                               t->pull_elems, (double *)d_vals);
  else
    k_copy_rows_out<float><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, t->rows.as<float>(), t->row_elems,
                                                              t->pull_elems, (float *)d_vals);
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

template <typename T, typename G>
void launch_push_w2v(const uint32_t *d_rows, uint64_t n, const G *g, T *rows, int D, double lr, double fudge,
                     int rule, hipStream_t s) {
  constexpr int E = 16 / sizeof(T);
  if (D % E == 0)
    k_push_w2v<T, G, E><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, g, rows, D, lr, fudge, rule);
  else
    k_push_w2v<T, G, 1><<<blocks_for(n * 64), 256, 0, s>>>(d_rows, n, g, rows, D, lr, fudge, rule);
}

// the push rule on known rows (W2V: mean gradients [n][2D], fp64 or, with
// grads_f32, fp32; LR: fp32 [n])
int table_push_rows(swps_table *t, const uint32_t *d_rows, uint64_t n, const void *d_grads, hipStream_t s,
                    bool grads_f32) {
  if (n == 0) return SWPS_OK;
  if (t->cfg.layout == SWPS_LAYOUT_W2V) {
    const double lr = (double)t->cfg.learning_rate, fudge = (double)t->cfg.fudge;
    const int D = t->cfg.dim;
    if (t->cfg.dtype == SWPS_F64) {
      if (grads_f32)
        launch_push_w2v(d_rows, n, (const float *)d_grads, t->rows.as<double>(), D, lr, fudge, t->cfg.push_rule, s);
      else
        launch_push_w2v(d_rows, n, (const double *)d_grads, t->rows.as<double>(), D, lr, fudge, t->cfg.push_rule, s);
    } else {
      if (grads_f32)
        launch_push_w2v(d_rows, n, (const float *)d_grads, t->rows.as<float>(), D, lr, fudge, t->cfg.push_rule, s);
      else
        launch_push_w2v(d_rows, n, (const double *)d_grads, t->rows.as<float>(), D, lr, fudge, t->cfg.push_rule, s);
    }
  } else {
    if (t->cfg.dtype == SWPS_F64)
      k_push_lr<double><<<blocks_for(n), 256, 0, s>>>(d_rows, n, (const float *)d_grads, t->rows.as<double>(),
                                                      (double)t->cfg.learning_rate, (double)t->cfg.fudge,
                                                      t->cfg.push_rule);
    else
      k_push_lr<float><<<blocks_for(n), 256, 0, s>>>(d_rows, n, (const float *)d_grads, t->rows.as<float>(),
                                                     t->cfg.learning_rate, t->cfg.fudge, t->cfg.push_rule);
  }
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

int table_push_sources(swps_table *t, const uint32_t *d_rows, uint64_t n, const void *d_grads, hipStream_t s,
                       bool grads_f32, bool distinct, DevMem *sort_cache, bool *sort_valid) {
  if (n == 0) return SWPS_OK;
  if (n >= (1ULL << 32)) return fail(SWPS_E_UNSUPPORTED, "more than 2^32 pushed keys in one call");
  const uint32_t cap = (uint32_t)t->cfg.capacity;
  // fast-mode payload on fp32 rows of D = 256*NCH + tail: the register-pass kernel
  const int D0 = t->cfg.dim;
  const int nch = D0 / 256, tail = D0 - 256 * nch;
  const bool slice = t->cfg.layout == SWPS_LAYOUT_W2V && t->cfg.dtype == SWPS_F32 && grads_f32 && nch >= 1 &&
                     nch <= 3 && tail > 0 && tail <= 64 && t->slice_push;
  auto go_slice = [&](const uint32_t *rows_s, const uint32_t *pos_s) {
    const double lr = (double)t->cfg.learning_rate, fudge = (double)t->cfg.fudge;
    const float *g = (const float *)d_grads;
    float *rows = t->rows.as<float>();
    if (nch == 1)
      k_push_w2v_multi_t<1><<<blocks_for(n * 64), 256, 0, s>>>(rows_s, pos_s, n, cap, g, rows, D0, lr, fudge,
                                                                t->cfg.push_rule);
    else if (nch == 2)
      k_push_w2v_multi_t<2><<<blocks_for(n * 64), 256, 0, s>>>(rows_s, pos_s, n, cap, g, rows, D0, lr, fudge,
                                                                t->cfg.push_rule);
    else
      k_push_w2v_multi_t<3><<<blocks_for(n * 64), 256, 0, s>>>(rows_s, pos_s, n, cap, g, rows, D0, lr, fudge,
                                                                t->cfg.push_rule);
  };
  if (distinct && t->distinct_push) {  // one source: every row once, no grouping sort
    if (slice) {
      go_slice(d_rows, nullptr);
      SWPS_HIP(hipGetLastError());
      return SWPS_OK;
    }
    return table_push_rows(t, d_rows, n, d_grads, s, grads_f32);
  }
  int bits = 1;
  while ((1ULL << bits) <= cap) bits++;
  uint32_t *key_s = nullptr, *pos_s = nullptr;
  if (sort_cache && sort_valid && *sort_valid) {  // the same rows as an earlier call: its grouping
    key_s = sort_cache->as<uint32_t>();
    pos_s = key_s + n;
  } else {
    SWPS_TRY(t->push_scratch.ensure(n * 16));
    uint32_t *key = t->push_scratch.as<uint32_t>(), *pos = key + n;
    key_s = pos + n;
    pos_s = key_s + n;
    k_push_keys<<<blocks_for(n), 256, 0, s>>>(d_rows, n, cap, key, pos);
    SWPS_HIP(hipGetLastError());
    size_t sb = 0;
    SWPS_HIP(sort_pairs(nullptr, sb, key, key_s, pos, pos_s, n, bits, s));
    SWPS_TRY(t->sort_tmp.ensure(sb));
    sb = t->sort_tmp.bytes;
    SWPS_HIP(sort_pairs(t->sort_tmp.p, sb, key, key_s, pos, pos_s, n, bits, s));
    if (sort_cache && sort_valid) {
      SWPS_TRY(sort_cache->ensure(n * 8));
      SWPS_HIP(hipMemcpyAsync(sort_cache->p, key_s, n * 8, hipMemcpyDeviceToDevice, s));  // key_s | pos_s
      *sort_valid = true;
    }
  }
  if (slice) {
    go_slice(key_s, pos_s);
  } else if (t->cfg.layout == SWPS_LAYOUT_W2V) {
    const double lr = (double)t->cfg.learning_rate, fudge = (double)t->cfg.fudge;
    const int D = t->cfg.dim;
    auto go = [&](auto *rows, const auto *g) {
      using T = std::remove_pointer_t<decltype(rows)>;
      using G = std::remove_cv_t<std::remove_pointer_t<decltype(g)>>;
      constexpr int E = 16 / sizeof(T);
      if (D % E == 0)
        k_push_w2v_multi<T, G, E><<<blocks_for(n * 64), 256, 0, s>>>(key_s, pos_s, n, cap, g, rows, D, lr, fudge,
                                                                       t->cfg.push_rule);
      else
        k_push_w2v_multi<T, G, 1><<<blocks_for(n * 64), 256, 0, s>>>(key_s, pos_s, n, cap, g, rows, D, lr, fudge,
                                                                       t->cfg.push_rule);
    };
    if (t->cfg.dtype == SWPS_F64) {
      if (grads_f32)
        go(t->rows.as<double>(), (const float *)d_grads);
      else
        go(t->rows.as<double>(), (const double *)d_grads);
    } else {
      if (grads_f32)
        go(t->rows.as<float>(), (const float *)d_grads);
      else
        go(t->rows.as<float>(), (const double *)d_grads);
    }
  } else if (t->cfg.dtype == SWPS_F64) {
    k_push_lr_multi<double><<<blocks_for(n), 256, 0, s>>>(key_s, pos_s, n, cap, (const float *)d_grads,
                                                          t->rows.as<double>(), (double)t->cfg.learning_rate,
                                                          (double)t->cfg.fudge, t->cfg.push_rule);
  } else {
    k_push_lr_multi<float><<<blocks_for(n), 256, 0, s>>>(key_s, pos_s, n, cap, (const float *)d_grads,
                                                         t->rows.as<float>(), t->cfg.learning_rate, t->cfg.fudge,
                                                         t->cfg.push_rule);
  }
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

}  // namespace swps

extern "C" {

int swps_table_create(const swps_table_cfg *cfg, swps_table **out) {
  if (!cfg || !out) return fail(SWPS_E_CFG, "null argument");
  *out = nullptr;
  if (cfg->layout != SWPS_LAYOUT_W2V && cfg->layout != SWPS_LAYOUT_LR) return fail(SWPS_E_CFG, "unknown layout");
  if (cfg->dtype != SWPS_F32 && cfg->dtype != SWPS_F64) return fail(SWPS_E_CFG, "unknown dtype");
  if (cfg->layout == SWPS_LAYOUT_W2V && cfg->dim <= 0) return fail(SWPS_E_CFG, "dim must be positive");
  if (cfg->capacity == 0 || cfg->capacity >= 0xFFFFFFF0ULL) return fail(SWPS_E_CFG, "capacity out of range");
  if (cfg->push_rule != SWPS_PUSH_ADAGRAD && cfg->push_rule != SWPS_PUSH_SGD)
    return fail(SWPS_E_UNSUPPORTED, "push rule " + std::to_string(cfg->push_rule) +
                                        ": the library implements SWPS_PUSH_ADAGRAD and SWPS_PUSH_SGD only");
  if (cfg->init_mode != SWPS_INIT_ZERO && cfg->init_mode != SWPS_INIT_HASH && cfg->init_mode != SWPS_INIT_FLCG)
    return fail(SWPS_E_UNSUPPORTED, "init mode " + std::to_string(cfg->init_mode) +
                                        ": the library implements SWPS_INIT_ZERO, SWPS_INIT_HASH and SWPS_INIT_FLCG");
  if (cfg->init_mode == SWPS_INIT_FLCG && cfg->layout != SWPS_LAYOUT_LR)
    return fail(SWPS_E_UNSUPPORTED, "SWPS_INIT_FLCG (LR's gen_float init) needs SWPS_LAYOUT_LR");
  SWPS_HIP(hipSetDevice(cfg->device));
  swps_table *t = new swps_table();
  t->cfg = *cfg;
  if (const char *e = getenv("SWPS_SLICE_PUSH")) t->slice_push = atoi(e) != 0;  // A/B timing, tests
  if (const char *e = getenv("SWPS_PUSH_DISTINCT")) t->distinct_push = atoi(e) != 0;  // A/B: the multi-source path
  if (t->cfg.fudge == 0.0f) t->cfg.fudge = 1e-6f;
  t->esize = cfg->dtype == SWPS_F64 ? 8 : 4;
  if (cfg->layout == SWPS_LAYOUT_W2V) {
    t->row_elems = 4 * cfg->dim;
    t->pull_elems = 2 * cfg->dim;
    t->push_elems = 2 * cfg->dim;
  } else {
    t->row_elems = 2;
    t->pull_elems = 1;
    t->push_elems = 1;
    t->cfg.dim = 1;
  }
  uint64_t ns = 1;
  while (ns < 2 * cfg->capacity) ns <<= 1;
  t->nslots = ns;
  t->mask = ns - 1;
  int rc = SWPS_OK;
  // the shard's stream (every app context's compute stream) at the highest priority, so helper streams
  // (the overlapped prep, RCCL exchanges) yield CUs to it (SWPS_TABLE_PRIO=0: default priority, A/B)
  int plo = 0, phi = 0;
  const char *pe = getenv("SWPS_TABLE_PRIO");
  if (hipDeviceGetStreamPriorityRange(&plo, &phi) != hipSuccess) plo = phi = 0;
  if (pe && atoi(pe) == 0) phi = 0;
  if (hipStreamCreateWithPriority(&t->stream, hipStreamNonBlocking, phi) != hipSuccess) rc = fail(SWPS_E_HIP, "stream");
  if (!rc) rc = t->keys.ensure(ns * 8);
  if (!rc) rc = t->slot_row.ensure(ns * 4);
  if (!rc) rc = t->row_key.ensure(cfg->capacity * 8);
  if (!rc) rc = t->rows.ensure(cfg->capacity * (uint64_t)t->row_elems * t->esize);
  if (!rc) rc = t->counters.ensure(16);
  if (!rc) rc = t->flcg.ensure(16);
  if (!rc) {  // the float LCG's state before the first draw (random.h:39-40: ULONG_MAX / 2)
    const uint64_t st[2] = {cfg->seed ? cfg->seed : ~0ULL / 2, 0};
    if (hipMemcpy(t->flcg.p, st, 16, hipMemcpyHostToDevice) != hipSuccess) rc = fail(SWPS_E_HIP, "memcpy");
  }
  if (!rc && hipMemsetAsync(t->keys.p, 0xFF, ns * 8, t->stream) != hipSuccess) rc = fail(SWPS_E_HIP, "memset");
  if (!rc && hipMemsetAsync(t->slot_row.p, 0xFF, ns * 4, t->stream) != hipSuccess) rc = fail(SWPS_E_HIP, "memset");
  if (!rc && hipMemsetAsync(t->counters.p, 0, 16, t->stream) != hipSuccess) rc = fail(SWPS_E_HIP, "memset");
  if (!rc && hipStreamSynchronize(t->stream) != hipSuccess) rc = fail(SWPS_E_HIP, "sync");
  if (rc) {
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
    return rc;
  }
  *out = t;
  return SWPS_OK;
}

int swps_table_destroy(swps_table *t) {
  if (!t) return SWPS_OK;
  (void)hipSetDevice(t->cfg.device);
  if (t->stream) {
    (void)hipStreamSynchronize(t->stream);
    (void)hipStreamDestroy(t->stream);
  }
  delete t;
  (void)hipGetLastError();  // leave no sticky error from the calls above
  return SWPS_OK;
}

int swps_table_sync(swps_table *t) {
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_HIP(hipDeviceSynchronize());  // async calls may have used caller streams
  return table_check_error(t, t->stream);
}

int swps_table_size(swps_table *t, uint64_t *n) {
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_TRY(table_check_error(t, t->stream));
  *n = t->host_nrows;
  return SWPS_OK;
}

int swps_table_row_elems(swps_table *t, int32_t *row, int32_t *pull, int32_t *push) {
  if (row) *row = t->row_elems;
  if (pull) *pull = t->pull_elems;
  if (push) *push = t->push_elems;
  return SWPS_OK;
}

int swps_pull_async(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_vals, void *stream) {
  hipStream_t s = stream ? (hipStream_t)stream : t->stream;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  if (t->comm) return routed_pull(t, d_keys, n, d_vals, s);
  if (n == 0) return SWPS_OK;
  SWPS_TRY(t->scratch.ensure(n * 4));
  uint32_t *rows = t->scratch.as<uint32_t>();
  SWPS_TRY(find_or_insert_async(t, d_keys, n, rows, s));
  return table_copy_pull(t, rows, n, d_vals, s);
}

int swps_push_async(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_grads, void *stream) {
  hipStream_t s = stream ? (hipStream_t)stream : t->stream;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  if (t->comm) return routed_push(t, d_keys, n, d_grads, s);
  if (n == 0) return SWPS_OK;
  SWPS_TRY(t->scratch.ensure(n * 4));
  uint32_t *rows = t->scratch.as<uint32_t>();
  SWPS_TRY(table_lookup(t, d_keys, n, rows, s));
  return table_push_rows(t, rows, n, d_grads, s);
}

int swps_pull(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_vals) {
  if (n == 0 && !t->comm) return SWPS_OK;
  SWPS_TRY(swps_pull_async(t, d_keys, n, d_vals, nullptr));
  return table_check_error(t, t->stream);
}

int swps_push(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_grads) {
  if (n == 0 && !t->comm) return SWPS_OK;
  SWPS_TRY(swps_push_async(t, d_keys, n, d_grads, nullptr));
  return table_check_error(t, t->stream);
}

int swps_assign(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_rows) {
  if (n == 0) return SWPS_OK;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_TRY(t->scratch.ensure(n * 4));
  uint32_t *rows = t->scratch.as<uint32_t>();
  // ClusterServer::load / an assignment never runs init_param (server.h:49-62): the new rows are
  // written whole below, and an SWPS_INIT_FLCG table's float-LCG stream does not move
  SWPS_TRY(table_find_or_insert(t, d_keys, n, rows, t->stream, false));
  SWPS_TRY(table_set_rows(t, rows, n, d_rows, t->stream));
  SWPS_HIP(hipStreamSynchronize(t->stream));
  return SWPS_OK;
}

int swps_export(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_rows) {
  if (n == 0) return SWPS_OK;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_TRY(t->scratch.ensure(n * 4));
  uint32_t *rows = t->scratch.as<uint32_t>();
  SWPS_TRY(table_lookup(t, d_keys, n, rows, t->stream));
  SWPS_TRY(table_get_rows(t, rows, n, d_rows, t->stream));
  return table_check_error(t, t->stream);
}

// Host-pointer forms for FFI callers without device memory: the reference's
// wire types (W2V fp64 [h|v] / [h_grad|v_grad], LR fp32), staged through HBM.
int swps_pull_h(swps_table *t, const uint64_t *keys, uint64_t n, void *vals) {
  if (n == 0 && !t->comm) return SWPS_OK;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  const int P = t->pull_elems;
  DevMem dk, dv;
  SWPS_TRY(dk.ensure(n * 8));
  SWPS_TRY(dv.ensure(n * P * t->esize));
  SWPS_HIP(hipMemcpyAsync(dk.p, keys, n * 8, hipMemcpyHostToDevice, t->stream));
  SWPS_TRY(swps_pull(t, dk.as<uint64_t>(), n, dv.p));  // syncs
  const bool w2v = t->cfg.layout == SWPS_LAYOUT_W2V;
  const size_t out_es = w2v ? 8 : 4;
  if (t->esize == out_es) {
    SWPS_HIP(hipMemcpy(vals, dv.p, n * P * out_es, hipMemcpyDeviceToHost));
    return SWPS_OK;
  }
  std::vector<char> tmp(n * P * t->esize);
  SWPS_HIP(hipMemcpy(tmp.data(), dv.p, tmp.size(), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < n * P; i++) {
    const double x = t->esize == 8 ? ((double *)tmp.data())[i] : (double)((float *)tmp.data())[i];
    if (w2v)
      ((double *)vals)[i] = x;
    else
      ((float *)vals)[i] = (float)x;
  }
  return SWPS_OK;
}

// SparseTableShard::find (sparsetable.h:28-37) for a batch of host keys: present[i] = 1 when the
// local shard holds keys[i].  Local tables only (a routed table's keys live on their owners).
int swps_table_find_h(swps_table *t, const uint64_t *keys, uint64_t n, uint8_t *present) {
  if (!t || (n && (!keys || !present))) return fail(SWPS_E_CFG, "null argument");
  if (t->comm) return fail(SWPS_E_UNSUPPORTED, "swps_table_find_h on a routed table");
  if (n == 0) return SWPS_OK;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  DevMem dk, dr;
  SWPS_TRY(dk.ensure(n * 8));
  SWPS_TRY(dr.ensure(n * 4));
  SWPS_HIP(hipMemcpyAsync(dk.p, keys, n * 8, hipMemcpyHostToDevice, t->stream));
  SWPS_TRY(table_probe(t, dk.as<uint64_t>(), n, dr.as<uint32_t>(), t->stream));
  std::vector<uint32_t> rows(n);
  SWPS_HIP(hipMemcpyAsync(rows.data(), dr.p, n * 4, hipMemcpyDeviceToHost, t->stream));
  SWPS_HIP(hipStreamSynchronize(t->stream));
  for (uint64_t i = 0; i < n; i++) present[i] = rows[i] != kNoRow ? 1 : 0;
  return SWPS_OK;
}

// swps_assign with host rows in the reference's value type (fp64, [n][row elems]), converted to
// the table dtype: SparseTableShard::assign (sparsetable.h:38-48) of whole rows, nothing drawn
int swps_assign_h(swps_table *t, const uint64_t *keys, uint64_t n, const double *rows) {
  if (!t || (n && (!keys || !rows))) return fail(SWPS_E_CFG, "null argument");
  if (t->comm) return fail(SWPS_E_UNSUPPORTED, "swps_assign_h on a routed table");
  if (n == 0) return SWPS_OK;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  const uint64_t m = n * (uint64_t)t->row_elems;
  DevMem dk, dv;
  SWPS_TRY(dk.ensure(n * 8));
  SWPS_TRY(dv.ensure(m * t->esize));
  SWPS_HIP(hipMemcpyAsync(dk.p, keys, n * 8, hipMemcpyHostToDevice, t->stream));
  if (t->esize == 8) {
    SWPS_HIP(hipMemcpyAsync(dv.p, rows, m * 8, hipMemcpyHostToDevice, t->stream));
    SWPS_HIP(hipStreamSynchronize(t->stream));
  } else {
    std::vector<float> f(rows, rows + m);
    SWPS_HIP(hipMemcpyAsync(dv.p, f.data(), m * 4, hipMemcpyHostToDevice, t->stream));
    SWPS_HIP(hipStreamSynchronize(t->stream));
  }
  return swps_assign(t, dk.as<uint64_t>(), n, dv.p);  // syncs before dk / dv go out of scope
}

int swps_push_h(swps_table *t, const uint64_t *keys, uint64_t n, const void *grads) {
  if (n == 0 && !t->comm) return SWPS_OK;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  const size_t gb = n * t->push_elems * (t->cfg.layout == SWPS_LAYOUT_W2V ? 8 : 4);
  DevMem dk, dg;
  SWPS_TRY(dk.ensure(n * 8));
  SWPS_TRY(dg.ensure(gb));
  SWPS_HIP(hipMemcpyAsync(dk.p, keys, n * 8, hipMemcpyHostToDevice, t->stream));
  SWPS_HIP(hipMemcpyAsync(dg.p, grads, gb, hipMemcpyHostToDevice, t->stream));
  return swps_push(t, dk.as<uint64_t>(), n, dg.p);  // syncs via the error check
}

int swps_table_keys(swps_table *t, uint64_t *keys, uint64_t cap, uint64_t *n) {
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_TRY(table_check_error(t, t->stream));
  uint64_t m = t->host_nrows;
  *n = m;
  if (cap < m) return fail(SWPS_E_CFG, "key buffer too small");
  if (m) SWPS_HIP(hipMemcpy(keys, t->row_key.p, m * 8, hipMemcpyDeviceToHost));
  return SWPS_OK;
}

// SparseTable::output (sparsetable.h:127-132) with WParam / LRParam's
// operator<< (word2vec_global.h:102-112, lr.cpp:24-27): ostream precision 6.
int swps_dump(swps_table *t, const char *path) {
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_TRY(table_check_error(t, t->stream));
  uint64_t m = t->host_nrows;
  std::vector<uint64_t> keys(m);
  std::vector<char> rows(m * t->row_elems * t->esize);
  if (m) {
    SWPS_HIP(hipMemcpy(keys.data(), t->row_key.p, m * 8, hipMemcpyDeviceToHost));
    SWPS_HIP(hipMemcpy(rows.data(), t->rows.p, rows.size(), hipMemcpyDeviceToHost));
  }
  FILE *f = fopen(path, "w");
  if (!f) return fail(SWPS_E_IO, std::string("cannot write ") + path);
  auto val = [&](uint64_t r, int e) -> double {
    size_t off = r * t->row_elems + e;
    return t->esize == 8 ? ((double *)rows.data())[off] : (double)((float *)rows.data())[off];
  };
  const int D = t->cfg.dim;
  for (uint64_t r = 0; r < m; r++) {
    fprintf(f, "%llu\t", (unsigned long long)keys[r]);
    if (t->cfg.layout == SWPS_LAYOUT_W2V) {
      for (int i = 0; i < D; i++) fprintf(f, i < D - 1 ? "%g " : "%g\t", val(r, D + i));
      for (int i = 0; i < D; i++) fprintf(f, i < D - 1 ? "%g " : "%g\n", val(r, i));
    } else {
      fprintf(f, "%g\n", val(r, 0));
    }
  }
  fclose(f);
  return SWPS_OK;
}

// ClusterServer::load (server.h:49-62): keep keys whose hash-frag node is
// `node_id`; h2/v2 (grad2sum) start at 0.
int swps_load(swps_table *t, const char *path, int32_t frag_num, int32_t world, int32_t node_id) {
  SWPS_HIP(hipSetDevice(t->cfg.device));
  std::ifstream f(path);
  if (!f) return fail(SWPS_E_IO, std::string("cannot open ") + path);
  std::vector<uint32_t> map;
  bool filter = world > 1 && node_id > 0;
  if (filter) {
    map.resize(frag_num);
    SWPS_TRY(swps_hashfrag_table(frag_num, world, map.data()));
  }
  const int D = t->cfg.dim, R = t->row_elems;
  std::vector<uint64_t> keys;
  std::vector<double> vals;
  std::string line;
  while (std::getline(f, line)) {
    if (line.empty()) continue;
    std::istringstream is(line);
    uint64_t key;
    if (!(is >> key)) return fail(SWPS_E_IO, "bad parameter line");
    std::vector<double> row(R, 0.0);
    if (t->cfg.layout == SWPS_LAYOUT_W2V) {
      for (int i = 0; i < D; i++) is >> row[D + i];  // v first (word2vec_global.h:113-121)
      for (int i = 0; i < D; i++) is >> row[i];
    } else {
      is >> row[0];
    }
    if (!is) return fail(SWPS_E_IO, "truncated parameter line");
    if (filter && (int)map[fmix64(key) % (uint64_t)frag_num] != node_id) continue;
    keys.push_back(key);
    vals.insert(vals.end(), row.begin(), row.end());
  }
  uint64_t n = keys.size();
  if (!n) return SWPS_OK;
  DevMem dk, dv;
  SWPS_TRY(upload(dk, keys, t->stream));
  if (t->esize == 8) {
    SWPS_TRY(upload(dv, vals, t->stream));
  } else {
    std::vector<float> fv(vals.begin(), vals.end());
    SWPS_TRY(upload(dv, fv, t->stream));
    SWPS_HIP(hipStreamSynchronize(t->stream));
  }
  SWPS_TRY(swps_assign(t, dk.as<uint64_t>(), n, dv.p));
  return SWPS_OK;
}

// ---- binary snapshots -------------------------------------------------------
// The reference can only dump values as text at 6 significant digits and
// without the AdaGrad sums (sparsetable.h:63-70): a resumed run
// diverges.  swps_save writes every row element bit for bit:
//   "SWPSTBL2" | u32 layout | u32 dtype | i32 dim | u32 row_elems |
//   f32 learning_rate | f32 fudge (the push rule's constants: a resume with
//   another server learning rate is not the same run) | u64 n |
//   keys u64[n] | rows [n][row_elems] (table dtype) | u64 checksum
// The checksum is kept in swps_table::snap_sum; swps_w2v_save_state records
// it, so a worker state resumes only against the table file of the same save.
static const char kTableMagic[8] = {'S', 'W', 'P', 'S', 'T', 'B', 'L', '2'};

int swps_save(swps_table *t, const char *path) {
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_TRY(table_check_error(t, t->stream));
  const uint64_t m = t->host_nrows;
  std::vector<uint64_t> keys(m);
  std::vector<char> rows(m * t->row_elems * t->esize);
  if (m) {
    SWPS_HIP(hipMemcpy(keys.data(), t->row_key.p, m * 8, hipMemcpyDeviceToHost));
    SWPS_HIP(hipMemcpy(rows.data(), t->rows.p, rows.size(), hipMemcpyDeviceToHost));
  }
  SnapFile f;
  SWPS_TRY(f.open(path, true));
  const uint32_t hdr[6] = {(uint32_t)t->cfg.layout, (uint32_t)t->cfg.dtype, (uint32_t)t->cfg.dim,
                           (uint32_t)t->row_elems, __float_as_uint_host(t->cfg.learning_rate),
                           __float_as_uint_host(t->cfg.fudge)};
  SWPS_TRY(f.put(kTableMagic, 8));
  SWPS_TRY(f.put(hdr, sizeof(hdr)));
  SWPS_TRY(f.put(&m, 8));
  SWPS_TRY(f.put(keys.data(), m * 8));
  SWPS_TRY(f.put(rows.data(), rows.size()));
  const uint64_t sum = f.sum;
  SWPS_TRY(f.finish_write());
  t->snap_sum = sum;
  return SWPS_OK;
}

// Read and verify the whole file before touching the table; then assign the
// rows (all of them, or those BasicHashFrag gives node_id, as swps_load).
int swps_restore(swps_table *t, const char *path, int32_t frag_num, int32_t world, int32_t node_id) {
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SnapFile f;
  SWPS_TRY(f.open(path, false));
  char magic[8];
  uint32_t hdr[6];
  uint64_t m = 0;
  if (f.get(magic, 8) != SWPS_OK || memcmp(magic, kTableMagic, 7) != 0)
    return fail(SWPS_E_IO, std::string("not a swps table snapshot: ") + path);
  if (magic[7] != kTableMagic[7])
    return fail(SWPS_E_IO, std::string("table snapshot format version ") + magic[7] + " (this library reads " +
                               kTableMagic[7] + "): " + path);
  SWPS_TRY(f.get(hdr, sizeof(hdr)));
  if (hdr[4] != __float_as_uint_host(t->cfg.learning_rate) || hdr[5] != __float_as_uint_host(t->cfg.fudge))
    return fail(SWPS_E_CFG, std::string("snapshot was taken with another push rule (server learning rate / AdaGrad "
                                        "fudge) than this table's: ") + path);
  if (hdr[0] != (uint32_t)t->cfg.layout || hdr[1] != (uint32_t)t->cfg.dtype || hdr[2] != (uint32_t)t->cfg.dim ||
      hdr[3] != (uint32_t)t->row_elems)
    return fail(SWPS_E_CFG, "snapshot (layout " + std::to_string(hdr[0]) + ", dtype " + std::to_string(hdr[1]) +
                                ", dim " + std::to_string(hdr[2]) + ") does not match the table (layout " +
                                std::to_string(t->cfg.layout) + ", dtype " + std::to_string(t->cfg.dtype) +
                                ", dim " + std::to_string(t->cfg.dim) + ")");
  SWPS_TRY(f.get(&m, 8));
  const size_t rb = (size_t)t->row_elems * t->esize;
  if (m > (1ULL << 40) / std::max<size_t>(rb, 1)) return fail(SWPS_E_IO, std::string("corrupt snapshot header: ") + path);
  std::vector<uint64_t> keys(m);
  std::vector<char> rows(m * rb);
  SWPS_TRY(f.get(keys.data(), m * 8));
  SWPS_TRY(f.get(rows.data(), rows.size()));
  const uint64_t sum = f.sum;
  SWPS_TRY(f.finish_read());
  t->snap_sum = sum;
  if (world > 1 && node_id > 0) {
    std::vector<uint32_t> map(frag_num);
    SWPS_TRY(swps_hashfrag_table(frag_num, world, map.data()));
    uint64_t k = 0;
    for (uint64_t i = 0; i < m; i++) {
      if ((int)map[fmix64(keys[i]) % (uint64_t)frag_num] != node_id) continue;
      if (k != i) {
        keys[k] = keys[i];
        memcpy(rows.data() + k * rb, rows.data() + i * rb, rb);
      }
      k++;
    }
    m = k;
  }
  if (!m) return SWPS_OK;
  if (m > t->cfg.capacity)  // keys new to a partly filled table are caught by the insert
    return fail(SWPS_E_OOM, "snapshot holds " + std::to_string(m) + " rows; table capacity is " +
                                std::to_string(t->cfg.capacity));
  DevMem dk, dv;
  SWPS_TRY(upload(dk, keys, t->stream));
  SWPS_TRY(upload(dv, rows, t->stream));
  return swps_assign(t, dk.as<uint64_t>(), m, dv.p);  // syncs before dk/dv go out of scope
}

}  // extern "C"
