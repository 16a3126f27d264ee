// Internal definitions shared by the libswps translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <memory>
#include <vector>

#include "swps.h"

namespace swps {

// ---- errors (thread-local message, negative codes; never abort) -----------
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define SWPS_HIP(call)                                                                            \
  do {                                                                                            \
    hipError_t e_ = (call);                                                                       \
    if (e_ != hipSuccess) return ::swps::fail(SWPS_E_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define SWPS_TRY(call)          \
  do {                          \
    int rc_ = (call);           \
    if (rc_ != SWPS_OK) return rc_; \
  } while (0)

// ---- device buffer ----------------------------------------------------------
struct DevMem {
  void *p = nullptr;
  size_t bytes = 0;
  DevMem() = default;
  DevMem(const DevMem &) = delete;
  DevMem &operator=(const DevMem &) = delete;
  ~DevMem() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  // grow-only, with 1/8 headroom so per-batch sizes that wander a little
  // (kept positions differ per epoch) do not reallocate — a hipFree is a
  // device-wide sync and a fresh hipMalloc maps pages; contents not preserved
  int ensure(size_t b) {
    if (b <= bytes && p) return SWPS_OK;
    release();
    size_t nb = b ? b + b / 8 : 16;
    if (hipMalloc(&p, nb) != hipSuccess) {
      (void)hipGetLastError();
      return fail(SWPS_E_OOM, "hipMalloc of " + std::to_string(nb) + " bytes failed");
    }
    bytes = nb;
    return SWPS_OK;
  }
  template <typename T> T *as() const { return reinterpret_cast<T *>(p); }
};

template <typename T> int upload(DevMem &m, const std::vector<T> &v, hipStream_t s) {
  SWPS_TRY(m.ensure(v.size() * sizeof(T)));
  if (!v.empty()) SWPS_HIP(hipMemcpyAsync(m.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
  return SWPS_OK;
}

// host staging buffers of a host-transport exchange
struct HostStage {
  std::vector<char> send, recv;
};

// ---- hashing / RNG (host + device) ----------------------------------------
__host__ __device__ inline uint64_t fmix64(uint64_t x) {  // utils/HashFunction.h:16-24
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

// Affine LCG x -> a*x + c (mod 2^64) advanced k steps by doubling.
// Main stream: a = 25214903917, c = 11; float stream: a = 4903917, c = 11
// (utils/random.h:29-36).
constexpr uint64_t kLcgA = 25214903917ULL;
constexpr uint64_t kFlcgA = 4903917ULL;
constexpr uint64_t kLcgC = 11ULL;

__host__ __device__ inline uint64_t lcg_jump(uint64_t x, uint64_t k, uint64_t a, uint64_t c) {
  uint64_t acc_a = 1, acc_c = 0, cur_a = a, cur_c = c;
  while (k) {
    if (k & 1) {
      acc_a = acc_a * cur_a;
      acc_c = acc_c * cur_a + cur_c;
    }
    cur_c = (cur_a + 1) * cur_c;
    cur_a = cur_a * cur_a;
    k >>= 1;
  }
  return acc_a * x + acc_c;
}

// gen_float of the float LCG state AFTER the step (random.h:33-36)
__host__ __device__ inline float flcg_value(uint64_t y) {
  return (float)y / 18446744073709551616.0f;
}

inline uint32_t __float_as_uint_host(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

// ---- host utilities (swps_host.cpp) -----------------------------------------
uint64_t bkdr(const char *s);
uint64_t checksum64(uint64_t h, const void *p, size_t n);
// binary snapshot files (swps_save / swps_w2v_save_state): every payload byte
// goes through a running 64-bit checksum, stored after the payload; short
// reads/writes and checksum mismatches fail with SWPS_E_IO
struct SnapFile {
  FILE *f = nullptr;
  uint64_t sum = 0x5357505353554dULL;
  std::string path, tmp;
  bool writing = false, committed = false;
  SnapFile() = default;
  SnapFile(const SnapFile &) = delete;
  SnapFile &operator=(const SnapFile &) = delete;
  ~SnapFile();
  int open(const std::string &p, bool write);
  int put(const void *p, size_t n);
  int get(void *p, size_t n);
  int finish_write();  // trailing checksum, fsync, atomic rename over path
  int finish_read();   // compare the trailing checksum
};
// glibc random_r TYPE_3 (the generator behind rand()): r[i] = r[i-3] + r[i-31]
struct GlibcRand {
  int32_t r[34];
  int idx = 0;
  uint64_t produced = 0;
  explicit GlibcRand(uint32_t seed);
  int32_t next();
  // k calls of next() whose outputs nobody reads: a jump of the linear recurrence (x^k mod
  // x^31 - x^28 - 1 by square-and-multiply) for long skips, stepping for short ones
  void discard(uint64_t k);
};
// Host open-addressed u64 -> int32 map (linear probing on fmix64, power-of-two capacity, a
// generation stamp per slot so clear() is O(1)): the host schedules' per-token counting, where
// std::unordered_map's node allocations dominated.  Iteration order is not exposed; callers that
// need the reference's std::unordered_set order keep one of those beside it.
struct FlatMap64 {
  std::vector<uint64_t> k;
  std::vector<int32_t> v;
  std::vector<uint32_t> st;
  uint32_t gen = 1;
  uint64_t mask = 0;
  size_t n = 0;
  explicit FlatMap64(size_t cap = 16) { reset(cap); }
  void reset(size_t cap) {
    size_t c = 16;
    while (c < 2 * cap) c <<= 1;
    k.assign(c, 0);
    v.assign(c, 0);
    st.assign(c, 0);
    mask = c - 1;
    n = 0;
    gen = 1;
  }
  void clear() {
    if (++gen == 0) {
      std::fill(st.begin(), st.end(), 0u);
      gen = 1;
    }
    n = 0;
  }
  size_t size() const { return n; }
  // the value slot of key (0 when inserted); *fresh = inserted by this call
  int32_t &at(uint64_t key, bool *fresh = nullptr) {
    if (2 * (n + 1) > mask + 1) grow();
    uint64_t i = fmix64(key) & mask;
    while (st[i] == gen) {
      if (k[i] == key) {
        if (fresh) *fresh = false;
        return v[i];
      }
      i = (i + 1) & mask;
    }
    st[i] = gen;
    k[i] = key;
    v[i] = 0;
    n++;
    if (fresh) *fresh = true;
    return v[i];
  }
  bool contains(uint64_t key) const {
    uint64_t i = fmix64(key) & mask;
    while (st[i] == gen) {
      if (k[i] == key) return true;
      i = (i + 1) & mask;
    }
    return false;
  }
  void grow() {
    std::vector<uint64_t> ok;
    std::vector<int32_t> ov;
    ok.reserve(n);
    ov.reserve(n);
    for (size_t i = 0; i <= mask; i++)
      if (st[i] == gen) {
        ok.push_back(k[i]);
        ov.push_back(v[i]);
      }
    reset(2 * (mask + 1));
    for (size_t i = 0; i < ok.size(); i++) at(ok[i]) = ov[i];
  }
};
// reference config file format (utils/ConfigParser.h:84-115)
struct Config {
  std::vector<std::pair<std::string, std::vector<std::pair<std::string, std::string>>>> sections;
  int parse(const std::string &path);
  bool get(const std::string &sec, const std::string &key, std::string &out) const;
};

}  // namespace swps

// ---- the HBM parameter shard -------------------------------------------------
struct swps_table {
  swps_table_cfg cfg{};
  int row_elems = 0, pull_elems = 0, push_elems = 0;
  size_t esize = 4;
  uint64_t nslots = 0, mask = 0;
  hipStream_t stream = nullptr;
  swps::DevMem keys;      // [nslots] u64, EMPTY = ~0 (sparsetable.h:25 empty key)
  swps::DevMem slot_row;  // [nslots] u32 dense row index
  swps::DevMem row_key;   // [capacity] u64
  swps::DevMem rows;      // [capacity][row_elems] T
  swps::DevMem counters;  // [0] = nrows (u32), [1] = error flag
  swps::DevMem scratch;   // per-call row indices
  uint32_t host_nrows = 0;
  swps::DevMem push_scratch, sort_tmp;  // table_push_sources: (row, position) pairs and their sort
  bool distinct_push = true;  // table_push_sources: one source skips the grouping sort (SWPS_PUSH_DISTINCT=0: off)
  bool slice_push = true;  // table_push_sources: k_push_w2v_multi_t for fp32 D = 256k + t (SWPS_SLICE_PUSH=0: off)
  uint64_t snap_sum = 0;  // checksum of the snapshot last saved from / restored into this table (0: none);
                          // worker-state snapshots record it so a resume pairs the two files of one save
  swps::DevMem isnew;     // find_or_insert: per-key "inserted by this call" flags
  swps::DevMem flcg;      // SWPS_INIT_FLCG: [float-LCG state, draws of the current call] (u64 x 2)
  swps::DevMem flcg_blk;  // SWPS_INIT_FLCG: per-block new-key counts -> offsets
  // key-sharded mode (swps_table_route, swps_comm.hip)
  swps_comm *comm = nullptr;
  int32_t frag_num = 0;
  swps::DevMem frag_map;  // u32[frag_num]: frag -> node id (1..world)
  swps::DevMem r_owner, r_pos, r_owner_s, r_perm, r_keys, r_buf, r_rkeys, r_rbuf, r_rows, r_tmp, r_cnt;
  swps::HostStage stage;  // host staging (host transport)
  uint64_t rstats[6] = {0, 0, 0, 0, 0, 0};
  bool finished = false;
};

namespace swps {
constexpr uint64_t kEmptyKey = ~0ULL;
constexpr uint32_t kNoRow = 0xFFFFFFFFu;
// table internals used by the app contexts (same library)
// init = false: no init_param for the new keys (their rows are about to be assigned whole; an
// SWPS_INIT_FLCG table draws nothing)
int table_find_or_insert(swps_table *t, const uint64_t *d_keys, uint64_t n, uint32_t *d_rows_out, hipStream_t s,
                         bool init = true);
int table_find_or_insert_placed(swps_table *t, const uint64_t *d_keys, uint64_t n, const uint32_t *place,
                                uint32_t *d_rows_out, hipStream_t s);
int table_lookup(swps_table *t, const uint64_t *d_keys, uint64_t n, uint32_t *d_rows_out, hipStream_t s);
int table_probe(swps_table *t, const uint64_t *d_keys, uint64_t n, uint32_t *d_rows_out, hipStream_t s);
int table_check_error(swps_table *t, hipStream_t s);
int table_set_rows(swps_table *t, const uint32_t *d_rows, uint64_t n, const void *d_vals, hipStream_t s);
int table_get_rows(swps_table *t, const uint32_t *d_rows, uint64_t n, void *d_vals, hipStream_t s);
int table_copy_pull(swps_table *t, const uint32_t *d_rows, uint64_t n, void *d_vals, hipStream_t s);
int table_push_rows(swps_table *t, const uint32_t *d_rows, uint64_t n, const void *d_grads, hipStream_t s,
                    bool grads_f32 = false);
// several sources' pushes concatenated in rank order (keys distinct within a
// source): each row gets its sources' AdaGrad steps in that order, one pass
// distinct: one source (no row repeats): no grouping sort
// sort_cache / sort_valid: the grouping sort's output for these same rows, kept across calls (a
// static per-step key set): reused when *sort_valid, else computed, stored and *sort_valid set
int table_push_sources(swps_table *t, const uint32_t *d_rows, uint64_t n, const void *d_grads, hipStream_t s,
                       bool grads_f32 = false, bool distinct = false, swps::DevMem *sort_cache = nullptr,
                       bool *sort_valid = nullptr);
// latched device error flags (table full, unknown key) -> error code, no sync
int table_error_code(uint32_t flags);
// key-sharded pull / push (swps_comm.hip): collective over t->comm
int routed_pull(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_vals, hipStream_t s);
int routed_push(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_grads, hipStream_t s);
// app contexts take AdaGrad shards only
int check_app_table(swps_table *t);
// communicator exchanges (swps_comm.hip), ordered on stream s
int comm_allgather(swps_comm *c, const void *in, void *out, uint64_t bytes, hipStream_t s);
// dst rows pos[i] = src rows i (row_bytes each, a multiple of 4), ordered on s
int scatter_rows(const void *src, const uint32_t *pos, uint64_t n, uint64_t row_bytes, void *dst, hipStream_t s);
// phase: what the exchange carries, named by the RCCL deadline guard when it does not retire
int comm_alltoallv(swps_comm *c, const void *d_send, const std::vector<uint64_t> &sb, void *d_recv,
                   const std::vector<uint64_t> &rb, hipStream_t s, HostStage &stg,
                   const char *phase = "all-to-all-v");
int comm_alltoallv_disp(swps_comm *c, const void *d_send, const std::vector<uint64_t> &sb,
                        const std::vector<uint64_t> &so, void *d_recv, const std::vector<uint64_t> &rb,
                        const std::vector<uint64_t> &ro, hipStream_t s, HostStage &stg,
                        const char *phase = "all-to-all-v");
// SWPS_OK, or SWPS_E_RCCL with the guard's message once the communicator was aborted
int comm_status(swps_comm *c);
int comm_rank(const swps_comm *c);
int comm_world(const swps_comm *c);
int comm_device(const swps_comm *c);
bool comm_is_rccl(const swps_comm *c);

// ---- library-driven sharded app loop (swps_driver.cpp) ---------------------
// An app context's sharded-mode entry points (swps_<app>_request /
// serve_pull / step / serve_push ...) and payload widths.
struct AppOps {
  void *h = nullptr;
  hipStream_t cs = nullptr;  // the app's compute stream
  uint64_t width = 0, val_bytes = 0, grad_bytes = 0;
  int (*batch_counts)(void *, uint64_t *, uint64_t, uint64_t *) = nullptr;
  int (*request)(void *, int32_t, uint64_t *, uint64_t *, uint64_t *) = nullptr;
  int (*serve_pull)(void *, const uint64_t *, const uint64_t *, int32_t, void *) = nullptr;
  int (*install)(void *, const void *) = nullptr;
  // optional: at world 1 with the key cache, serve_pull(..., nullptr) only looks the slot's rows up
  // and the step's install reads them from the shard in place (no value copy)
  bool pull_in_place = false;
  int (*step)(void *, const void *, void *) = nullptr;
  int (*serve_push)(void *, const uint64_t *, const void *, const uint64_t *) = nullptr;
  int (*prep)(void *) = nullptr;                      // optional: the next step's param-free half
  int (*set_serve_stream)(void *, void *) = nullptr;  // optional: server work on the driver's stream
  // optional: the step slot (position in the epoch) the next serve_pull / serve_push belong to, -1 =
  // none; their received keys are the same every epoch, so the app may cache per-slot lookups
  int (*set_slot)(void *, int64_t) = nullptr;
  // optional: after step(), the event (hipEvent_t) recorded once the first half of every owner's
  // keys has its gradients (the rest follow in a second pass), or nullptr: one all-to-all
  void *(*half_event)(void *) = nullptr;
  // optional: d_flags[j] = 1 when the j-th of the n keys served at slot `cur` (set_slot ids) was
  // also served at slot `prev`, from the rows cached for both (0: no push of `prev` touches it)
  int (*late_mask)(void *, int64_t cur, int64_t prev, uint8_t *d_flags, uint64_t n) = nullptr;
  // optional: the next step() takes its pull values in two parts (value i of part q belongs to the
  // batch's key pos_q[i]) instead of one array in key order
  int (*install_parts)(void *, const void *, const uint32_t *, uint64_t, const void *, const uint32_t *,
                       uint64_t) = nullptr;
};

struct ShardDriver {
  AppOps ops;
  swps_comm *c = nullptr;
  int rank = 0, world = 1;
  uint64_t nb = 0, spe = 0, cursor = 0;  // own batches, steps per epoch (max over ranks), steps run
  std::vector<uint64_t> send, recv;      // [step][rank] key counts
  DevMem keys, rkeys, vals, myvals, grads, rgrads;  // per step, sized at setup for the largest step
  DevMem fp_keys, fp_rkeys, fp_vals, fp_myvals;      // the full pull's (whole local vocab)
  uint64_t step_keys = 0, step_rkeys = 0;
  // the keys each owner receives at a step are the same every epoch (static batch schedules): the
  // first epoch's key exchange fills rk_cache[slot], later epochs skip the request and the exchange
  DevMem rk_cache;
  std::vector<uint64_t> rk_off;  // [spe] element offsets into rk_cache
  std::vector<char> rk_valid;    // [spe]
  bool key_cache = false;
  bool split_grads = false;  // the gradient all-to-all in two halves (AppOps::half_event)
  // Early / late pulls (AppOps::late_mask; SWPS_SPLIT_PULL=0 off): of the keys an owner serves at
  // slot st, those that no rank pulled at slot st-1 receive no push at st-1, so push(st-1) cannot
  // change their rows: they are served and exchanged while step st-1 learns, and only the rest
  // waits for push(st-1).  Per slot, from its second epoch on (the key cache and both slots' row
  // lookups exist by then).  Same values in the same positions: bit-identical to lockstep.
  struct SplitSlot {
    bool ready = false;
    DevMem ek, lk;                // owner: the early / late keys, per source in rank order
    std::vector<uint64_t> es, ls;  // owner: early / late counts per source (what I send)
    std::vector<uint64_t> ed, ld;  // requester: early / late counts per owner (what I receive)
    DevMem pe, pl;                // requester: my values' positions (K order) of the early / late values
    uint64_t ne = 0, nl = 0;      // requester: totals
  };
  bool split_pull = false;
  std::vector<std::unique_ptr<SplitSlot>> sp;  // [spe]
  // requester: early values (received while the previous step learns; two buffers, since the
  // step may still be installing one slot's when the next slot's arrive), late values
  DevMem evals[2], lvals;
  int ebuf = 0;  // the buffer serve_early writes next
  bool early_pending = false;
  uint64_t early_slot = 0;
  int early_buf = 0;
  uint64_t split_steps = 0;  // steps whose pull was split (stats)
  int split_prepare(uint64_t st);
  int serve_early(uint64_t st);
  HostStage stage;
  hipStream_t S = nullptr;
  hipEvent_t ev_pull = nullptr, ev_learn = nullptr, ev_x0 = nullptr, ev_x1 = nullptr;
  bool xprof = false;  // exchange accounting: bytes and event-timed exchanges (syncs per exchange)
  uint64_t bytes_total = 0, bytes_remote = 0, calls = 0;
  double xms = 0;
  ~ShardDriver();
  int setup();
  int full_pull();
  int steps(uint64_t count);
  int sync();
  int exchange(const void *d_send, const uint64_t *sk, void *d_recv, const uint64_t *rk, uint64_t w, hipStream_t s,
               const char *phase = "all-to-all-v");
  int exchange_disp(const void *d_send, const std::vector<uint64_t> &sb, const std::vector<uint64_t> &so,
                    void *d_recv, const std::vector<uint64_t> &rb, const std::vector<uint64_t> &ro, hipStream_t s,
                    const char *phase = "all-to-all-v");
};
}  // namespace swps
