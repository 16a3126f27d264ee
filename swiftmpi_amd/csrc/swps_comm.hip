// Communicator and key-sharded table: the reference's src/transfer (ZeroMQ
// request/response, transfer.h:86-241), src/cluster (rank <-> server route,
// hashfrag.h:33-56) and the server's pull / push handlers (server.h:129-176)
// as owner-routed all-to-all exchanges, issued by the library itself:
//   RCCL (ncclSend / ncclRecv groups over xGMI, device buffers, on the
//   table's stream), or the caller's host callbacks (payloads staged
//   through host memory: several ranks on one GPU, CPU-side transports).
//
// One routed call = one "round":
//   1. owner of each key = BasicHashFrag node - 1 (k_owner); a stable radix
//      sort by owner groups the keys (position order kept inside a group);
//      per-owner counts come back to the host (the only sync of a round)
//   2. header all-gather {op, counts[world]} from every rank: each rank
//      learns what it receives and checks that all active ranks agree on the
//      op (a rank inside swps_finish contributes op FINISH and no keys)
//   3. all-to-all-v of keys (and, for a push, of the mean gradients)
//   4. owners: find-or-insert + pull values (pull) or lookup + the push rule
//      applied per source in rank order (push; table_push_sources)
//   5. pull: all-to-all-v of the values back, un-permuted to key order.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>

#include "swps_internal.h"
#include "swps_sort.h"

using namespace swps;

struct TcpStar;
// RCCL deadline guard.  A peer that dies or stops inside a collective leaves this rank's RCCL
// kernels spinning and its host blocked in a stream wait until some outer timeout kills the job.
// The guard bounds that: every collective is followed by an event on its stream, and a watchdog
// thread polls the oldest pending event and ncclCommGetAsyncError; when an exchange has not
// retired within the deadline (SWPS_COMM_TIMEOUT_S, default 120 s, or swps_comm_set_timeout), or
// RCCL reports an asynchronous error, it aborts the communicator (ncclCommAbort: the spinning
// kernels exit, so the blocked stream waits return) and latches a message naming the rank and the
// exchange; every later call on the communicator fails with SWPS_E_RCCL and that message.  The
// communicator is non-blocking (ncclConfig_t.blocking = 0), so its initialisation is polled
// against the same deadline instead of blocking in ncclCommInitRank.
struct CommGuard {
  struct Pending {
    hipEvent_t ev;
    const char *phase;
    std::chrono::steady_clock::time_point t0;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Pending> pending;
  std::vector<hipEvent_t> spare;
  std::thread th;
  bool stop = false;
  std::atomic<bool> aborted{false};
  std::string msg;  // set once, before `aborted`
};

// Device-initiated all-to-all-v (swps_comm_enable_ipc, opt-in; the ranks of one node).  Every rank
// owns an inbox (world sources x 2 parities x slot bytes) and a block of control words, both in
// uncached device memory, and maps every peer's pair through hipIpcOpenMemHandle.  One exchange is
// one kernel on the caller's stream (k_ipc_a2a): per (peer, channel) a send workgroup copies its
// part of the segment into the peer's inbox and bumps the peer's ready word; a receive workgroup
// waits for its ready word, copies the inbox out to the receive buffer and bumps the sender's ack
// word, which frees that parity for the sender's round after next.  Ready / ack words are
// monotonic round counts kept in step on both sides by the host (each side knows every segment's
// length: the collective's counts), so nothing is reset between exchanges and no handshake runs
// on the host.  Spins are bounded by the communicator's deadline: a rank whose peer never comes
// sets a local dead word (the rest of its workgroups stop) and a host-mapped error word, and the
// next call on the communicator fails with SWPS_E_RCCL.  Headers and counts still go through the
// communicator's own transport.
constexpr int kIpcMaxWorld = 8;   // one node
constexpr int kIpcCh = 8;         // channels (workgroups) per peer and direction
constexpr uint64_t kIpcMinPart = 4096;  // a segment is split over channels in parts of >= 4 KiB
constexpr int kIpcAck = kIpcMaxWorld * kIpcCh;  // control words: ready[src][ch], ack[dst][ch], dead
constexpr int kIpcDead = 2 * kIpcMaxWorld * kIpcCh;
constexpr uint64_t kIpcCtrlBytes = 4096;

struct IpcState {
  uint64_t slot = 0, sub = 0;  // per (source, parity) inbox slot; per channel sub-slot
  void *inbox = nullptr, *ctrl = nullptr;  // this rank's (uncached device memory)
  std::vector<void *> peer_inbox, peer_ctrl;  // every rank's, as mapped here (own: local)
  uint64_t *err_host = nullptr, *err_dev = nullptr;  // host-mapped error word
  std::vector<uint64_t> sc, rc;  // rounds sent to / received from [peer][channel] so far
  hipEvent_t last = nullptr;  // the previous exchange's kernel: exchanges run in issue order
  bool issued = false;
  uint64_t ticks_per_s = 0;
  uint64_t calls = 0, bytes_remote = 0;
};

struct swps_comm {
  int32_t rank = 0, world = 1, device = 0;
  bool rccl = false;
  ncclComm_t nc = nullptr;
  swps_transport tr{};
  TcpStar *tcp = nullptr;  // swps_comm_create_tcp's transport state (owned)
  DevMem d_hdr;  // RCCL header all-gather buffers
  double timeout_s = 120.0;  // RCCL deadline per exchange (CommGuard)
  std::unique_ptr<CommGuard> guard;  // RCCL, world > 1
  std::unique_ptr<IpcState> ipc;  // swps_comm_enable_ipc
  HostStage stage;  // swps_comm_alltoallv over a host transport
  // swps_comm_alltoallv called with the null stream on an RCCL communicator: the exchange runs on
  // this non-blocking stream instead, ordered after and before the null stream by two events (an
  // RCCL communicator never sees the null stream)
  hipStream_t nstream = nullptr;
  hipEvent_t nev_in = nullptr, nev_out = nullptr;
};

namespace {

enum { kOpPull = 0, kOpPush = 1, kOpFinish = 2 };

// a non-blocking communicator may answer ncclInProgress: the call is queued (comm_settle waits)
#define SWPS_NCCL(call)                                                                                   \
  do {                                                                                                    \
    ncclResult_t r_ = (call);                                                                             \
    if (r_ != ncclSuccess && r_ != ncclInProgress)                                                        \
      return ::swps::fail(SWPS_E_RCCL, std::string(#call) + ": " + ncclGetErrorString(r_));              \
  } while (0)

double seconds_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// abort the communicator once (watchdog or a host-side deadline) and latch the message
void comm_abort(swps_comm *c, const std::string &why) {
  CommGuard *g = c->guard.get();
  if (!g) return;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->aborted.load()) return;
    g->msg = "rank " + std::to_string(c->rank) + " of " + std::to_string(c->world) + ": " + why;
    g->aborted.store(true);
  }
  fprintf(stderr, "swps: %s; aborting the RCCL communicator\n", g->msg.c_str());
  fflush(stderr);
  (void)ncclCommAbort(c->nc);  // frees the communicator: never destroyed again
}

// the IPC exchange's error word: 0, or 1 << 63 | receive << 8 | peer of a wait that timed out, or
// 1 << 63 | 1 << 9: an exchange found the dead word set
std::string ipc_error(const swps_comm *c) {
  const IpcState *p = c->ipc.get();
  if (!p || !p->err_host) return "";
  const uint64_t e = __atomic_load_n(p->err_host, __ATOMIC_ACQUIRE);
  if (!e) return "";
  if ((e >> 9) & 1)
    return "rank " + std::to_string(c->rank) + " of " + std::to_string(c->world) +
           ": IPC exchange: a rank gave up on an earlier exchange (a peer rank lost or stuck)";
  return "rank " + std::to_string(c->rank) + " of " + std::to_string(c->world) + ": IPC exchange: no " +
         ((e >> 8) & 1 ? "data from" : "acknowledgement from") + " rank " + std::to_string(e & 0xff) +
         " within " + std::to_string((int)c->timeout_s) + " s (a peer rank lost or stuck)";
}

int comm_aborted(swps_comm *c) {
  if (c->guard && c->guard->aborted.load()) return fail(SWPS_E_RCCL, c->guard->msg);
  const std::string e = ipc_error(c);
  if (!e.empty()) return fail(SWPS_E_RCCL, e);
  return SWPS_OK;
}

// a non-blocking communicator's queued call: poll ncclCommGetAsyncError until it leaves
// ncclInProgress, against the deadline
int comm_settle(swps_comm *c, const char *phase) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    SWPS_TRY(comm_aborted(c));
    ncclResult_t st = ncclSuccess;
    const ncclResult_t r = ncclCommGetAsyncError(c->nc, &st);
    if (r != ncclSuccess) return fail(SWPS_E_RCCL, std::string("ncclCommGetAsyncError: ") + ncclGetErrorString(r));
    if (st == ncclSuccess) return SWPS_OK;
    if (st != ncclInProgress) {
      comm_abort(c, std::string(phase) + ": " + ncclGetErrorString(st));
      return comm_aborted(c);
    }
    if (seconds_since(t0) > c->timeout_s) {
      comm_abort(c, std::string(phase) + " still in progress after " + std::to_string((int)c->timeout_s) + " s");
      return comm_aborted(c);
    }
    std::this_thread::yield();
  }
}

// after a collective is queued on s: settle it, then hand its completion event to the watchdog
int comm_track(swps_comm *c, hipStream_t s, const char *phase) {
  SWPS_TRY(comm_settle(c, phase));
  CommGuard *g = c->guard.get();
  if (!g) return SWPS_OK;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->spare.empty()) {
      ev = g->spare.back();
      g->spare.pop_back();
    }
  }
  if (!ev) SWPS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  SWPS_HIP(hipEventRecord(ev, s));
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->pending.push_back({ev, phase, std::chrono::steady_clock::now()});
  }
  g->cv.notify_one();
  return SWPS_OK;
}

void watchdog(swps_comm *c) {
  CommGuard *g = c->guard.get();
  (void)hipSetDevice(c->device);
  std::unique_lock<std::mutex> lk(g->mu);
  while (!g->stop) {
    g->cv.wait_for(lk, std::chrono::milliseconds(20));
    if (g->stop || g->aborted.load()) continue;
    std::string why;
    while (!g->pending.empty()) {
      CommGuard::Pending &p = g->pending.front();
      const hipError_t q = hipEventQuery(p.ev);
      if (q == hipSuccess) {
        g->spare.push_back(p.ev);
        g->pending.pop_front();
        continue;
      }
      if (q != hipErrorNotReady) {
        (void)hipGetLastError();
        why = std::string(p.phase) + ": " + hipGetErrorString(q);
      } else if (seconds_since(p.t0) > c->timeout_s) {
        why = std::string(p.phase) + " did not complete within " + std::to_string((int)c->timeout_s) +
              " s (a peer rank lost or stuck)";
      }
      break;
    }
    if (why.empty() && !g->pending.empty()) {
      ncclResult_t st = ncclSuccess;
      if (ncclCommGetAsyncError(c->nc, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress)
        why = std::string(g->pending.front().phase) + ": RCCL asynchronous error: " + ncclGetErrorString(st);
    }
    if (!why.empty()) {
      lk.unlock();
      comm_abort(c, why);
      lk.lock();
    }
  }
}

inline unsigned nblocks(uint64_t threads, unsigned bs = 256) {
  return (unsigned)std::max<uint64_t>(1, (threads + bs - 1) / bs);
}

// owner rank of each key: node_id(key) - 1 (hashfrag.h:51-56)
__global__ void k_owner(const uint64_t *__restrict__ keys, uint64_t n, const uint32_t *__restrict__ map,
                        uint32_t frag_num, uint32_t *__restrict__ owner, uint32_t *__restrict__ pos) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  owner[i] = map[fmix64(keys[i]) % frag_num] - 1;
  pos[i] = (uint32_t)i;
}

// per-owner counts of the owner-sorted keys (one thread per owner, binary search)
__global__ void k_owner_counts(const uint32_t *__restrict__ owner_s, uint64_t n, int world,
                               uint64_t *__restrict__ cnt) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= world) return;
  auto lower = [&](uint32_t v) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (owner_s[mid] < v)
        lo = mid + 1;
      else
        hi = mid;
    }
    return lo;
  };
  cnt[r] = lower((uint32_t)r + 1) - lower((uint32_t)r);
}

// out[i] = in[perm[i]] for rows of wb bytes (16-B, 4-B or byte lanes)
__global__ void k_gather_rows(const uint32_t *__restrict__ perm, uint64_t n, const char *__restrict__ in,
                              char *__restrict__ out, uint64_t wb) {
  const uint64_t row = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const char *src = in + (uint64_t)perm[row] * wb;
  char *dst = out + row * wb;
  if (wb % 16 == 0) {
    for (uint64_t c = lane; c < wb / 16; c += 64) ((uint4 *)dst)[c] = ((const uint4 *)src)[c];
  } else if (wb % 4 == 0) {
    for (uint64_t c = lane; c < wb / 4; c += 64) ((uint32_t *)dst)[c] = ((const uint32_t *)src)[c];
  } else {
    for (uint64_t c = lane; c < wb; c += 64) dst[c] = src[c];
  }
}

// out[perm[i]] = in[i]
__global__ void k_scatter_rows(const uint32_t *__restrict__ perm, uint64_t n, const char *__restrict__ in,
                               char *__restrict__ out, uint64_t wb) {
  const uint64_t row = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= n) return;
  const char *src = in + row * wb;
  char *dst = out + (uint64_t)perm[row] * wb;
  if (wb % 16 == 0) {
    for (uint64_t c = lane; c < wb / 16; c += 64) ((uint4 *)dst)[c] = ((const uint4 *)src)[c];
  } else if (wb % 4 == 0) {
    for (uint64_t c = lane; c < wb / 4; c += 64) ((uint32_t *)dst)[c] = ((const uint32_t *)src)[c];
  } else {
    for (uint64_t c = lane; c < wb; c += 64) dst[c] = src[c];
  }
}

// One round.  op: kOpPull (d_io = values out, table dtype [n][pull elems]),
// kOpPush (d_io = mean gradients in, the push wire type [n][push elems]) or
// kOpFinish (n = 0).  Returns the op every active rank ran (or kOpFinish when
// all ranks are finishing) in *ran.
int route_round(swps_table *t, int op, const uint64_t *d_keys, uint64_t n, void *d_io, hipStream_t s, int *ran) {
  swps_comm *c = t->comm;
  const int world = c->world;
  const size_t pb = (size_t)t->pull_elems * t->esize;
  const size_t gb = (size_t)t->push_elems * (t->cfg.layout == SWPS_LAYOUT_W2V ? 8 : 4);
  if (n >= (1ULL << 32)) return fail(SWPS_E_UNSUPPORTED, "more than 2^32 keys in one routed call");
  // ---- 1. group by owner ----
  std::vector<int64_t> hdr(2 + world, 0);
  hdr[0] = op;
  uint32_t *perm = nullptr;
  uint64_t *keys_s = nullptr;
  if (n) {
    SWPS_TRY(t->r_owner.ensure(n * 4));
    SWPS_TRY(t->r_pos.ensure(n * 4));
    SWPS_TRY(t->r_owner_s.ensure(n * 4));
    SWPS_TRY(t->r_perm.ensure(n * 4));
    SWPS_TRY(t->r_keys.ensure(n * 8));
    SWPS_TRY(t->r_cnt.ensure(world * 8));
    k_owner<<<nblocks(n), 256, 0, s>>>(d_keys, n, t->frag_map.as<uint32_t>(), (uint32_t)t->frag_num,
                                        t->r_owner.as<uint32_t>(), t->r_pos.as<uint32_t>());
    SWPS_HIP(hipGetLastError());
    int bits = 1;
    while ((1 << bits) < world) bits++;
    size_t sb = 0;
    SWPS_HIP(sort_pairs(nullptr, sb, t->r_owner.as<uint32_t>(), t->r_owner_s.as<uint32_t>(), t->r_pos.as<uint32_t>(),
                        t->r_perm.as<uint32_t>(), n, bits, s));
    SWPS_TRY(t->r_tmp.ensure(sb));
    sb = t->r_tmp.bytes;
    SWPS_HIP(sort_pairs(t->r_tmp.p, sb, t->r_owner.as<uint32_t>(), t->r_owner_s.as<uint32_t>(),
                        t->r_pos.as<uint32_t>(), t->r_perm.as<uint32_t>(), n, bits, s));
    perm = t->r_perm.as<uint32_t>();
    keys_s = t->r_keys.as<uint64_t>();
    k_gather_rows<<<nblocks(n * 64), 256, 0, s>>>(perm, n, (const char *)d_keys, (char *)keys_s, 8);
    k_owner_counts<<<nblocks(world), 256, 0, s>>>(t->r_owner_s.as<uint32_t>(), n, world, t->r_cnt.as<uint64_t>());
    SWPS_HIP(hipGetLastError());
    SWPS_HIP(hipMemcpyAsync(hdr.data() + 2, t->r_cnt.p, world * 8, hipMemcpyDeviceToHost, s));
    SWPS_HIP(hipStreamSynchronize(s));
  }
  // ---- 2. header all-gather ----
  std::vector<int64_t> all((size_t)world * (2 + world));
  SWPS_TRY(comm_allgather(c, hdr.data(), all.data(), (2 + world) * 8, s));
  int agreed = kOpFinish;
  for (int r = 0; r < world; r++) {
    const int o = (int)all[(size_t)r * (2 + world)];
    if (o == kOpFinish) continue;
    if (agreed != kOpFinish && agreed != o)
      return fail(SWPS_E_STATE, "ranks disagree on the routed call (one pulls while another pushes)");
    agreed = o;
  }
  *ran = agreed;
  if (agreed == kOpFinish) return SWPS_OK;
  if (op != kOpFinish && op != agreed) return fail(SWPS_E_STATE, "ranks disagree on the routed call");
  std::vector<uint64_t> send_k(world), recv_k(world);
  uint64_t nrecv = 0, remote = 0;
  for (int r = 0; r < world; r++) {
    send_k[r] = (uint64_t)all[(size_t)c->rank * (2 + world) + 2 + r];
    recv_k[r] = (uint64_t)all[(size_t)r * (2 + world) + 2 + c->rank];
    nrecv += recv_k[r];
    if (r != c->rank) remote += send_k[r];
  }
  // ---- 3. keys (+ gradients) to their owners ----
  SWPS_TRY(t->r_rkeys.ensure(std::max<uint64_t>(nrecv, 1) * 8));
  auto scaled = [&](const std::vector<uint64_t> &k, uint64_t w) {
    std::vector<uint64_t> b(world);
    for (int r = 0; r < world; r++) b[r] = k[r] * w;
    return b;
  };
  SWPS_TRY(comm_alltoallv(t->comm, keys_s, scaled(send_k, 8), t->r_rkeys.p, scaled(recv_k, 8), s, t->stage,
                          "routed keys"));
  const size_t vb = agreed == kOpPull ? pb : gb;
  SWPS_TRY(t->r_rows.ensure(std::max<uint64_t>(nrecv, 1) * 4));
  SWPS_TRY(t->r_rbuf.ensure(std::max<uint64_t>(nrecv, 1) * vb));
  SWPS_TRY(t->r_buf.ensure(std::max<uint64_t>(n, 1) * vb));
  t->rstats[0]++;
  t->rstats[1] += n;
  t->rstats[2] += remote;
  t->rstats[5] += nrecv;
  if (agreed == kOpPush) {
    if (n) k_gather_rows<<<nblocks(n * 64), 256, 0, s>>>(perm, n, (const char *)d_io, t->r_buf.as<char>(), gb);
    SWPS_HIP(hipGetLastError());
    SWPS_TRY(comm_alltoallv(t->comm, t->r_buf.p, scaled(send_k, gb), t->r_rbuf.p, scaled(recv_k, gb), s, t->stage,
                            "routed push gradients"));
    t->rstats[3] += n * (8 + gb);
    t->rstats[4] += remote * (8 + gb);
    // ---- 4. owner: the push rule, one step per source in rank order ----
    if (nrecv) {
      SWPS_TRY(table_lookup(t, t->r_rkeys.as<uint64_t>(), nrecv, t->r_rows.as<uint32_t>(), s));
      int nsrc = 0;
      for (int r = 0; r < world; r++) nsrc += recv_k[r] > 0;
      SWPS_TRY(table_push_sources(t, t->r_rows.as<uint32_t>(), nrecv, t->r_rbuf.p, s, false, nsrc <= 1));
    }
    return SWPS_OK;
  }
  // ---- 4. owner: find-or-insert (init_param on a miss) + pull values ----
  if (nrecv) {
    SWPS_TRY(table_find_or_insert(t, t->r_rkeys.as<uint64_t>(), nrecv, t->r_rows.as<uint32_t>(), s));
    SWPS_TRY(table_copy_pull(t, t->r_rows.as<uint32_t>(), nrecv, t->r_rbuf.p, s));
  }
  // ---- 5. values back to the requesters, then to the caller's key order ----
  SWPS_TRY(comm_alltoallv(t->comm, t->r_rbuf.p, scaled(recv_k, pb), t->r_buf.p, scaled(send_k, pb), s, t->stage,
                          "routed pull values"));
  t->rstats[3] += n * 8 + nrecv * pb;
  t->rstats[4] += remote * 8;
  for (int r = 0; r < world; r++)
    if (r != c->rank) t->rstats[4] += recv_k[r] * pb;
  if (n) k_scatter_rows<<<nblocks(n * 64), 256, 0, s>>>(perm, n, t->r_buf.as<char>(), (char *)d_io, pb);
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

int tcp_send_all(int fd, const void *p, size_t n) {
  const char *b = (const char *)p;
  while (n) {
    const ssize_t k = ::send(fd, b, n, MSG_NOSIGNAL);
    if (k <= 0) return -1;
    b += k;
    n -= (size_t)k;
  }
  return 0;
}

int tcp_recv_all(int fd, void *p, size_t n, int timeout_ms) {
  char *b = (char *)p;
  while (n) {
    pollfd pf{fd, POLLIN, 0};
    if (::poll(&pf, 1, timeout_ms) <= 0) return -1;
    const ssize_t k = ::recv(fd, b, n, 0);
    if (k <= 0) return -1;
    b += k;
    n -= (size_t)k;
  }
  return 0;
}

// ---- native TCP host transport (swps_comm_create_tcp) ----------------------
// A star through rank 0: every rank keeps one socket to rank 0, which
// relays the all-gather and the all-to-all-v blocks.  For jobs without RCCL
// (several ranks on one GPU — RCCL refuses duplicate devices — or host-only
// interconnects); the exchanges of a routed table are small next to its
// compute at the sizes this is meant for.
}  // namespace

struct TcpStar {
  int rank = 0, world = 1;
  std::vector<int> fd;  // rank 0: fd[r] for r >= 1; others: fd[0] = the socket to rank 0
  int timeout_ms = 600000;
  ~TcpStar() {
    for (int f : fd)
      if (f >= 0) ::close(f);
  }
};

namespace {
// the TCP transport's receive deadline: set it to ms (< 0: leave it); the previous value (-1 when the
// communicator has no TCP transport)
int tcp_timeout(swps_comm *c, int ms) {
  if (!c->tcp) return -1;
  const int old = c->tcp->timeout_ms;
  if (ms >= 0) c->tcp->timeout_ms = ms;
  return old;
}
}  // namespace

namespace {

int star_allgather(void *ctx, const void *in, void *out, uint64_t bytes) {
  TcpStar *t = (TcpStar *)ctx;
  char *o = (char *)out;
  if (t->rank != 0) {
    if (tcp_send_all(t->fd[0], in, bytes)) return 1;
    return tcp_recv_all(t->fd[0], o, bytes * t->world, t->timeout_ms) ? 1 : 0;
  }
  memcpy(o, in, bytes);
  for (int r = 1; r < t->world; r++)
    if (tcp_recv_all(t->fd[r], o + (uint64_t)r * bytes, bytes, t->timeout_ms)) return 1;
  for (int r = 1; r < t->world; r++)
    if (tcp_send_all(t->fd[r], o, bytes * t->world)) return 1;
  return 0;
}

int star_alltoallv(void *ctx, const void *send, const uint64_t *sb, void *recv, const uint64_t *rb) {
  TcpStar *t = (TcpStar *)ctx;
  const int W = t->world;
  uint64_t st = 0, rt = 0;
  for (int r = 0; r < W; r++) {
    st += sb[r];
    rt += rb[r];
  }
  if (t->rank != 0) {
    if (tcp_send_all(t->fd[0], sb, W * 8) || (st && tcp_send_all(t->fd[0], send, st))) return 1;
    return (rt && tcp_recv_all(t->fd[0], recv, rt, t->timeout_ms)) ? 1 : 0;
  }
  // rank 0: every source's counts and payload, then each destination's blocks in source order
  std::vector<std::vector<uint64_t>> cnt(W, std::vector<uint64_t>(W));
  std::vector<std::vector<char>> pay(W);
  cnt[0].assign(sb, sb + W);
  pay[0].assign((const char *)send, (const char *)send + st);
  for (int r = 1; r < W; r++) {
    if (tcp_recv_all(t->fd[r], cnt[r].data(), W * 8, t->timeout_ms)) return 1;
    uint64_t n = 0;
    for (int d = 0; d < W; d++) n += cnt[r][d];
    pay[r].resize(n);
    if (n && tcp_recv_all(t->fd[r], pay[r].data(), n, t->timeout_ms)) return 1;
  }
  std::vector<uint64_t> off(W, 0);  // per source: offset of its block for destination d
  for (int d = 0; d < W; d++) {
    std::vector<char> blk;
    for (int src = 0; src < W; src++) {
      uint64_t o = 0;
      for (int k = 0; k < d; k++) o += cnt[src][k];
      blk.insert(blk.end(), pay[src].begin() + o, pay[src].begin() + o + cnt[src][d]);
    }
    if (d == 0) {
      if (blk.size() != rt) return 1;
      if (rt) memcpy(recv, blk.data(), rt);
    } else if (!blk.empty() && tcp_send_all(t->fd[d], blk.data(), blk.size())) {
      return 1;
    }
  }
  return 0;
}

}  // namespace

namespace swps {

// all-gather of a small host block (round headers, count matrices)
int comm_allgather(swps_comm *c, const void *in, void *out, uint64_t bytes, hipStream_t s) {
  if (c->world == 1) {
    memcpy(out, in, bytes);
    return SWPS_OK;
  }
  if (!c->rccl) {
    if (c->tr.allgather(c->tr.ctx, in, out, bytes) != 0) return fail(SWPS_E_RCCL, "host transport all-gather failed");
    return SWPS_OK;
  }
  SWPS_TRY(comm_aborted(c));
  SWPS_TRY(c->d_hdr.ensure(bytes * (c->world + 1)));
  char *d = c->d_hdr.as<char>();
  SWPS_HIP(hipMemcpyAsync(d, in, bytes, hipMemcpyHostToDevice, s));
  SWPS_NCCL(ncclAllGather(d, d + bytes, bytes, ncclChar, c->nc, s));
  SWPS_TRY(comm_track(c, s, "header all-gather"));
  SWPS_HIP(hipMemcpyAsync(out, d + bytes, bytes * c->world, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));  // returns once the guard aborts a stuck exchange
  return comm_aborted(c);
}

template <typename V>
__global__ void k_scatter_rows(const V *__restrict__ src, const uint32_t *__restrict__ pos, uint64_t n, uint32_t rv,
                               V *__restrict__ dst) {
  // one wave per row, rv V-elements per row
  const uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const V *a = src + i * rv;
  V *b = dst + (uint64_t)pos[i] * rv;
  for (uint32_t e = lane; e < rv; e += 64) b[e] = a[e];
}

int scatter_rows(const void *src, const uint32_t *pos, uint64_t n, uint64_t row_bytes, void *dst, hipStream_t s) {
  if (!n) return SWPS_OK;
  const unsigned blocks = (unsigned)((n * 64 + 255) / 256);
  if (row_bytes % 16 == 0)
    k_scatter_rows<uint4><<<blocks, 256, 0, s>>>((const uint4 *)src, pos, n, (uint32_t)(row_bytes / 16), (uint4 *)dst);
  else
    k_scatter_rows<uint32_t><<<blocks, 256, 0, s>>>((const uint32_t *)src, pos, n, (uint32_t)(row_bytes / 4),
                                                    (uint32_t *)dst);
  SWPS_HIP(hipGetLastError());
  return SWPS_OK;
}

// ---- the IPC exchange (IpcState) ----
struct IpcArgs {
  char *inbox[kIpcMaxWorld];
  uint64_t *ctrl[kIpcMaxWorld];
  const char *send;
  char *recv;
  uint64_t sb[kIpcMaxWorld], so[kIpcMaxWorld], rb[kIpcMaxWorld], ro[kIpcMaxWorld];
  uint64_t sc[kIpcMaxWorld][kIpcCh], rc[kIpcMaxWorld][kIpcCh];  // rounds before this exchange
  uint64_t slot, sub, deadline;  // deadline in wall-clock ticks
  uint64_t *err;
  int32_t rank, world;
};

// channel ch's part of an L-byte segment: parts of ceil(L / kIpcCh) bytes rounded up to 16, at
// least kIpcMinPart (a small segment uses the first channels only); the same on both sides
__host__ __device__ inline void ipc_span(uint64_t L, int ch, uint64_t *off, uint64_t *len) {
  uint64_t part = ((L + kIpcCh - 1) / kIpcCh + 15) & ~15ull;
  if (part < kIpcMinPart) part = kIpcMinPart;
  const uint64_t o = part * (uint64_t)ch;
  *off = o < L ? o : L;
  *len = o < L ? (L - o < part ? L - o : part) : 0;
}

// block-wide copy (256 threads): 16-B words when both ends and the length allow it
__device__ inline void ipc_copy(char *dst, const char *src, uint64_t n) {
  const uint64_t t = threadIdx.x;
  const uint64_t al = (uint64_t)(uintptr_t)dst | (uint64_t)(uintptr_t)src | n;
  if ((al & 15) == 0) {
    const uint4 *s = (const uint4 *)src;
    uint4 *d = (uint4 *)dst;
    const uint64_t m = n >> 4;
    uint64_t i = t;
    for (; i + 768 < m; i += 1024) {  // four loads in flight per lane
      const uint4 a = s[i], b = s[i + 256], c = s[i + 512], e = s[i + 768];
      d[i] = a;
      d[i + 256] = b;
      d[i + 512] = c;
      d[i + 768] = e;
    }
    for (; i < m; i += 256) d[i] = s[i];
  } else if ((al & 3) == 0) {
    const uint32_t *s = (const uint32_t *)src;
    uint32_t *d = (uint32_t *)dst;
    for (uint64_t i = t; i < (n >> 2); i += 256) d[i] = s[i];
  } else {
    for (uint64_t i = t; i < n; i += 256) dst[i] = src[i];
  }
}

// lane 0 polls w (relaxed, system scope) until it reaches v; false (and the error words set) once
// the deadline passes or a workgroup of this rank or of a peer gave up; uniform over the block
__device__ bool ipc_wait(uint64_t *w, uint64_t v, const IpcArgs &a, uint64_t code) {
  __shared__ int ok;
  if (threadIdx.x == 0) {
    int r = 1;
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
      uint64_t *dead = a.ctrl[a.rank] + kIpcDead;
      const uint64_t t0 = wall_clock64();
      for (unsigned it = 1;; it++) {
        __builtin_amdgcn_s_sleep(2);
        if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= v) break;
        if ((it & 63) == 0 && (__hip_atomic_load(dead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ||
                               wall_clock64() - t0 > a.deadline)) {
          // this rank's other workgroups and every peer's stop at their next check (a peer's
          // next exchange then fails instead of waiting out its own deadline)
          for (int r = 0; r < a.world; r++)
            __hip_atomic_store(a.ctrl[r] + kIpcDead, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __hip_atomic_store(a.err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          r = 0;
          break;
        }
      }
    }
    ok = r;
  }
  __syncthreads();
  return ok != 0;
}

// grid: world x kIpcCh send workgroups, then as many receive workgroups
__device__ __forceinline__ void ipc_body(const IpcArgs &a) {
  const int ch = blockIdx.x % kIpcCh;
  const int peer = (blockIdx.x / kIpcCh) % a.world;
  const bool rx = blockIdx.x >= (unsigned)(a.world * kIpcCh);
  const int me = a.rank;
  uint64_t off, len;
  if (!rx) {
    ipc_span(a.sb[peer], ch, &off, &len);
    if (!len) return;
    const char *src = a.send + a.so[peer] + off;
    if (peer == me) {  // the own segment: straight into the receive buffer
      ipc_copy(a.recv + a.ro[me] + off, src, len);
      return;
    }
    uint64_t *ready = a.ctrl[peer] + me * kIpcCh + ch;          // the peer's word for (me, ch)
    uint64_t *ack = a.ctrl[me] + kIpcAck + peer * kIpcCh + ch;  // mine, bumped by the peer
    char *box = a.inbox[peer] + (uint64_t)me * 2 * a.slot + (uint64_t)ch * a.sub;
    const uint64_t code = (1ull << 63) | (uint64_t)peer;
    uint64_t g = a.sc[peer][ch];
    for (uint64_t d = 0; d < len; d += a.sub, g++) {
      if (g >= 2 && !ipc_wait(ack, g - 1, a, code)) return;  // round g-2 (same parity) consumed
      ipc_copy(box + (g & 1) * a.slot, src + d, len - d < a.sub ? len - d : a.sub);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(ready, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  } else {
    ipc_span(a.rb[peer], ch, &off, &len);
    if (!len || peer == me) return;
    uint64_t *ready = a.ctrl[me] + peer * kIpcCh + ch;
    uint64_t *ack = a.ctrl[peer] + kIpcAck + me * kIpcCh + ch;
    const char *box = a.inbox[me] + (uint64_t)peer * 2 * a.slot + (uint64_t)ch * a.sub;
    char *dst = a.recv + a.ro[peer] + off;
    const uint64_t code = (1ull << 63) | (1ull << 8) | (uint64_t)peer;
    uint64_t g = a.rc[peer][ch];
    for (uint64_t d = 0; d < len; d += a.sub, g++) {
      if (!ipc_wait(ready, g + 1, a, code)) return;
      if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      ipc_copy(dst + d, box + (g & 1) * a.slot, len - d < a.sub ? len - d : a.sub);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the inbox reads are done before the ack
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(ack, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(256) void k_ipc_a2a(IpcArgs a) {
  // a rank (this one or a peer) that gave up on an earlier exchange marked every rank dead: an
  // exchange whose waits all happen to be met (stale rounds) must still fail.  The load is in
  // flight during the copies.
  uint64_t d0 = 0;
  if (threadIdx.x == 0) d0 = __hip_atomic_load(a.ctrl[a.rank] + kIpcDead, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  ipc_body(a);
  if (threadIdx.x == 0 && d0)
    __hip_atomic_store(a.err, (1ull << 63) | (1ull << 9), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int ipc_alltoallv(swps_comm *c, const void *d_send, const uint64_t *sb, const uint64_t *so, void *d_recv,
                  const uint64_t *rb, const uint64_t *ro, hipStream_t s) {
  IpcState &p = *c->ipc;
  SWPS_TRY(comm_aborted(c));
  // argument errors first: the round counters below must advance on every rank or on none
  if (sb[c->rank] != rb[c->rank]) return fail(SWPS_E_STATE, "IPC exchange: own segment sizes differ");
  IpcArgs a{};
  const int W = c->world;
  for (int r = 0; r < W; r++) {
    a.inbox[r] = (char *)p.peer_inbox[r];
    a.ctrl[r] = (uint64_t *)p.peer_ctrl[r];
    a.sb[r] = sb[r];
    a.so[r] = so[r];
    a.rb[r] = rb[r];
    a.ro[r] = ro[r];
    for (int ch = 0; ch < kIpcCh; ch++) {
      a.sc[r][ch] = p.sc[r * kIpcCh + ch];
      a.rc[r][ch] = p.rc[r * kIpcCh + ch];
      uint64_t off, len;
      ipc_span(sb[r], ch, &off, &len);
      if (r != c->rank) p.sc[r * kIpcCh + ch] += (len + p.sub - 1) / p.sub;
      ipc_span(rb[r], ch, &off, &len);
      if (r != c->rank) p.rc[r * kIpcCh + ch] += (len + p.sub - 1) / p.sub;
    }
    if (r != c->rank) p.bytes_remote += sb[r];
  }
  a.send = (const char *)d_send;
  a.recv = (char *)d_recv;
  a.slot = p.slot;
  a.sub = p.sub;
  a.deadline = (uint64_t)(c->timeout_s * (double)p.ticks_per_s);
  a.err = p.err_dev;
  a.rank = c->rank;
  a.world = W;
  if (p.issued) SWPS_HIP(hipStreamWaitEvent(s, p.last, 0));
  k_ipc_a2a<<<2 * W * kIpcCh, 256, 0, s>>>(a);
  SWPS_HIP(hipGetLastError());
  SWPS_HIP(hipEventRecord(p.last, s));
  p.issued = true;
  p.calls++;
  return SWPS_OK;
}

// all-to-all-v of device buffers (byte counts per peer, blocks in rank
// order), ordered on stream s: RCCL send/recv groups, or host staging
// through `st` and the transport's callback (synchronous)
int comm_alltoallv(swps_comm *c, const void *d_send, const std::vector<uint64_t> &sb, void *d_recv,
                   const std::vector<uint64_t> &rb, hipStream_t s, HostStage &stg, const char *phase) {
  uint64_t st = 0, rt = 0;
  for (int r = 0; r < c->world; r++) {
    st += sb[r];
    rt += rb[r];
  }
  if (c->world == 1) {
    if (st) SWPS_HIP(hipMemcpyAsync(d_recv, d_send, st, hipMemcpyDeviceToDevice, s));
    return SWPS_OK;
  }
  if (c->ipc) {
    std::vector<uint64_t> so(c->world), ro(c->world);
    for (int r = 1; r < c->world; r++) {
      so[r] = so[r - 1] + sb[r - 1];
      ro[r] = ro[r - 1] + rb[r - 1];
    }
    return ipc_alltoallv(c, d_send, sb.data(), so.data(), d_recv, rb.data(), ro.data(), s);
  }
  if (c->rccl) {
    SWPS_TRY(comm_aborted(c));
    SWPS_NCCL(ncclGroupStart());
    uint64_t so = 0, ro = 0;
    for (int r = 0; r < c->world; r++) {
      if (sb[r]) SWPS_NCCL(ncclSend((const char *)d_send + so, sb[r], ncclChar, r, c->nc, s));
      if (rb[r]) SWPS_NCCL(ncclRecv((char *)d_recv + ro, rb[r], ncclChar, r, c->nc, s));
      so += sb[r];
      ro += rb[r];
    }
    SWPS_NCCL(ncclGroupEnd());
    return comm_track(c, s, phase);
  }
  stg.send.resize(std::max<uint64_t>(st, 1));
  stg.recv.resize(std::max<uint64_t>(rt, 1));
  if (st) SWPS_HIP(hipMemcpyAsync(stg.send.data(), d_send, st, hipMemcpyDeviceToHost, s));
  SWPS_HIP(hipStreamSynchronize(s));
  if (c->tr.alltoallv(c->tr.ctx, stg.send.data(), sb.data(), stg.recv.data(), rb.data()) != 0)
    return fail(SWPS_E_RCCL, "host transport all-to-all-v failed");
  if (rt) SWPS_HIP(hipMemcpyAsync(d_recv, stg.recv.data(), rt, hipMemcpyHostToDevice, s));
  SWPS_HIP(hipStreamSynchronize(s));  // stg.recv is reused by the next exchange
  return SWPS_OK;
}

// all-to-all-v with explicit byte displacements: peer r gets sb[r] bytes from d_send + so[r] and
// sends rb[r] bytes that land at d_recv + ro[r] (a part of a larger exchange, e.g. half of every
// peer's segment)
int comm_alltoallv_disp(swps_comm *c, const void *d_send, const std::vector<uint64_t> &sb,
                        const std::vector<uint64_t> &so, void *d_recv, const std::vector<uint64_t> &rb,
                        const std::vector<uint64_t> &ro, hipStream_t s, HostStage &stg, const char *phase) {
  uint64_t st = 0, rt = 0;
  for (int r = 0; r < c->world; r++) {
    st += sb[r];
    rt += rb[r];
  }
  if (c->world == 1) {
    if (sb[0]) SWPS_HIP(hipMemcpyAsync((char *)d_recv + ro[0], (const char *)d_send + so[0], sb[0],
                                       hipMemcpyDeviceToDevice, s));
    return SWPS_OK;
  }
  if (c->ipc) return ipc_alltoallv(c, d_send, sb.data(), so.data(), d_recv, rb.data(), ro.data(), s);
  if (c->rccl) {
    SWPS_TRY(comm_aborted(c));
    SWPS_NCCL(ncclGroupStart());
    for (int r = 0; r < c->world; r++) {
      if (sb[r]) SWPS_NCCL(ncclSend((const char *)d_send + so[r], sb[r], ncclChar, r, c->nc, s));
      if (rb[r]) SWPS_NCCL(ncclRecv((char *)d_recv + ro[r], rb[r], ncclChar, r, c->nc, s));
    }
    SWPS_NCCL(ncclGroupEnd());
    return comm_track(c, s, phase);
  }
  stg.send.resize(std::max<uint64_t>(st, 1));
  stg.recv.resize(std::max<uint64_t>(rt, 1));
  uint64_t o = 0;
  for (int r = 0; r < c->world; r++) {  // pack the segments for the host transport
    if (sb[r])
      SWPS_HIP(hipMemcpyAsync(stg.send.data() + o, (const char *)d_send + so[r], sb[r], hipMemcpyDeviceToHost, s));
    o += sb[r];
  }
  SWPS_HIP(hipStreamSynchronize(s));
  if (c->tr.alltoallv(c->tr.ctx, stg.send.data(), sb.data(), stg.recv.data(), rb.data()) != 0)
    return fail(SWPS_E_RCCL, "host transport all-to-all-v failed");
  o = 0;
  for (int r = 0; r < c->world; r++) {
    if (rb[r])
      SWPS_HIP(hipMemcpyAsync((char *)d_recv + ro[r], stg.recv.data() + o, rb[r], hipMemcpyHostToDevice, s));
    o += rb[r];
  }
  SWPS_HIP(hipStreamSynchronize(s));  // stg.recv is reused by the next exchange
  return SWPS_OK;
}

int comm_status(swps_comm *c) { return c ? comm_aborted(c) : SWPS_OK; }
int comm_rank(const swps_comm *c) { return c->rank; }
int comm_world(const swps_comm *c) { return c->world; }
int comm_device(const swps_comm *c) { return c->device; }
bool comm_is_rccl(const swps_comm *c) { return c->rccl; }

int routed_pull(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_vals, hipStream_t s) {
  if (t->finished) return fail(SWPS_E_STATE, "pull after swps_finish");
  int ran = 0;
  SWPS_TRY(route_round(t, kOpPull, d_keys, n, d_vals, s, &ran));
  if (ran != kOpPull) return fail(SWPS_E_STATE, "routed pull while every other rank has finished");
  return SWPS_OK;
}

int routed_push(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_grads, hipStream_t s) {
  if (t->finished) return fail(SWPS_E_STATE, "push after swps_finish");
  int ran = 0;
  SWPS_TRY(route_round(t, kOpPush, d_keys, n, const_cast<void *>(d_grads), s, &ran));
  if (ran != kOpPush) return fail(SWPS_E_STATE, "routed push while every other rank has finished");
  return SWPS_OK;
}

}  // namespace swps

extern "C" {

int swps_comm_unique_id(uint8_t *id) {
  if (!id) return fail(SWPS_E_CFG, "null id");
  ncclUniqueId u;
  SWPS_NCCL(ncclGetUniqueId(&u));
  memcpy(id, u.internal, SWPS_COMM_ID_BYTES);
  return SWPS_OK;
}

int swps_comm_bootstrap_tcp(const char *addr, int32_t port, int32_t rank, int32_t world, int32_t timeout_ms,
                            uint8_t *id) {
  if (!addr || !id || world < 1 || rank < 0 || rank >= world || port <= 0 || port > 65535)
    return fail(SWPS_E_CFG, "bad bootstrap arguments");
  if (world == 1) return swps_comm_unique_id(id);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, addr, &sa.sin_addr) != 1) return fail(SWPS_E_CFG, std::string("bad IPv4 address ") + addr);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  if (rank == 0) {
    SWPS_TRY(swps_comm_unique_id(id));
    const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
    if (ls < 0) return fail(SWPS_E_IO, "socket");
    const int one = 1;
    setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    if (::bind(ls, (sockaddr *)&sa, sizeof(sa)) != 0 || ::listen(ls, world) != 0) {
      ::close(ls);
      return fail(SWPS_E_IO, "bootstrap: cannot listen on " + std::string(addr) + ":" + std::to_string(port));
    }
    int served = 0, rc = SWPS_OK;
    while (served < world - 1) {
      const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                           deadline - std::chrono::steady_clock::now()).count();
      pollfd pf{ls, POLLIN, 0};
      if (left <= 0 || ::poll(&pf, 1, left) <= 0) {
        rc = fail(SWPS_E_IO, "bootstrap: timed out waiting for ranks");
        break;
      }
      const int fd = ::accept(ls, nullptr, nullptr);
      if (fd < 0) continue;
      const int bad = tcp_send_all(fd, id, SWPS_COMM_ID_BYTES);
      ::close(fd);
      if (bad) {
        rc = fail(SWPS_E_IO, "bootstrap: send failed");
        break;
      }
      served++;
    }
    ::close(ls);
    return rc;
  }
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return fail(SWPS_E_IO, "socket");
    if (::connect(fd, (sockaddr *)&sa, sizeof(sa)) == 0) {
      const int bad = tcp_recv_all(fd, id, SWPS_COMM_ID_BYTES, std::max(timeout_ms, 1));
      ::close(fd);
      if (bad) return fail(SWPS_E_IO, "bootstrap: receive failed");
      return SWPS_OK;
    }
    ::close(fd);
    if (std::chrono::steady_clock::now() >= deadline)
      return fail(SWPS_E_IO, "bootstrap: cannot reach rank 0 at " + std::string(addr) + ":" + std::to_string(port));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

int swps_comm_create_rccl(const uint8_t *id, int32_t rank, int32_t world, int32_t device, swps_comm **out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) return fail(SWPS_E_CFG, "bad communicator arguments");
  *out = nullptr;
  SWPS_HIP(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(u.internal, id, SWPS_COMM_ID_BYTES);
  std::unique_ptr<swps_comm> c(new swps_comm());
  c->rank = rank;
  c->world = world;
  c->device = device;
  c->rccl = true;
  if (const char *e = getenv("SWPS_COMM_TIMEOUT_S")) c->timeout_s = std::max(1.0, atof(e));
  // non-blocking: the initialisation is polled against the deadline (comm_settle), and so is every
  // queued call after it (SWPS_RCCL_BLOCKING=1: a blocking communicator, no deadline on init)
  const char *bl = getenv("SWPS_RCCL_BLOCKING");
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = (bl && atoi(bl)) ? 1 : 0;
  ncclComm_t nc = nullptr;
  const ncclResult_t r = ncclCommInitRankConfig(&nc, world, u, rank, &cfg);
  if (r != ncclSuccess && r != ncclInProgress) {
    if (nc) (void)ncclCommAbort(nc);
    return fail(SWPS_E_RCCL, std::string("rank ") + std::to_string(rank) + ": ncclCommInitRankConfig: " +
                                 ncclGetErrorString(r));
  }
  c->nc = nc;
  c->guard.reset(new CommGuard());  // world 1 too: the init deadline and the same code path
  const int rc = comm_settle(c.get(), "RCCL initialisation");
  if (rc != SWPS_OK) return rc;  // aborted (and freed) by comm_abort
  c->guard->th = std::thread(watchdog, c.get());
  *out = c.release();
  return SWPS_OK;
}

int swps_comm_create_host(const swps_transport *tr, int32_t rank, int32_t world, int32_t device, swps_comm **out) {
  if (!tr || !out || world < 1 || rank < 0 || rank >= world) return fail(SWPS_E_CFG, "bad communicator arguments");
  if (world > 1 && (!tr->allgather || !tr->alltoallv)) return fail(SWPS_E_CFG, "transport callbacks missing");
  swps_comm *c = new swps_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  c->tr = *tr;
  *out = c;
  return SWPS_OK;
}

int swps_comm_create_tcp(const char *addr, int32_t port, int32_t rank, int32_t world, int32_t device,
                         int32_t timeout_ms, swps_comm **out) {
  if (!addr || !out || world < 1 || rank < 0 || rank >= world || port <= 0 || port > 65535)
    return fail(SWPS_E_CFG, "bad communicator arguments");
  *out = nullptr;
  std::unique_ptr<TcpStar> st(new TcpStar());
  st->rank = rank;
  st->world = world;
  st->timeout_ms = std::max(timeout_ms, 1000);
  if (world > 1) {
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, addr, &sa.sin_addr) != 1) return fail(SWPS_E_CFG, std::string("bad IPv4 address ") + addr);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    const int one = 1;
    if (rank == 0) {
      st->fd.assign(world, -1);
      const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
      if (ls < 0) return fail(SWPS_E_IO, "socket");
      setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
      if (::bind(ls, (sockaddr *)&sa, sizeof(sa)) != 0 || ::listen(ls, world) != 0) {
        ::close(ls);
        return fail(SWPS_E_IO, "tcp transport: cannot listen on " + std::string(addr) + ":" + std::to_string(port));
      }
      for (int got = 1; got < world;) {
        const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                             deadline - std::chrono::steady_clock::now()).count();
        pollfd pf{ls, POLLIN, 0};
        if (left <= 0 || ::poll(&pf, 1, left) <= 0) {
          ::close(ls);
          return fail(SWPS_E_IO, "tcp transport: timed out waiting for ranks");
        }
        const int fd = ::accept(ls, nullptr, nullptr);
        if (fd < 0) continue;
        int32_t r = -1;
        if (tcp_recv_all(fd, &r, 4, st->timeout_ms) || r <= 0 || r >= world || st->fd[r] >= 0) {
          ::close(fd);
          ::close(ls);
          return fail(SWPS_E_IO, "tcp transport: bad hello");
        }
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        st->fd[r] = fd;
        got++;
      }
      ::close(ls);
    } else {
      for (;;) {
        const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) return fail(SWPS_E_IO, "socket");
        if (::connect(fd, (sockaddr *)&sa, sizeof(sa)) == 0) {
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          const int32_t r = rank;
          if (tcp_send_all(fd, &r, 4)) {
            ::close(fd);
            return fail(SWPS_E_IO, "tcp transport: hello failed");
          }
          st->fd.assign(1, fd);
          break;
        }
        ::close(fd);
        if (std::chrono::steady_clock::now() >= deadline)
          return fail(SWPS_E_IO, "tcp transport: cannot reach rank 0 at " + std::string(addr) + ":" +
                                     std::to_string(port));
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
      }
    }
  }
  swps_transport tr{st.get(), star_allgather, star_alltoallv};
  swps_comm *c = nullptr;
  SWPS_TRY(swps_comm_create_host(&tr, rank, world, device, &c));
  c->tcp = st.release();
  *out = c;
  return SWPS_OK;
}

int swps_comm_destroy(swps_comm *c) {
  if (!c) return SWPS_OK;
  (void)hipSetDevice(c->device);
  if (IpcState *p = c->ipc.get(); p && c->world > 1) {
    // peers store into this rank's inbox / ctrl words until their last exchange has retired: every
    // rank syncs its device and then joins one all-gather of its status (the dead word) — also a
    // rank that gave up on an exchange, so a peer whose exchanges all completed never waits alone.
    // The all-gather is bounded by a short deadline (a peer whose process is gone costs that, not
    // the communicator's full timeout); a communicator already aborted cannot join it.
    uint64_t dead = 1;
    if (hipDeviceSynchronize() == hipSuccess)
      (void)hipMemcpy(&dead, (uint64_t *)p->ctrl + kIpcDead, 8, hipMemcpyDeviceToHost);
    (void)hipGetLastError();
    hipStream_t hs = nullptr;
    if (comm_aborted(c) == SWPS_OK && hipStreamCreateWithFlags(&hs, hipStreamNonBlocking) == hipSuccess) {
      const double t_keep = c->timeout_s;
      const int tcp_keep = tcp_timeout(c, -1);
      const double t_short = std::min(t_keep, 10.0);
      c->timeout_s = t_short;
      (void)tcp_timeout(c, (int)(t_short * 1000));
      std::vector<int64_t> all(c->world);
      const int64_t st = (int64_t)dead;
      (void)comm_allgather(c, &st, all.data(), 8, hs);
      (void)hipStreamDestroy(hs);
      c->timeout_s = t_keep;
      (void)tcp_timeout(c, tcp_keep);
    }
    for (int r = 0; r < c->world; r++)
      if (r != c->rank) {
        if (p->peer_inbox[r]) (void)hipIpcCloseMemHandle(p->peer_inbox[r]);
        if (p->peer_ctrl[r]) (void)hipIpcCloseMemHandle(p->peer_ctrl[r]);
      }
    (void)hipFree(p->inbox);
    (void)hipFree(p->ctrl);
    (void)hipHostFree(p->err_host);
    if (p->last) (void)hipEventDestroy(p->last);
    c->ipc.reset();
  }
  if (c->nstream) (void)hipStreamDestroy(c->nstream);
  if (c->nev_in) (void)hipEventDestroy(c->nev_in);
  if (c->nev_out) (void)hipEventDestroy(c->nev_out);
  if (CommGuard *g = c->guard.get()) {
    {
      std::lock_guard<std::mutex> lk(g->mu);
      g->stop = true;
    }
    g->cv.notify_all();
    if (g->th.joinable()) g->th.join();
  }
  if (c->nc && !(c->guard && c->guard->aborted.load())) {
    // non-blocking: finalize (flushes the queued exchanges), wait for quiescence, then free
    const ncclResult_t r = ncclCommFinalize(c->nc);
    if (r == ncclSuccess || r == ncclInProgress) (void)comm_settle(c, "RCCL finalize");
    if (!c->guard->aborted.load()) (void)ncclCommDestroy(c->nc);
  }
  if (c->guard) {
    for (auto &p : c->guard->pending) (void)hipEventDestroy(p.ev);
    for (auto ev : c->guard->spare) (void)hipEventDestroy(ev);
  }
  delete c->tcp;
  delete c;
  return SWPS_OK;
}

int swps_comm_set_timeout(swps_comm *c, double seconds) {
  if (!c || !(seconds > 0)) return fail(SWPS_E_CFG, "null communicator or non-positive timeout");
  c->timeout_s = seconds;
  return SWPS_OK;
}

int swps_comm_check(swps_comm *c) {
  if (!c) return fail(SWPS_E_CFG, "null communicator");
  return comm_aborted(c);
}

int swps_comm_abort(swps_comm *c, const char *why) {
  if (!c) return fail(SWPS_E_CFG, "null communicator");
  if (!c->guard) return SWPS_OK;
  comm_abort(c, why ? why : "aborted by the caller");
  return SWPS_OK;
}

int swps_comm_info(swps_comm *c, int32_t *rank, int32_t *world) {
  if (!c) return fail(SWPS_E_CFG, "null communicator");
  if (rank) *rank = c->rank;
  if (world) *world = c->world;
  return SWPS_OK;
}

int swps_comm_transport(swps_comm *c, int32_t *kind, int32_t *ranks) {
  if (!c) return fail(SWPS_E_CFG, "null communicator");
  int32_t n = c->world;
  SWPS_TRY(comm_aborted(c));
  if (c->nc) SWPS_NCCL(ncclCommCount(c->nc, &n));  // what RCCL itself reports for the communicator
  if (kind) *kind = c->rccl ? SWPS_COMM_RCCL : c->tcp ? SWPS_COMM_TCP : SWPS_COMM_HOST;
  if (ranks) *ranks = n;
  return SWPS_OK;
}

int swps_comm_enable_ipc(swps_comm *c, uint64_t slot_bytes) {
  if (!c) return fail(SWPS_E_CFG, "null communicator");
  if (c->ipc) return fail(SWPS_E_STATE, "IPC exchange already enabled");
  if (c->world > kIpcMaxWorld)
    return fail(SWPS_E_CFG, "IPC exchange: world " + std::to_string(c->world) + " > " +
                                std::to_string(kIpcMaxWorld) + " (one node)");
  SWPS_TRY(comm_aborted(c));
  if (!slot_bytes) {
    const char *e = getenv("SWPS_COMM_IPC_SLOT_MB");
    slot_bytes = (uint64_t)((e ? std::max(1.0, atof(e)) : 4.0) * (1 << 20));
  }
  const uint64_t q = (uint64_t)kIpcCh * 4096;  // sub-slots of whole pages
  slot_bytes = (slot_bytes + q - 1) / q * q;
  SWPS_HIP(hipSetDevice(c->device));
  std::unique_ptr<IpcState> p(new IpcState());
  p->slot = slot_bytes;
  p->sub = slot_bytes / kIpcCh;
  const int W = c->world;
  p->sc.assign((size_t)W * kIpcCh, 0);
  p->rc.assign((size_t)W * kIpcCh, 0);
  p->peer_inbox.assign(W, nullptr);
  p->peer_ctrl.assign(W, nullptr);
  if (W > 1) {
    int khz = 0;
    SWPS_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    p->ticks_per_s = (uint64_t)std::max(khz, 1) * 1000;
    auto undo = [&](const std::string &why) {
      for (int r = 0; r < W; r++)
        if (r != c->rank) {
          if (p->peer_inbox[r]) (void)hipIpcCloseMemHandle(p->peer_inbox[r]);
          if (p->peer_ctrl[r]) (void)hipIpcCloseMemHandle(p->peer_ctrl[r]);
        }
      if (p->inbox) (void)hipFree(p->inbox);
      if (p->ctrl) (void)hipFree(p->ctrl);
      if (p->err_host) (void)hipHostFree(p->err_host);
      (void)hipGetLastError();
      return fail(SWPS_E_RCCL, "IPC exchange: " + why);
    };
    // collective from here on: a rank whose own setup fails still joins the handle all-gather (with
    // ok = 0), and the handles' opens are confirmed by a second all-gather, so every rank enables
    // the exchange or every rank undoes it — none waits alone in a collective the others left
    std::string why;
    hipIpcMemHandle_t mh[2];
    if (hipExtMallocWithFlags(&p->inbox, (size_t)W * 2 * p->slot, hipDeviceMallocUncached) != hipSuccess ||
        hipExtMallocWithFlags(&p->ctrl, kIpcCtrlBytes, hipDeviceMallocUncached) != hipSuccess)
      why = "uncached allocation failed";
    else if (hipMemset(p->ctrl, 0, kIpcCtrlBytes) != hipSuccess ||
             hipHostMalloc((void **)&p->err_host, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      why = "control words";
    else if ((*p->err_host = 0, hipHostGetDevicePointer((void **)&p->err_dev, p->err_host, 0) != hipSuccess) ||
             hipDeviceSynchronize() != hipSuccess)
      why = "error word";
    else if (hipIpcGetMemHandle(&mh[0], p->inbox) != hipSuccess || hipIpcGetMemHandle(&mh[1], p->ctrl) != hipSuccess)
      why = "hipIpcGetMemHandle failed";
    (void)hipGetLastError();
    struct Hdr {
      int64_t ok;
      hipIpcMemHandle_t h[2];
    } mine{}, all[kIpcMaxWorld];
    mine.ok = why.empty() ? 1 : 0;
    if (mine.ok) {
      mine.h[0] = mh[0];
      mine.h[1] = mh[1];
    }
    // every rank's ctrl words are zero before its handles leave it, so a peer's first store lands after
    hipStream_t hs = nullptr;
    if (hipStreamCreateWithFlags(&hs, hipStreamNonBlocking) != hipSuccess) return undo("stream");
    if (comm_allgather(c, &mine, all, sizeof(Hdr), hs) != SWPS_OK) {
      (void)hipStreamDestroy(hs);
      return undo("handle all-gather failed");
    }
    for (int r = 0; r < W; r++)
      if (!all[r].ok) {
        (void)hipStreamDestroy(hs);
        return undo(r == c->rank ? why : "rank " + std::to_string(r) + " could not set up its buffers");
      }
    for (int r = 0; r < W && why.empty(); r++) {
      if (r == c->rank) {
        p->peer_inbox[r] = p->inbox;
        p->peer_ctrl[r] = p->ctrl;
        continue;
      }
      if (hipIpcOpenMemHandle(&p->peer_inbox[r], all[r].h[0], hipIpcMemLazyEnablePeerAccess) != hipSuccess ||
          hipIpcOpenMemHandle(&p->peer_ctrl[r], all[r].h[1], hipIpcMemLazyEnablePeerAccess) != hipSuccess)
        why = "hipIpcOpenMemHandle of rank " + std::to_string(r) + "'s buffers failed";
    }
    (void)hipGetLastError();
    int64_t opened = why.empty() ? 1 : 0, okv[kIpcMaxWorld];
    const int ag2 = comm_allgather(c, &opened, okv, 8, hs);
    (void)hipStreamDestroy(hs);
    if (ag2 != SWPS_OK) return undo("open confirmation all-gather failed");
    for (int r = 0; r < W; r++)
      if (!okv[r]) return undo(r == c->rank ? why : "rank " + std::to_string(r) + " could not map its peers' buffers");
    if (hipEventCreateWithFlags(&p->last, hipEventDisableTiming) != hipSuccess) return undo("event");
  }
  c->ipc = std::move(p);
  return SWPS_OK;
}

int swps_comm_alltoallv(swps_comm *c, const void *d_send, const uint64_t *send_bytes, void *d_recv,
                        const uint64_t *recv_bytes, void *stream) {
  if (!c || !send_bytes || !recv_bytes) return fail(SWPS_E_CFG, "null argument");
  SWPS_HIP(hipSetDevice(c->device));
  const std::vector<uint64_t> sb(send_bytes, send_bytes + c->world), rb(recv_bytes, recv_bytes + c->world);
  hipStream_t s = (hipStream_t)stream;
  if (!s && c->rccl && c->world > 1) {  // an RCCL communicator never sees the null stream
    if (!c->nstream) {
      SWPS_HIP(hipStreamCreateWithFlags(&c->nstream, hipStreamNonBlocking));
      SWPS_HIP(hipEventCreateWithFlags(&c->nev_in, hipEventDisableTiming));
      SWPS_HIP(hipEventCreateWithFlags(&c->nev_out, hipEventDisableTiming));
    }
    SWPS_HIP(hipEventRecord(c->nev_in, nullptr));
    SWPS_HIP(hipStreamWaitEvent(c->nstream, c->nev_in, 0));
    SWPS_TRY(comm_alltoallv(c, d_send, sb, d_recv, rb, c->nstream, c->stage, "all-to-all-v"));
    SWPS_HIP(hipEventRecord(c->nev_out, c->nstream));
    SWPS_HIP(hipStreamWaitEvent(nullptr, c->nev_out, 0));
    return SWPS_OK;
  }
  return comm_alltoallv(c, d_send, sb, d_recv, rb, s, c->stage, "all-to-all-v");
}

int swps_comm_ipc_info(swps_comm *c, uint64_t *out4) {
  if (!c || !out4) return fail(SWPS_E_CFG, "null argument");
  const IpcState *p = c->ipc.get();
  out4[0] = p ? 1 : 0;
  out4[1] = p ? p->slot : 0;
  out4[2] = p ? p->calls : 0;
  out4[3] = p ? p->bytes_remote : 0;
  return SWPS_OK;
}

int swps_table_route(swps_table *t, swps_comm *c, int32_t frag_num) {
  if (!t || !c) return fail(SWPS_E_CFG, "null argument");
  if (c->device != t->cfg.device) return fail(SWPS_E_CFG, "communicator and table are on different devices");
  if (frag_num < c->world) return fail(SWPS_E_CFG, "frag_num < world (hashfrag.h divides by frag_num / world)");
  SWPS_HIP(hipSetDevice(t->cfg.device));
  std::vector<uint32_t> map(frag_num);
  SWPS_TRY(swps_hashfrag_table(frag_num, c->world, map.data()));
  SWPS_TRY(upload(t->frag_map, map, t->stream));
  SWPS_HIP(hipStreamSynchronize(t->stream));
  t->comm = c;
  t->frag_num = frag_num;
  t->finished = false;
  return SWPS_OK;
}

int swps_finish(swps_table *t) {
  if (!t) return fail(SWPS_E_CFG, "null table");
  if (!t->comm) return SWPS_OK;
  SWPS_HIP(hipSetDevice(t->cfg.device));
  t->finished = true;
  for (;;) {  // serve the other ranks' rounds until every rank is finishing
    int ran = 0;
    SWPS_TRY(route_round(t, kOpFinish, nullptr, 0, nullptr, t->stream, &ran));
    if (ran == kOpFinish) break;
  }
  SWPS_HIP(hipStreamSynchronize(t->stream));
  return table_check_error(t, t->stream);
}

int swps_barrier(swps_table *t) {
  if (!t) return fail(SWPS_E_CFG, "null table");
  SWPS_HIP(hipSetDevice(t->cfg.device));
  SWPS_HIP(hipDeviceSynchronize());
  if (t->comm && t->comm->world > 1) {
    std::vector<int64_t> all(t->comm->world);
    const int64_t one = 1;
    SWPS_TRY(comm_allgather(t->comm, &one, all.data(), 8, t->stream));
  }
  return table_check_error(t, t->stream);
}

int swps_route_stats(swps_table *t, uint64_t *out6) {
  if (!t || !out6) return fail(SWPS_E_CFG, "null argument");
  for (int i = 0; i < 6; i++) out6[i] = t->rstats[i];
  return SWPS_OK;
}

}  // extern "C"
