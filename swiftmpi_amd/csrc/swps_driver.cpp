// Library-driven sharded app loop (swps_w2v_shard_comm / swps_lr_shard_comm):
// the lockstep minibatch exchange of SURVEY.md §8(e) issued by the library
// over its own communicator, so a C/C++ host (include/swiftmpi_compat.h's
// Word2VecApp / LRApp) trains on several GPUs without moving payloads itself.
// Per minibatch i, every rank (weak scaling: its own corpus; owner of the
// keys BasicHashFrag gives node rank+1):
//   serve stream S:  request(i) -> a2a keys -> serve_pull -> a2a values
//   compute stream C:   wait -> step(i): install, learn, mean gradients
//                       -> prep(i+1): records, sort, index (param-free)
//   S:  wait step(i) -> a2a gradients -> serve_push (one AdaGrad step per
//       source, in rank order; server.h:156-176)
// so every pull sees every earlier push (the reference's single-worker
// semantics, lockstep) and prep(i+1) overlaps push(i) / pull(i+1).  Ranks
// whose corpora have fewer minibatches run empty steps (steps_per_epoch =
// the maximum over ranks); per-step key counts come from the static batch
// schedules and are exchanged once at setup, so no step needs a handshake.
// The same protocol as swiftmpi_amd/dist.py's Python driver.
#include <algorithm>
#include <cstdlib>
#include <memory>

#include "swps_internal.h"

namespace swps {

ShardDriver::~ShardDriver() {
  if (ev_pull) (void)hipEventDestroy(ev_pull);
  if (ev_learn) (void)hipEventDestroy(ev_learn);
  if (ev_x0) (void)hipEventDestroy(ev_x0);
  if (ev_x1) (void)hipEventDestroy(ev_x1);
  if (S && S != ops.cs) {
    (void)hipStreamSynchronize(S);
    (void)hipStreamDestroy(S);
  }
}

int ShardDriver::setup() {
  rank = comm_rank(c);
  world = comm_world(c);
  // apps whose server work cannot move to another stream run everything on theirs
  if (ops.set_serve_stream) {
    // the serve stream (exchanges, owner kernels) at the highest priority, so prep(i+1) on the
    // compute stream does not delay the critical push -> pull chain: same-box A/B at world 1
    // (--sharded) 4.0e8 -> 4.29e8 words/s; SWPS_SERVE_PRIO=0: default priority
    const char *e = getenv("SWPS_SERVE_PRIO");
    if (!(e && atoi(e) == 0)) {
      int lo = 0, hi = 0;
      SWPS_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
      SWPS_HIP(hipStreamCreateWithPriority(&S, hipStreamNonBlocking, hi));
    } else {
      SWPS_HIP(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
    }
  } else
    S = ops.cs;
  SWPS_HIP(hipEventCreateWithFlags(&ev_pull, hipEventDisableTiming));
  SWPS_HIP(hipEventCreateWithFlags(&ev_learn, hipEventDisableTiming));
  SWPS_HIP(hipEventCreate(&ev_x0));
  SWPS_HIP(hipEventCreate(&ev_x1));
  uint64_t n = 0;
  std::vector<uint64_t> bc(1);
  (void)ops.batch_counts(ops.h, bc.data(), 0, &n);  // "buffer too small", but *n = the batch count
  nb = n;
  bc.assign(std::max<uint64_t>(nb * world, 1), 0);
  SWPS_TRY(ops.batch_counts(ops.h, bc.data(), bc.size(), &n));
  // steps per epoch = max over ranks; then everyone's [step][dst] counts
  std::vector<int64_t> nbs(world);
  const int64_t mine = (int64_t)nb;
  SWPS_TRY(comm_allgather(c, &mine, nbs.data(), 8, ops.cs));
  spe = 0;
  for (auto v : nbs) spe = std::max<uint64_t>(spe, (uint64_t)v);
  std::vector<uint64_t> mat(spe * world, 0), all(spe * world * world);
  std::copy(bc.begin(), bc.begin() + nb * world, mat.begin());
  if (spe) SWPS_TRY(comm_allgather(c, mat.data(), all.data(), spe * world * 8, ops.cs));
  send.assign(spe * world, 0);
  recv.assign(spe * world, 0);
  for (uint64_t st = 0; st < spe; st++)
    for (int r = 0; r < world; r++) {
      send[st * world + r] = all[((uint64_t)rank * spe + st) * world + r];  // I send to r
      recv[st * world + r] = all[((uint64_t)r * spe + st) * world + rank];  // r sends to me
    }
  // size the step buffers once (a grow inside a step would free memory in flight)
  uint64_t ms = 1, mr = 1;
  for (uint64_t st = 0; st < spe; st++) {
    uint64_t ns = 0, nr = 0;
    for (int r = 0; r < world; r++) {
      ns += send[st * world + r];
      nr += recv[st * world + r];
    }
    ms = std::max(ms, ns);
    mr = std::max(mr, nr);
  }
  const uint64_t vb = ops.width * ops.val_bytes, gb = ops.width * ops.grad_bytes;
  SWPS_TRY(keys.ensure(ms * 8));
  SWPS_TRY(myvals.ensure(ms * vb));
  SWPS_TRY(grads.ensure(ms * gb));
  SWPS_TRY(rkeys.ensure(mr * 8));
  SWPS_TRY(vals.ensure(mr * vb));
  SWPS_TRY(rgrads.ensure(mr * gb));
  step_keys = ms;
  step_rkeys = mr;
  // per-slot received keys (SWPS_KEY_CACHE=0: off), when they fit in 2 GiB
  rk_off.assign(spe + 1, 0);
  for (uint64_t st = 0; st < spe; st++) {
    uint64_t nr = 0;
    for (int r = 0; r < world; r++) nr += recv[st * world + r];
    rk_off[st + 1] = rk_off[st] + nr;
  }
  const char *kc = getenv("SWPS_KEY_CACHE");
  key_cache = !(kc && atoi(kc) == 0) && rk_off[spe] * 8 <= (2ULL << 30);
  // the gradient exchange in two all-to-alls (first halves of every segment as soon as the learner
  // has them, the rest after it), for apps whose learner computes them in two passes
  const char *sg = getenv("SWPS_SPLIT_GRADS");
  split_grads = ops.half_event != nullptr && !(sg && atoi(sg) == 0);
  if (key_cache) {
    SWPS_TRY(rk_cache.ensure(std::max<uint64_t>(rk_off[spe], 1) * 8));
    rk_valid.assign(spe, 0);
  }
  // opt-in (SWPS_SPLIT_PULL=1): forced at world 1 it costs 4.19e8 -> 4.05e8 words/s (same box;
  // 4.13e8 -> 3.95e8 with an assembly pass instead of the two-part install), and at the bench's
  // text8 shape only 6.6 % of a minibatch's keys are early, so at N = 8 it would hide ~25 MB of a
  // 1.1 GB exchange; at config 4's shape (34 % early) it hides ~0.4 GB per step
  const char *spl = getenv("SWPS_SPLIT_PULL");
  split_pull = key_cache && ops.late_mask && ops.set_slot && spe > 1 && spl && atoi(spl) != 0;
  if (split_pull)
    for (uint64_t st = 0; st < spe; st++) sp.emplace_back(new SplitSlot());
  return SWPS_OK;
}

// The early / late partition of slot st's pull, once (its second epoch): the owner flags the keys
// it serves at st that it also served at st-1 (late), sends the flags back to the requesters,
// and both sides keep their halves of the slot (keys and counts per peer; value positions).
int ShardDriver::split_prepare(uint64_t st) {
  const uint64_t prev = (st + spe - 1) % spe;
  const uint64_t *sk = &send[st * world], *rk = &recv[st * world];
  uint64_t n = 0, m = 0;
  for (int r = 0; r < world; r++) {
    n += rk[r];
    m += sk[r];
  }
  SWPS_TRY(sync());  // one-time per slot: the buffers below may grow
  DevMem flags, myflags;
  SWPS_TRY(flags.ensure(std::max<uint64_t>(n, 1)));
  SWPS_TRY(myflags.ensure(std::max<uint64_t>(m, 1)));
  SWPS_TRY(ops.late_mask(ops.h, (int64_t)(3 * st), (int64_t)(3 * prev), flags.as<uint8_t>(), n));
  SWPS_TRY(exchange(flags.p, rk, myflags.p, sk, 1, S, "early/late pull flags"));  // the owners' flags to their requesters
  std::vector<uint8_t> hf(n), hm(m);
  std::vector<uint64_t> keys(n);
  if (n) SWPS_HIP(hipMemcpyAsync(hf.data(), flags.p, n, hipMemcpyDeviceToHost, S));
  if (n) SWPS_HIP(hipMemcpyAsync(keys.data(), rk_cache.as<uint64_t>() + rk_off[st], n * 8, hipMemcpyDeviceToHost, S));
  if (m) SWPS_HIP(hipMemcpyAsync(hm.data(), myflags.p, m, hipMemcpyDeviceToHost, S));
  SWPS_HIP(hipStreamSynchronize(S));
  SplitSlot &e = *sp[st];
  e.es.assign(world, 0);
  e.ls.assign(world, 0);
  e.ed.assign(world, 0);
  e.ld.assign(world, 0);
  std::vector<uint64_t> ek, lk;
  uint64_t o = 0;
  for (int r = 0; r < world; r++)  // owner: my served keys, per source
    for (uint64_t j = 0; j < rk[r]; j++, o++) {
      if (hf[o]) {
        lk.push_back(keys[o]);
        e.ls[r]++;
      } else {
        ek.push_back(keys[o]);
        e.es[r]++;
      }
    }
  std::vector<uint32_t> pe, pl;
  o = 0;
  for (int r = 0; r < world; r++)  // requester: my keys at each owner, in my value order
    for (uint64_t j = 0; j < sk[r]; j++, o++) {
      if (hm[o]) {
        pl.push_back((uint32_t)o);
        e.ld[r]++;
      } else {
        pe.push_back((uint32_t)o);
        e.ed[r]++;
      }
    }
  e.ne = pe.size();
  e.nl = pl.size();
  SWPS_TRY(upload(e.ek, ek, S));
  SWPS_TRY(upload(e.lk, lk, S));
  SWPS_TRY(upload(e.pe, pe, S));
  SWPS_TRY(upload(e.pl, pl, S));
  const uint64_t vb = ops.width * ops.val_bytes;
  SWPS_TRY(evals[0].ensure(std::max<uint64_t>(e.ne, 1) * vb));
  SWPS_TRY(evals[1].ensure(std::max<uint64_t>(e.ne, 1) * vb));
  SWPS_TRY(lvals.ensure(std::max<uint64_t>(e.nl, 1) * vb));
  SWPS_HIP(hipStreamSynchronize(S));
  e.ready = true;
  return SWPS_OK;
}

// slot st's early values: served and exchanged into evals[ebuf] (S); the buffers alternate
int ShardDriver::serve_early(uint64_t st) {
  SplitSlot &e = *sp[st];
  const uint64_t vb = ops.width * ops.val_bytes;
  SWPS_TRY(ops.set_slot(ops.h, (int64_t)(3 * st + 1)));
  SWPS_TRY(ops.serve_pull(ops.h, e.ek.as<uint64_t>(), e.es.data(), 0, vals.p));
  SWPS_TRY(exchange(vals.p, e.es.data(), evals[ebuf].p, e.ed.data(), vb, S, "early pull values"));
  early_buf = ebuf;
  ebuf ^= 1;
  return SWPS_OK;
}

static std::vector<uint64_t> scaled(const uint64_t *k, int world, uint64_t w) {
  std::vector<uint64_t> b(world);
  for (int r = 0; r < world; r++) b[r] = k[r] * w;
  return b;
}

int ShardDriver::exchange(const void *d_send, const uint64_t *sk, void *d_recv, const uint64_t *rk, uint64_t w,
                          hipStream_t s, const char *phase) {
  if (world == 1 && d_send == d_recv) {  // an aliased world-1 exchange: nothing moves
    if (xprof) {
      bytes_total += sk[0] * w;
      calls++;
    }
    return SWPS_OK;
  }
  if (xprof) {
    SWPS_HIP(hipEventRecord(ev_x0, s));
    for (int r = 0; r < world; r++) {
      bytes_total += sk[r] * w;
      if (r != rank) bytes_remote += sk[r] * w;
    }
    calls++;
  }
  SWPS_TRY(comm_alltoallv(c, d_send, scaled(sk, world, w), d_recv, scaled(rk, world, w), s, stage, phase));
  if (xprof) {
    SWPS_HIP(hipEventRecord(ev_x1, s));
    SWPS_HIP(hipEventSynchronize(ev_x1));  // profiled runs only
    SWPS_TRY(comm_status(c));
    float ms = 0;
    SWPS_HIP(hipEventElapsedTime(&ms, ev_x0, ev_x1));
    xms += ms;
  }
  return SWPS_OK;
}

int ShardDriver::exchange_disp(const void *d_send, const std::vector<uint64_t> &sb, const std::vector<uint64_t> &so,
                               void *d_recv, const std::vector<uint64_t> &rb, const std::vector<uint64_t> &ro,
                               hipStream_t s, const char *phase) {
  if (xprof) {
    SWPS_HIP(hipEventRecord(ev_x0, s));
    for (int r = 0; r < world; r++) {
      bytes_total += sb[r];
      if (r != rank) bytes_remote += sb[r];
    }
    calls++;
  }
  SWPS_TRY(comm_alltoallv_disp(c, d_send, sb, so, d_recv, rb, ro, s, stage, phase));
  if (xprof) {
    SWPS_HIP(hipEventRecord(ev_x1, s));
    SWPS_HIP(hipEventSynchronize(ev_x1));  // profiled runs only
    SWPS_TRY(comm_status(c));
    float ms = 0;
    SWPS_HIP(hipEventElapsedTime(&ms, ev_x0, ev_x1));
    xms += ms;
  }
  return SWPS_OK;
}

int ShardDriver::full_pull() {
  SWPS_TRY(sync());  // the full pull reuses the step buffers
  // its request / serve_pull run on ops.cs like its exchanges (a second full pull would otherwise
  // find them on the serve stream S set below, unordered with the exchanges)
  if (ops.set_serve_stream) SWPS_TRY(ops.set_serve_stream(ops.h, nullptr));
  std::vector<uint64_t> cnt(world), all((size_t)world * world);
  uint64_t n = 0;
  SWPS_TRY(ops.request(ops.h, 1, cnt.data(), nullptr, &n));
  DevMem &fk = fp_keys, &frk = fp_rkeys, &fv = fp_vals, &fmv = fp_myvals;  // full-vocab sized, freed after
  SWPS_TRY(fk.ensure(std::max<uint64_t>(n, 1) * 8));
  SWPS_TRY(ops.request(ops.h, 1, cnt.data(), fk.as<uint64_t>(), &n));
  SWPS_TRY(comm_allgather(c, cnt.data(), all.data(), world * 8, ops.cs));
  std::vector<uint64_t> rc(world);
  uint64_t nr = 0;
  for (int r = 0; r < world; r++) nr += (rc[r] = all[(size_t)r * world + rank]);
  SWPS_TRY(frk.ensure(std::max<uint64_t>(nr, 1) * 8));
  SWPS_TRY(fv.ensure(std::max<uint64_t>(nr, 1) * ops.width * ops.val_bytes));
  SWPS_TRY(fmv.ensure(std::max<uint64_t>(n, 1) * ops.width * ops.val_bytes));
  SWPS_TRY(exchange(fk.p, cnt.data(), frk.p, rc.data(), 8, ops.cs, "full-pull keys"));
  SWPS_TRY(ops.serve_pull(ops.h, frk.as<uint64_t>(), rc.data(), 1, fv.p));
  SWPS_TRY(exchange(fv.p, rc.data(), fmv.p, cnt.data(), ops.width * ops.val_bytes, ops.cs, "full-pull values"));
  SWPS_TRY(ops.install(ops.h, fmv.p));
  SWPS_HIP(hipStreamSynchronize(ops.cs));
  SWPS_TRY(comm_status(c));
  fk.release();
  frk.release();
  fv.release();
  fmv.release();
  // server-side work of the steps goes to S from here on
  if (ops.set_serve_stream) SWPS_TRY(ops.set_serve_stream(ops.h, S));
  return SWPS_OK;
}

int ShardDriver::steps(uint64_t count) {
  const uint64_t vb = ops.width * ops.val_bytes, gb = ops.width * ops.grad_bytes;
  // one stream (apps without a serve stream: LR): its own order is the events' order, so the
  // cross-stream records and waits are skipped (each costs host time and a packet in the queue)
  const bool one = S == ops.cs;
  for (uint64_t k = 0; k < count; k++) {
    const uint64_t st = cursor % spe;
    const uint64_t *sk = &send[st * world], *rk = &recv[st * world];
    uint64_t ns = 0, nr = 0;
    for (int r = 0; r < world; r++) {
      ns += sk[r];
      nr += rk[r];
    }
    if (ns > step_keys || nr > step_rkeys) return fail(SWPS_E_STATE, "step larger than the setup's schedule");
    const bool mine = st < nb;
    // world 1: the owner's values are the learner's and its gradients the owner's, in the same
    // order — no self-copy (the exchange below sees send == recv); not with the split pull, whose
    // early serve rewrites vals while the step may still be installing them
    const bool alias = world == 1 && !split_pull;
    void *mv = alias ? vals.p : myvals.p, *rg = alias ? grads.p : rgrads.p;
    // ---- S: pull(i) (C's earlier work on these buffers is ordered by events) ----
    if (!one) SWPS_HIP(hipStreamWaitEvent(S, ev_learn, 0));
    // every rank runs the same steps, so every rank takes the same branch (the exchange is collective)
    const bool kc = key_cache && rk_valid[st];
    uint64_t *rkp = key_cache ? rk_cache.as<uint64_t>() + rk_off[st] : rkeys.as<uint64_t>();
    if (!kc) {
      if (mine && ns) {
        std::vector<uint64_t> cnt(world);
        uint64_t n = 0;
        SWPS_TRY(ops.request(ops.h, 0, cnt.data(), keys.as<uint64_t>(), &n));
      }
      SWPS_TRY(exchange(keys.p, sk, rkp, rk, 8, S, "pull keys"));
      if (key_cache) rk_valid[st] = 1;
    }
    // slot ids of the app's per-slot caches: 3*st the whole key set (pull and push), 3*st + 1 its
    // early and 3*st + 2 its late part
    const uint64_t prev = (st + spe - 1) % spe;
    bool split = false;
    if (split_pull && kc && rk_valid[prev]) {  // the slot's keys and both slots' row lookups exist
      if (sp[st]->ready)
        split = true;
      else
        SWPS_TRY(split_prepare(st));  // collective: every rank reaches it at the same step
    }
    if (split) {
      SplitSlot &e = *sp[st];
      if (!(early_pending && early_slot == st)) SWPS_TRY(serve_early(st));
      early_pending = false;
      SWPS_TRY(ops.set_slot(ops.h, (int64_t)(3 * st + 2)));
      SWPS_TRY(ops.serve_pull(ops.h, e.lk.as<uint64_t>(), e.ls.data(), 0, vals.p));
      SWPS_TRY(exchange(vals.p, e.ls.data(), lvals.p, e.ld.data(), vb, S, "late pull values"));
      const void *ev = evals[early_buf].p;
      if (ops.install_parts) {  // the step installs both parts itself (no assembly pass)
        if (mine && ns)
          SWPS_TRY(ops.install_parts(ops.h, ev, e.pe.as<uint32_t>(), e.ne, lvals.p, e.pl.as<uint32_t>(), e.nl));
      } else {
        SWPS_TRY(scatter_rows(lvals.p, e.pl.as<uint32_t>(), e.nl, vb, myvals.p, S));
        SWPS_TRY(scatter_rows(ev, e.pe.as<uint32_t>(), e.ne, vb, myvals.p, S));
      }
      split_steps++;
    } else {
      if (ops.set_slot) SWPS_TRY(ops.set_slot(ops.h, key_cache ? (int64_t)(3 * st) : -1));
      if (alias && key_cache && ops.pull_in_place && ops.set_slot) {  // world 1: the step reads the shard
        SWPS_TRY(ops.serve_pull(ops.h, rkp, rk, 0, nullptr));
      } else {
        SWPS_TRY(ops.serve_pull(ops.h, rkp, rk, 0, vals.p));
        SWPS_TRY(exchange(vals.p, rk, mv, sk, vb, S, "pull values"));
      }
    }
    if (!one) SWPS_HIP(hipEventRecord(ev_pull, S));
    // ---- C: learn(i), then prep(i+1) ----
    if (!one) SWPS_HIP(hipStreamWaitEvent(ops.cs, ev_pull, 0));
    if (mine) SWPS_TRY(ops.step(ops.h, ns ? mv : nullptr, ns ? grads.p : nullptr));
    if (!one) SWPS_HIP(hipEventRecord(ev_learn, ops.cs));
    const uint64_t nxt = (cursor + 1) % spe;
    if (ops.prep && k + 1 < count && nxt < nb) SWPS_TRY(ops.prep(ops.h));
    // ---- S: the next step's early pull, while this one learns (its rows cannot change at push(i)) ----
    if (split_pull && k + 1 < count && sp[nxt]->ready && rk_valid[nxt] && rk_valid[st]) {
      SWPS_TRY(serve_early(nxt));
      early_pending = true;
      early_slot = nxt;
    }
    if (ops.set_slot) SWPS_TRY(ops.set_slot(ops.h, key_cache ? (int64_t)(3 * st) : -1));  // push(i)'s keys
    // ---- S: push(i) ----
    // split_grads is the same on every rank (build, environment, world), so every rank issues the
    // same two collectives; eh (the learner ran its two passes) only decides when the first starts
    hipEvent_t eh = (mine && ops.half_event) ? (hipEvent_t)ops.half_event(ops.h) : nullptr;
    if (split_grads && world > 1) {
      // first halves of every peer's segment (counts floor(n/2), the learner's split), then the rest
      std::vector<uint64_t> sb(world), so(world), rb(world), ro(world);
      uint64_t a = 0, b = 0;
      for (int r = 0; r < world; r++) {
        sb[r] = (sk[r] / 2) * gb;
        so[r] = a * gb;
        rb[r] = (rk[r] / 2) * gb;
        ro[r] = b * gb;
        a += sk[r];
        b += rk[r];
      }
      if (eh) SWPS_HIP(hipStreamWaitEvent(S, eh, 0));
      else if (!one) SWPS_HIP(hipStreamWaitEvent(S, ev_learn, 0));
      SWPS_TRY(exchange_disp(grads.p, sb, so, rgrads.p, rb, ro, S, "push gradients"));
      for (int r = 0; r < world; r++) {
        so[r] += sb[r];
        ro[r] += rb[r];
        sb[r] = (sk[r] - sk[r] / 2) * gb;
        rb[r] = (rk[r] - rk[r] / 2) * gb;
      }
      if (!one) SWPS_HIP(hipStreamWaitEvent(S, ev_learn, 0));
      SWPS_TRY(exchange_disp(grads.p, sb, so, rgrads.p, rb, ro, S, "push gradients"));
    } else {
      if (!one) SWPS_HIP(hipStreamWaitEvent(S, ev_learn, 0));
      SWPS_TRY(exchange(grads.p, sk, rg, rk, gb, S, "push gradients"));
    }
    SWPS_TRY(ops.serve_push(ops.h, rkp, rg, rk));
    if (ops.set_slot) SWPS_TRY(ops.set_slot(ops.h, -1));
    cursor++;
  }
  if (S != ops.cs) {
    SWPS_HIP(hipEventRecord(ev_learn, S));  // the next call's C work waits for this push
    SWPS_HIP(hipStreamWaitEvent(ops.cs, ev_learn, 0));
  }
  return SWPS_OK;
}

int ShardDriver::sync() {
  SWPS_HIP(hipStreamSynchronize(S));  // returns once the RCCL guard aborts a stuck exchange
  SWPS_HIP(hipStreamSynchronize(ops.cs));
  return comm_status(c);
}

}  // namespace swps
