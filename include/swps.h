/*
 * swps.h — C ABI of the MI355X-native SwiftMPI hot path (libswps.so).
 *
 * One process per GPU.  The library owns all device memory; callers pass
 * plain pointers and sizes (device pointers where noted "d_", host pointers
 * otherwise).  Every function returns 0 (SWPS_OK) or a negative SWPS_E_*
 * code and never aborts; the message of the last failure on the calling
 * thread is returned by swps_last_error().
 *
 * Reference interfaces replaced (paths relative to logicxin/SwiftMPI src/):
 *   swps_table_*      SparseTable / SparseTableShard   parameter/sparsetable.h:17-149
 *                     + the server's pull/push handlers cluster/server.h:106-176
 *   swps_pull         GlobalPullAccess::pull_with_barrier
 *                         parameter/global_pull_access.h:28-43  (+ accessmethod.h:63-70)
 *   swps_push         GlobalPushAccess::push_with_barrier
 *                         parameter/global_push_access.h:26-43  (+ accessmethod.h:102-121)
 *   swps_assign/load  SparseTable::assign, ClusterServer::load  sparsetable.h:117, server.h:49-62
 *   swps_dump         SparseTable::output                        sparsetable.h:127-132
 *   swps_save/restore binary checkpoint (the reference has only the 6-digit text dump of
 *   swps_w2v_save_state  sparsetable.h:63-70 and cannot resume)
 *   swps_to_node_id   BasicHashFrag::to_node_id                  cluster/hashfrag.h:51-56
 *   swps_w2v_*        Word2Vec<MiniBatch>::train / MiniBatch     apps/word2vec/word2vec_global.h:284-731
 *   swps_lr_*         LR::train / learn_instance / predict       apps/logistic/lr.cpp:157-398
 *   swps_s2v_*        Sent2Vec::train / learn_instance           apps/sent2vec/sent2vec.cpp:37-181
 */
#ifndef SWPS_H_
#define SWPS_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes --------------------------------------------------------- */
#define SWPS_OK 0
#define SWPS_E_OOM (-1)         /* device or host allocation failed / table full */
#define SWPS_E_BADKEY (-2)      /* push of a key the table never saw (server.h CHECK) */
#define SWPS_E_HIP (-3)         /* HIP runtime error */
#define SWPS_E_RCCL (-4)        /* RCCL error */
#define SWPS_E_CFG (-5)         /* invalid configuration */
#define SWPS_E_STATE (-6)       /* call out of order */
#define SWPS_E_UNSUPPORTED (-7) /* input whose reference behaviour is undefined */
#define SWPS_E_IO (-8)          /* file I/O */

const char *swps_last_error(void);
int swps_version(void);
/* sha256 (hex) of the sources the library was built from: every file of
 * swiftmpi_amd/csrc/ and this header, by name then content (swiftmpi_amd/build.py
 * source_hash); a prebuilt library is checked against the checked-out tree */
const char *swps_build_hash(void);

/* ---- parameter table (server shard in HBM) ------------------------------ */
/* Layouts: one row per key.
 *   SWPS_LAYOUT_W2V : [h(D) | v(D) | h2sum(D) | v2sum(D)]   (WParam, word2vec_global.h:34-48)
 *     pull value  = [h(D) | v(D)]                           (WLocalParam's values)
 *     push value  = [mean h_grad(D) | mean v_grad(D)] fp64  (WLocalGrad's mean, :122-134)
 *     push rule   = AdaGrad ascent                          (:176-185)
 *   Value BLOCKS, not the reference's byte stream: its BinaryBuffer wire
 *   interleaves h[i], v[i] per element (word2vec_global.h:129-132, 144-147)
 *   after each key.  The element type matches the wire's (fp64); a bridge to
 *   reference peers must (de)interleave — swiftmpi_compat.h's WLocalParam /
 *   WLocalGrad do, see INTEGRATION.md. */
/*
 *   SWPS_LAYOUT_LR  : [w | grad2sum]                         (LRParam, lr.cpp:7-10)
 *     pull value  = [w]; push value = [mean grad] fp32;  AdaGrad (lr.cpp:68-75)
 */
#define SWPS_LAYOUT_W2V 0
#define SWPS_LAYOUT_LR 1

#define SWPS_F32 0 /* fp32 storage, fp64 arithmetic */
#define SWPS_F64 1 /* fp64 storage (the reference's Vec precision) */

/* key initialisation on a pull miss (PullAccessMethod::init_param) */
#define SWPS_INIT_ZERO 0
#define SWPS_INIT_HASH 1 /* W2V: (u-0.5)/D, LR: u in [0,1); u from (seed,key,i) */
#define SWPS_INIT_FLCG 2 /* LR only: w = global_random().gen_float() per new key in the order the
                          * call lists them (LRPullAccessMethod::init_param, lr.cpp:48-50; random.h:
                          * 33-36) — the float LCG continues across calls; `seed` = its state before
                          * the first draw (0: the reference's ULONG_MAX / 2) */

/* push rule (PushAccessMethod::apply_push_value, accessmethod.h:26-35) */
#define SWPS_PUSH_ADAGRAD 0 /* W2V word2vec_global.h:176-185, LR lr.cpp:68-75: g2 += g*g;
                             * w += lr*g/sqrt(g2+fudge) — every reference app's rule */
#define SWPS_PUSH_SGD 1     /* w += lr*g (the accumulators are left alone); PS level only:
                             * the app contexts (swps_w2v_*, swps_lr_*) reject such tables */

typedef struct swps_table swps_table;

typedef struct {
  int32_t device;     /* HIP device ordinal */
  int32_t layout;     /* SWPS_LAYOUT_* */
  int32_t dtype;      /* SWPS_F32 / SWPS_F64 */
  int32_t dim;        /* D (W2V) — ignored for LR */
  uint64_t capacity;  /* max keys held by this shard */
  float learning_rate; /* server.initial_learning_rate */
  float fudge;        /* AdaGrad fudge factor (reference: 1e-6f) */
  int32_t init_mode;  /* SWPS_INIT_* */
  uint64_t seed;
  int32_t push_rule;  /* SWPS_PUSH_* (0 = AdaGrad) */
} swps_table_cfg;

int swps_table_create(const swps_table_cfg *cfg, swps_table **out);
int swps_table_destroy(swps_table *t);
int swps_table_size(swps_table *t, uint64_t *nkeys);
int swps_table_sync(swps_table *t);
/* per-key element counts of a full row / a pull value / a push value */
int swps_table_row_elems(swps_table *t, int32_t *row, int32_t *pull, int32_t *push);

/* Batched pull: find-or-insert each key (keys in one call must be distinct,
 * as the reference's std::unordered_set key sets are) and write its pull
 * value to d_vals[n][pull elems] in the table dtype. */
int swps_pull(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_vals);
/* Batched push: apply the push rule with the mean gradients d_grads[n][push
 * elems] (fp64 for W2V, fp32 for LR).  Unknown key -> SWPS_E_BADKEY. */
int swps_push(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_grads);
/* The same with HOST arrays in the reference's wire types (W2V: fp64
 * [h|v] pull values and [mean h_grad|mean v_grad] push values; LR: fp32),
 * staged through HBM by the library — the form a C++ PS client binds
 * (include/swiftmpi_compat.h: GlobalPullAccess / GlobalPushAccess). */
int swps_pull_h(swps_table *t, const uint64_t *keys, uint64_t n, void *vals);
int swps_push_h(swps_table *t, const uint64_t *keys, uint64_t n, const void *grads);
/* Host forms of a key probe and a whole-row assignment on a local (unrouted) table:
 * SparseTableShard::find / ::assign (sparsetable.h:28-48).  present[i] = 1 when the shard holds
 * keys[i]; rows[n][row elems] in fp64, converted to the table dtype (no init_param draws). */
int swps_table_find_h(swps_table *t, const uint64_t *keys, uint64_t n, uint8_t *present);
int swps_assign_h(swps_table *t, const uint64_t *keys, uint64_t n, const double *rows);
/* Stream-ordered forms of swps_pull / swps_push on a local (unrouted) table:
 * issued on `stream` (a hipStream_t of the table's device; NULL = the
 * table's own stream) with no host sync.  Table-full / unknown-key errors are
 * latched on the device and reported by the next swps_table_sync or
 * swps_barrier.  The table's scratch buffers are shared: calls on different
 * streams must be ordered by the caller (events).  A routed table
 * (swps_table_route) needs the per-owner key counts on the host, so these
 * forms sync once per call there, like swps_pull / swps_push. */
int swps_pull_async(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_vals, void *stream);
int swps_push_async(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_grads, void *stream);
/* Overwrite / read full rows (table dtype, d_rows[n][row elems]). */
int swps_assign(swps_table *t, const uint64_t *d_keys, uint64_t n, const void *d_rows);
int swps_export(swps_table *t, const uint64_t *d_keys, uint64_t n, void *d_rows);
/* all keys currently held (host array of capacity cap) */
int swps_table_keys(swps_table *t, uint64_t *keys, uint64_t cap, uint64_t *n);
/* Text dump/load in the reference format (sparsetable.h:63-70):
 *   W2V: "key\tv0 v1 ... v(D-1)\th0 ... h(D-1)\n"   (word2vec_global.h:102-112)
 *   LR : "key\tw\n"                                  (lr.cpp:24-27)
 * at ostream default precision (6 significant digits). load keeps only keys
 * owned by `node_id` under the hash-frag map (server.h:49-62); node_id 0 or
 * world 1 keeps all. */
int swps_dump(swps_table *t, const char *path);
int swps_load(swps_table *t, const char *path, int32_t frag_num, int32_t world, int32_t node_id);
/* Binary snapshot: every key and every row element bit for bit (incl. the
 * AdaGrad sums the text dump drops), with a trailing checksum.  restore
 * verifies the whole file (magic, layout/dtype/dim, checksum) before it
 * assigns any row, and keeps only node_id's keys like swps_load. */
int swps_save(swps_table *t, const char *path);
int swps_restore(swps_table *t, const char *path, int32_t frag_num, int32_t world, int32_t node_id);

/* ---- key -> node map (BasicHashFrag) ------------------------------------ */
uint64_t swps_fmix64(uint64_t x);                       /* utils/HashFunction.h:16-24 */
uint64_t swps_bkdr(const char *s);                      /* utils/string.h:130-137 */
int swps_hashfrag_table(int32_t frag_num, int32_t num_nodes, uint32_t *out); /* hashfrag.h:33-49 */
int swps_to_node_id(const uint64_t *keys, uint64_t n, int32_t frag_num, const uint32_t *table,
                    int32_t *out);                      /* hashfrag.h:51-56 (host) */

/* ---- communicator (replaces src/transfer + the MPI bootstrap) ------------
 * One process per GPU.  Two transports:
 *   RCCL (xGMI): swps_comm_create_rccl from a 128-byte unique id that rank 0
 *     makes (swps_comm_unique_id) and the caller distributes — with
 *     swps_comm_bootstrap_tcp (rank 0 serves it on addr:port; the launcher's
 *     MASTER_ADDR / MASTER_PORT) or any channel of its own.  Payloads move
 *     device to device with ncclSend / ncclRecv groups.
 *   host: the caller's all-gather and all-to-all-v callbacks on host buffers
 *     (MPI, gloo, sockets, ...); payloads are staged through host memory.
 *     Lets several ranks share one GPU (RCCL refuses that). */
typedef struct swps_comm swps_comm;
#define SWPS_COMM_ID_BYTES 128
typedef struct {
  void *ctx;
  /* every rank contributes `bytes` bytes; out receives world*bytes, rank order */
  int (*allgather)(void *ctx, const void *in, void *out, uint64_t bytes);
  /* send holds the blocks for ranks 0..world-1 back to back (send_bytes[r]
   * each); recv receives the blocks from ranks 0..world-1 (recv_bytes[r]) */
  int (*alltoallv)(void *ctx, const void *send, const uint64_t *send_bytes, void *recv, const uint64_t *recv_bytes);
} swps_transport;

int swps_comm_unique_id(uint8_t *id); /* ncclGetUniqueId: one rank calls it */
/* rank 0 makes the id and sends it to every other rank over TCP (it listens
 * on port; the others connect to addr:port, retrying for up to timeout_ms);
 * every rank returns with the same id */
int swps_comm_bootstrap_tcp(const char *addr, int32_t port, int32_t rank, int32_t world, int32_t timeout_ms,
                            uint8_t *id);
int swps_comm_create_rccl(const uint8_t *id, int32_t rank, int32_t world, int32_t device, swps_comm **out);
int swps_comm_create_host(const swps_transport *tr, int32_t rank, int32_t world, int32_t device, swps_comm **out);
/* the library's own host transport: TCP, a star through rank 0 (it listens
 * on addr:port; the others connect, retrying for up to timeout_ms).  For
 * jobs without RCCL: several ranks on one GPU, host-only interconnects. */
int swps_comm_create_tcp(const char *addr, int32_t port, int32_t rank, int32_t world, int32_t device,
                         int32_t timeout_ms, swps_comm **out);
int swps_comm_destroy(swps_comm *c);
int swps_comm_info(swps_comm *c, int32_t *rank, int32_t *world);
/* the communicator's transport (SWPS_COMM_RCCL / _TCP / _HOST) and its rank count as the
 * transport reports it (RCCL: ncclCommCount) */
#define SWPS_COMM_RCCL 1
#define SWPS_COMM_TCP 2
#define SWPS_COMM_HOST 3
int swps_comm_transport(swps_comm *c, int32_t *kind, int32_t *ranks);
/* RCCL deadline (no reference counterpart: its ZeroMQ requests block forever, transfer.h:86-241).
 * An RCCL communicator is non-blocking and guarded: its initialisation and every exchange must
 * retire within `seconds` (default 120, env SWPS_COMM_TIMEOUT_S); otherwise — or on an RCCL
 * asynchronous error — the library aborts the communicator (ncclCommAbort: a rank waiting on a
 * lost peer stops waiting), prints "swps: rank R of N: <exchange> ..." to stderr, and every later
 * call on it (and on tables / app contexts routed over it) fails with SWPS_E_RCCL and that
 * message.  swps_comm_check reports that state; swps_comm_abort aborts on the caller's behalf (a
 * launcher that saw a sibling rank die).  The TCP transport's deadline is its timeout_ms. */
int swps_comm_set_timeout(swps_comm *c, double seconds);
int swps_comm_check(swps_comm *c);
int swps_comm_abort(swps_comm *c, const char *why);
/* Device-initiated all-to-all-v over IPC-mapped peer memory (opt-in, collective; the ranks of one
 * node, world <= 8; replaces the payload path of every later exchange on this communicator — the
 * reference's ZeroMQ request / response payloads, transfer.h:86-241, as the pull / push traffic of
 * global_pull_access.h:28-107 and server.h:156-176).  Each rank allocates an inbox of
 * world x 2 x slot_bytes (0: SWPS_COMM_IPC_SLOT_MB, default 4 MiB) and control words in uncached
 * device memory and maps every peer's through hipIpcGetMemHandle / hipIpcOpenMemHandle; one
 * exchange is then one kernel on the caller's stream, with no host synchronisation and no RCCL or
 * host-transport call (headers and counts still use the communicator's transport).  Segments
 * larger than a slot stream through it in rounds.  Waits are bounded by the communicator's
 * deadline (swps_comm_set_timeout): a lost peer makes the next call fail with SWPS_E_RCCL. */
int swps_comm_enable_ipc(swps_comm *c, uint64_t slot_bytes);
/* out4 = {enabled, slot bytes, exchanges issued, bytes sent to other ranks} */
int swps_comm_ipc_info(swps_comm *c, uint64_t *out4);
/* Collective all-to-all-v of device buffers on `stream` (a hipStream_t; NULL: the null stream):
 * send holds the segments for ranks 0..world-1 back to back (send_bytes[r] each), recv receives
 * rank r's segment at the sum of recv_bytes[0..r-1].  Over RCCL and IPC it is stream-ordered and
 * returns at once; over a host transport it returns once the exchange is done. */
int swps_comm_alltoallv(swps_comm *c, const void *d_send, const uint64_t *send_bytes, void *d_recv,
                        const uint64_t *recv_bytes, void *stream);

/* ---- key-sharded table (the GPU-to-shard map, src/cluster) --------------
 * swps_table_route binds a local shard to a communicator: this table then
 * serves the keys BasicHashFrag (hashfrag.h:33-56, S = world) maps to node
 * rank+1, and swps_pull / swps_push / swps_pull_h / swps_push_h /
 * swps_*_async become COLLECTIVE: keys are grouped by owner, exchanged
 * (all-to-all-v), owners find-or-insert / apply the push rule, pull values
 * come back in the caller's key order (GlobalPullAccess::pull_with_barrier,
 * global_pull_access.h:46-107; GlobalPushAccess::push_with_barrier,
 * global_push_access.h:48-96; the server handlers server.h:129-176).  An
 * owner applies the pushes of several sources for one key as separate steps
 * in source-rank order (the reference: one step per worker request).
 * Every rank must make the same sequence of calls; n = 0 is allowed and
 * still joins the exchange.  A rank whose worker is done calls swps_finish:
 * it keeps serving the other ranks' pulls / pushes and returns once every
 * rank has called it (the reference's servers outlive their workers). */
int swps_table_route(swps_table *t, swps_comm *c, int32_t frag_num);
int swps_finish(swps_table *t);
/* routed: every rank's earlier calls on this table have retired (all ranks
 * call it); local: swps_table_sync.  Reports latched device errors. */
int swps_barrier(swps_table *t);
/* routed-call counters: [rounds, keys sent, keys sent to other ranks,
 * payload bytes sent, payload bytes sent to other ranks, keys served] */
int swps_route_stats(swps_table *t, uint64_t *out6);

/* ---- word2vec CBOW negative sampling (apps/word2vec) --------------------- */
typedef struct swps_w2v swps_w2v;

#define SWPS_KEY_BKDR 0 /* word2vec_global.h:205-207 hash_fn */
#define SWPS_KEY_ATOI 1 /* word2vec.h:221 hash_fn2 */

#define SWPS_W2V_INIT_REF 0   /* reference: glibc rand() stream, _local_keys order */
#define SWPS_W2V_INIT_TABLE 1 /* keep whatever the table holds (HASH/ZERO/loaded) */

typedef struct {
  int32_t window;              /* word2vec.window */
  int32_t negative;            /* word2vec.negative */
  int32_t min_sentence_length; /* word2vec.min_sentence_length */
  int32_t minibatch;           /* worker.minibatch (lines) */
  float sample;                /* word2vec.sample (<0: no subsampling) */
  float alpha;                 /* word2vec.learning_rate */
  uint64_t unigram_size;       /* table_size (reference: 1e8) */
  int32_t key_mode;            /* SWPS_KEY_* */
  int32_t init_mode;           /* SWPS_W2V_INIT_* */
  uint32_t rand_seed;          /* glibc srand seed (reference: 1) */
  uint64_t rand_offset;        /* rand() calls before the first pull (reference: 2 port binds) */
  int32_t fp64_intermediates;  /* fp32 tables, the type of learn_instance's intermediates neu1/neu1e:
                                * SWPS_INTER_FP64 (1): fp64 like the reference's Vec (parity mode);
                                * SWPS_INTER_FP32 (0): fp32 (fast mode); SWPS_INTER_BFP40 (2) / _BFP32 (3):
                                * block floating point rows — int32 (+ int8) mantissas under one exponent
                                * per row, 5 (4) B/element, 2^-40 (2^-32) of the row's largest element —
                                * with fp64 sums, mean and push payload (dim % 4 == 0, dim <= 512).
                                * fp64 tables: always fp64 */
  int32_t profile;             /* 1: time kernels with HIP events */
  int32_t minibatch_vocab;     /* 0: apps/word2vec/word2vec_global.h (w2v.cpp): one vocab and unigram
                                * table for the corpus, a full-vocab worker cache, B+3-line gather windows;
                                * 1: apps/word2vec/word2vec.h's MiniBatch (w2v_local.cpp): per-minibatch
                                * vocab and table (std::map order), B+1-line windows, to_sample over the
                                * never-reset _num_words */
  int32_t sampler;             /* SWPS_SAMPLER_TABLE (the reference's cumulative unigram^0.75 table,
                                * bit-exact draws) or SWPS_SAMPLER_ALIAS (Walker/Vose alias table over the
                                * same weights: V x 8 B instead of table_size x 4 B, one L2-resident read per
                                * draw; same LCG consumption, different words — a non-parity fast mode) */
  int32_t host_ingest;         /* 0: corpus ingest on the GPU (tokenize, hash, vocab counts, the minibatch
                                * key sets; bit-identical to the host restatement); 1: on the host (kept
                                * for A/B and parity tests; minibatch_vocab mode always ingests on the host) */
} swps_w2v_cfg;

#define SWPS_INTER_FP32 0
#define SWPS_INTER_FP64 1
#define SWPS_INTER_BFP40 2
#define SWPS_INTER_BFP32 3

#define SWPS_SAMPLER_TABLE 0
#define SWPS_SAMPLER_ALIAS 1

/* The table must use SWPS_LAYOUT_W2V; ctx is bound to the table's device. */
int swps_w2v_create(swps_table *t, const swps_w2v_cfg *cfg, swps_w2v **out);
int swps_w2v_destroy(swps_w2v *w);
/* Corpus ingest.  text: one instance per line, words split on ' ' only.
 * tokens: word ids into word_keys (the key each word string hashes to);
 * line_off has nlines+1 entries. */
int swps_w2v_load_text(swps_w2v *w, const char *path);
int swps_w2v_load_tokens(swps_w2v *w, const uint32_t *word_ids, uint64_t ntok, const uint64_t *line_off,
                         uint64_t nlines, const uint64_t *word_keys, uint64_t nwords);
/* introspection (tests): every token's vid and line (host arrays of cap >= ntok) */
int swps_w2v_corpus(swps_w2v *w, int32_t *vid, int32_t *line, uint64_t cap);
/* batch b of the epoch schedule: its lines [lines2[0], lines2[1]) and its gathered key set (vids,
 * ascending; sharded contexts: grouped by owner) into out[cap], count via *n */
int swps_w2v_batch_keys(swps_w2v *w, uint64_t b, int32_t *out, uint64_t cap, uint64_t *n, uint64_t *lines2);
/* vocab in _wordids order (vid order): keys[V], counts[V]; V via *n */
int swps_w2v_vocab(swps_w2v *w, uint64_t *keys, int32_t *counts, uint64_t cap, uint64_t *n);
int swps_w2v_info(swps_w2v *w, uint64_t *out8); /* V, train_words, nlines, ntok, nbatches, max_batch_tok, lstate, fstate */
/* first full pull: insert every vocab key (init per cfg.init_mode) and fill the cache */
int swps_w2v_init(swps_w2v *w);
/* Train the next `count` minibatches of the per-epoch schedule
 * (word2vec_global.h:591-651); the batch cursor wraps into the next epoch. */
int swps_w2v_train_batches(swps_w2v *w, uint64_t count);
int swps_w2v_train_epochs(swps_w2v *w, int32_t niters);
int swps_w2v_sync(swps_w2v *w);
/* cumulative stats: [batches, kept positions, train words, gradient records, lstate, fstate,
 *  pulled keys, pushed keys, context rows read, target rows read]; the two row counts
 *  (roofline accounting) advance only while swps_w2v_set_profile is on */
int swps_w2v_stats(swps_w2v *w, uint64_t *out10);
/* cumulative work of the segmented gradient sums (k_gather + k_combine), for the
 * roofline: [gradient records summed (key in the batch), gather items (chunks of <= 128
 * records of one key and kind)] (no reference counterpart: measurement only) */
int swps_w2v_gather_stats(swps_w2v *w, uint64_t *out2);
/* the same split by who sums them, for the roofline of the fused sums + push: [gradient
 * records, items, records of multi-chunk (key, kind) runs (k_gather_t's share when the push
 * is fused), items of those runs, batches pushed by the fused in-place k_push_thp, batches
 * with gradient sums, batches whose mean gradients (sharded learner) came from the fused
 * k_push_thp, batches whose multi-chunk gather ran beside the push on a side stream]
 * (measurement only) */
int swps_w2v_sum_stats(swps_w2v *w, uint64_t *out8);
/* rows of all vocab keys in vid order, host buffer [V][4D] fp64 */
int swps_w2v_get_params(swps_w2v *w, double *out);
/* set h,v of all vocab keys (vid order, host [V][2D] fp64), zero h2/v2, refresh the cache */
int swps_w2v_set_params(swps_w2v *w, const double *hv);
/* unigram table entries (vids) at host-given slots */
int swps_w2v_unigram_at(swps_w2v *w, const uint64_t *idx, uint64_t n, uint32_t *out);
/* negative-draw trace of the next traced batch (vids), -1 = cleared */
int swps_w2v_trace_negatives(swps_w2v *w, uint64_t cap);
int swps_w2v_negatives(swps_w2v *w, int64_t *out, uint64_t cap, uint64_t *n);
/* per-kernel device time (ms) and launch counts since the last reset:
 * out[2*k] = ms, out[2*k+1] = launches for k in {plan, forward, sort, gather, push, pull, records} */
int swps_w2v_kernel_times(swps_w2v *w, double *out14, int32_t reset);
/* switch HIP-event kernel timing on/off (syncs the stream) */
int swps_w2v_set_profile(swps_w2v *w, int32_t on);
/* the HIP stream all of this context's work is issued on */
void *swps_w2v_stream(swps_w2v *w);
/* Worker checkpoint (with swps_save of its table, an exact resume point at
 * any batch boundary): batch cursor, both LCG streams at the epoch start,
 * counters and the worker cache (the stale rows negatives outside the batch
 * key set read), plus config and corpus fingerprints.  restore_state needs a
 * fresh context (corpus loaded, not initialised; sharded contexts already
 * swps_w2v_shard-ed) whose table already holds the vocab rows (swps_restore):
 * a different corpus or config fails with SWPS_E_CFG. */
int swps_w2v_save_state(swps_w2v *w, const char *path);
int swps_w2v_restore_state(swps_w2v *w, const char *path);

/* ---- sharded mode (several GPUs; the caller moves the payloads) ---------
 * Every rank = a worker with its own corpus + a server for the keys whose
 * BasicHashFrag node is rank+1 (hashfrag.h:33-56).  Per batch:
 *   swps_w2v_request     keys of the next batch grouped by owner rank (u64)
 *   -> all-to-all ->     swps_w2v_serve_pull (owner: [n][h|v] pull values)
 *   -> all-to-all ->     swps_w2v_step       (install values, learn, emit
 *                                             mean gradients [U][h|v])
 *   -> all-to-all ->     swps_w2v_serve_push (owner: AdaGrad per source rank,
 *                                             sources in rank order)
 * Initial full pull: swps_w2v_request(init=1) -> serve_pull(insert=1) ->
 * swps_w2v_install_init.  Tables must use SWPS_INIT_HASH (the reference's
 * rand() order would depend on message arrival). */
int swps_w2v_shard(swps_w2v *w, int32_t rank, int32_t world, int32_t frag_num);
/* per-batch key counts per owner: out[nb][world] */
int swps_w2v_batch_counts(swps_w2v *w, uint64_t *out, uint64_t cap, uint64_t *nb);
/* counts[world] (host); keys into d_keys (device, may be NULL to query n) */
int swps_w2v_request(swps_w2v *w, int32_t init, uint64_t *counts, uint64_t *d_keys, uint64_t *n);
/* keys from all sources concatenated in rank order, src_counts[world] (host) */
int swps_w2v_serve_pull(swps_w2v *w, const uint64_t *d_keys, const uint64_t *src_counts, int32_t insert,
                        void *d_vals);
int swps_w2v_install_init(swps_w2v *w, const void *d_vals);
/* d_grads: mean gradients [U][h|v] in the context's intermediate type — fp64
 * (the reference's wire format; SWPS_INTER_FP64 and the BFP modes) unless the table is
 * SWPS_F32 with SWPS_INTER_FP32 (fast mode), then fp32 (half the exchange bytes). */
int swps_w2v_step(swps_w2v *w, const void *d_vals, void *d_grads);
/* Prepare the next minibatch's parameter-independent half (epoch plan, local
 * key map, learn_instance's draws as position/gradient records, the sorted
 * inverted index) on the compute stream; swps_w2v_step / train_batches do it
 * themselves when it was not done.  Issued right after a step, it overlaps
 * that step's push and the next pull (sharded mode). */
int swps_w2v_prep(swps_w2v *w);
/* d_keys: the keys received for the matching serve_pull (src_counts as there) */
int swps_w2v_serve_push(swps_w2v *w, const uint64_t *d_keys, const void *d_grads, const uint64_t *src_counts);
/* Issue request / serve_pull / serve_push on `stream` (a hipStream_t of the
 * context's device; NULL = the compute stream, the default).  The caller
 * orders the two streams (the pipelined driver in swiftmpi_amd/dist.py). */
int swps_w2v_set_serve_stream(swps_w2v *w, void *stream);
/* Library-driven sharded mode: swps_w2v_shard for comm's rank / world, and
 * the library runs the exchange itself over `comm` — swps_w2v_init is the
 * first full pull, swps_w2v_train_batches / _epochs run lockstep minibatches
 * (collective: every rank calls them with the same count; ranks with fewer
 * minibatches per epoch run empty steps, steps per epoch = the maximum over
 * ranks), with the server work and exchanges on a second stream and the next
 * minibatch's parameter-independent half overlapping them.  The table may be
 * the local shard or one routed over the same comm. */
int swps_w2v_shard_comm(swps_w2v *w, swps_comm *comm, int32_t frag_num);
/* exchange accounting of the library-driven mode: out4 = [bytes sent to other
 * ranks, bytes sent in all, exchanges, ms of exchange on the serve stream]
 * since the last reset; on = 1 / 0 switches the (per-exchange syncing) event
 * timing on / off and resets, -1 only reads */
int swps_w2v_exchange_stats(swps_w2v *w, int32_t on, double *out4);

/* ---- host-only helpers (no device needed; used by the CPU test-suite) ---- */
/* run-length form of gen_unigram_table (word2vec_global.h:467-497): start slot
 * of each word in vocab order (V+1 entries, starts[V] = table_size) */
int swps_unigram_starts(const uint64_t *keys, const int32_t *counts, uint64_t V, uint64_t table_size,
                        uint64_t *starts);
/* glibc rand() after srand(seed), `skip` outputs discarded (Vec::randInit's stream) */
int swps_glibc_rand(uint32_t seed, uint64_t skip, uint64_t n, int32_t *out);

/* ---- sent2vec (apps/sent2vec/sent2vec.cpp on apps/word2vec/word2vec.h) ---
 * Sentence vectors against frozen word vectors: Sent2Vec::train
 * (sent2vec.cpp:37-181).  `words` is an SWPS_LAYOUT_W2V table holding the
 * word vectors (swps_load of a word2vec dump = ClusterServer::load,
 * server.h:49-62); it is never updated, only keys a minibatch pull misses
 * are inserted (accessmethod.h:63-70).  Corpus lines are atoi-keyed words
 * (word2vec.h:206); the sentence id is BKDR of the line (sent2vec.cpp:75). */
typedef struct swps_s2v swps_s2v;

typedef struct {
  int32_t window;              /* word2vec.window */
  int32_t negative;            /* word2vec.negative */
  int32_t min_sentence_length; /* word2vec.min_sentence_length */
  int32_t minibatch;           /* worker.minibatch (lines) */
  int32_t niters;              /* -niters: learn_instance passes per sentence */
  float alpha;                 /* word2vec.learning_rate */
  uint64_t unigram_size;       /* table_size (reference: 1e8) */
  uint32_t rand_seed;          /* glibc srand seed (reference: 1) */
  uint64_t rand_offset;        /* rand() calls before the first minibatch pull
                                * (port binds, table construction, the load) */
  uint64_t rand_insert_extra;  /* extra rand() calls per key the server inserts:
                                * 2*D for sparsehash's dense_hash_map::operator[],
                                * which default-constructs a WParam; 0 otherwise */
  int32_t profile;             /* 1: time kernels with HIP events */
} swps_s2v_cfg;

int swps_s2v_create(swps_table *words, const swps_s2v_cfg *cfg, swps_s2v **out);
int swps_s2v_destroy(swps_s2v *s);
/* corpus text (one sentence per line) or pre-split tokens: tok_keys[ntok],
 * line_off[nlines+1], sent_ids[nlines]; fixes the minibatch schedule */
int swps_s2v_load_text(swps_s2v *s, const char *path);
/* Doc-sharded multi-GPU sent2vec (BASELINE config 5): call
 * before loading; the loaders then keep only the lines whose sentence id
 * BasicHashFrag maps to node rank+1 (no exchange: documents are independent,
 * the word table is read-only and replicated on every GPU). */
int swps_s2v_shard(swps_s2v *s, int32_t rank, int32_t world, int32_t frag_num);
int swps_s2v_load_tokens(swps_s2v *s, const uint64_t *tok_keys, uint64_t ntok, const uint64_t *line_off,
                         uint64_t nlines, const uint64_t *sent_ids);
/* Sent2Vec::train (sent2vec.cpp:95-103) as the reference runs it: ONE pass that loads and trains —
 * each minibatch's vocabulary, unigram run starts, pull and rand() bookkeeping are built on host
 * threads while the GPU trains the minibatches before it (groups of 2, 4, then 8).  Returns after
 * the pass (synced); the same results as swps_s2v_load_tokens + swps_s2v_train, bit for bit.  The
 * arrays are read during the call only; no table call may run concurrently. */
int swps_s2v_run_tokens(swps_s2v *s, const uint64_t *tok_keys, uint64_t ntok, const uint64_t *line_off,
                        uint64_t nlines, const uint64_t *sent_ids);
/* nlines, sentences, minibatches, tokens, inserted keys, max sentences per
 * minibatch, max records per minibatch, rand() calls, LCG state at the end */
int swps_s2v_info(swps_s2v *s, uint64_t *out9);
/* the next `count` minibatches (wrapping to the corpus start) / one full pass */
int swps_s2v_train_batches(swps_s2v *s, uint64_t count);
int swps_s2v_train(swps_s2v *s);
int swps_s2v_sync(swps_s2v *s);
/* every sentence: ids[n], vectors [n][D] fp64, learn_instance's last g*g */
int swps_s2v_docs(swps_s2v *s, uint64_t *ids, double *vecs, float *errs, uint64_t cap, uint64_t *n);
/* the reference's output file: "sent_id\tVec:\tv0 v1 ... \n" (sent2vec.cpp:84) */
int swps_s2v_dump(swps_s2v *s, const char *path);
/* [minibatches, sentences, positions, context rows read, target rows read] */
int swps_s2v_stats(swps_s2v *s, uint64_t *out5);
int swps_s2v_set_profile(swps_s2v *s, int32_t on);
/* out[2k] = ms, out[2k+1] = launches for k in {records, docs} */
int swps_s2v_kernel_times(swps_s2v *s, double *out4, int32_t reset);
void *swps_s2v_stream(swps_s2v *s);

/* ---- sparse logistic regression (apps/logistic/lr.cpp) ------------------- */
typedef struct swps_lr swps_lr;

typedef struct {
  int32_t minibatch;  /* worker.minibatch: a batch is B+1 valid lines (lr.cpp:308-354) */
  int32_t init_ref;   /* 1: first-pull init from the float LCG in _local_keys order (lr.cpp:48-50) */
  int32_t profile;
  int32_t fast_sums;  /* 0: each key's gradient sum is the reference's sequential fp32 chain in record
                       * order (bit-exact); 1: fp64 sums, long runs tree-reduced across a wave (fast
                       * mode: deterministic, not bit-exact — within 1e-5 of the oracle) */
  int32_t plan;       /* SWPS_LR_PLAN_STEP (0): each minibatch's key-sorted index is built inside its
                       * training step, on a second stream beside the previous step (lr.cpp:215-227
                       * gathers each minibatch inside the loop) — single GPU, fast sums; otherwise,
                       * and with SWPS_LR_PLAN_LOAD (1), every minibatch's index is built once at load
                       * and reused every epoch.  Same results either way. */
} swps_lr_cfg;
#define SWPS_LR_PLAN_STEP 0
#define SWPS_LR_PLAN_LOAD 1
/* no index at all (single GPU, fast sums): each record's term e*x_i is added to its key's sum as
 * a 64-bit fixed-point integer (scale 2^s fixed at load so no sum reaches 2^62) by atomics — exact
 * integer sums, so deterministic in any order; each key's mean within ~2^-s of the fp64 sum's */
#define SWPS_LR_PLAN_NONE 2

int swps_lr_create(swps_table *t, const swps_lr_cfg *cfg, swps_lr **out);
int swps_lr_destroy(swps_lr *l);
/* libsvm/libfm text (lr.cpp:103-131) or CSR arrays (row_off has nrows+1) */
int swps_lr_load_text(swps_lr *l, const char *path);
int swps_lr_load_csr(swps_lr *l, const float *labels, uint64_t nrows, const uint64_t *row_off, const uint32_t *feat,
                     const float *vals);
int swps_lr_init(swps_lr *l);
/* one epoch per iter; err_out[niters] = mean squared error (lr.cpp:231) */
int swps_lr_train(swps_lr *l, int32_t niters, double *err_out);
int swps_lr_train_batches(swps_lr *l, uint64_t count);
int swps_lr_predict(swps_lr *l, float *pred_out, float *target_out, uint64_t cap);
int swps_lr_params(swps_lr *l, uint32_t *keys, float *w, float *g2, uint64_t cap, uint64_t *n);
int swps_lr_info(swps_lr *l, uint64_t *out4); /* nrows, nkeys, nbatches, nnz */
/* the plan the step runs (after load): out5 = {plan running, plan asked for, fixed-point scale bits s,
 * the floor s must reach, 1 when the fixed point (SWPS_LR_PLAN_NONE) was asked for and its scale
 * fell below the floor — heavy-tailed x_i: the load then switched to SWPS_LR_PLAN_STEP (fp64 sums)}.
 * Loads refuse non-finite labels or feature values with SWPS_E_CFG (lr.cpp:103-131 would train on
 * them). */
int swps_lr_plan_info(swps_lr *l, int32_t *out5);
int swps_lr_sync(swps_lr *l);
int swps_lr_set_profile(swps_lr *l, int32_t on); /* per-kernel HIP-event timing on/off (swps_lr_cfg.profile at create) */
int swps_lr_kernel_times(swps_lr *l, double *out8, int32_t reset);
/* mean of (y-p)^2 over all rows as of each row's last training (lr.cpp:231) */
int swps_lr_epoch_error(swps_lr *l, double *err);
void *swps_lr_stream(swps_lr *l);

/* ---- sharded LR (several GPUs; the caller moves the payloads) ------------
 * Same protocol as sharded word2vec, 1 fp32 value per key (lr.cpp:32-81):
 *   swps_lr_request -> all-to-all -> swps_lr_serve_pull (owner: weights [n])
 *   -> all-to-all -> swps_lr_step (install, forward, mean gradients [U] fp32
 *   in request order) -> all-to-all -> swps_lr_serve_push (owner: AdaGrad
 *   per source rank, in rank order).
 * First full pull (lr.cpp:161-166): swps_lr_request(init=1) ->
 * serve_pull(insert=1) -> swps_lr_install, which also refreshes the worker
 * cache swps_lr_predict reads.  Tables use SWPS_INIT_HASH and init_ref = 0. */
int swps_lr_shard(swps_lr *l, int32_t rank, int32_t world, int32_t frag_num);
int swps_lr_batch_counts(swps_lr *l, uint64_t *out, uint64_t cap, uint64_t *nb);
int swps_lr_request(swps_lr *l, int32_t init, uint64_t *counts, uint64_t *d_keys, uint64_t *n);
int swps_lr_serve_pull(swps_lr *l, const uint64_t *d_keys, const uint64_t *src_counts, int32_t insert,
                       float *d_vals);
int swps_lr_install(swps_lr *l, const float *d_vals);
int swps_lr_step(swps_lr *l, const float *d_vals, float *d_grads);
int swps_lr_serve_push(swps_lr *l, const uint64_t *d_keys, const float *d_grads, const uint64_t *src_counts);
/* library-driven sharded LR over `comm` (as swps_w2v_shard_comm): swps_lr_init,
 * swps_lr_train / train_batches and swps_lr_predict (a full pull first)
 * become collective; swps_lr_train's errors are this rank's rows'. */
int swps_lr_shard_comm(swps_lr *l, swps_comm *comm, int32_t frag_num);
/* as swps_w2v_exchange_stats, for the library-driven sharded LR */
int swps_lr_exchange_stats(swps_lr *l, int32_t on, double *out4);
/* the fixed-point step (SWPS_LR_PLAN_NONE) on one batch, for roofline accounting: out8 = {step
 * kernel bytes, push kernel bytes, form (1 bucketed, 2 atomic, 0 not running), hot keys, buckets,
 * step blocks, non-hot records, distinct non-hot keys}; zeros before the first step */
int swps_lr_fx_bytes(swps_lr *l, uint64_t batch, uint64_t *out8);

#ifdef __cplusplus
}
#endif
#endif /* SWPS_H_ */
