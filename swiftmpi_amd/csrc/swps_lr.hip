// Sparse logistic regression on one MI355X: the reference's minibatch loop
// (apps/logistic/lr.cpp:157-238, nthreads = 1 semantics) as HIP kernels.
//
// Per minibatch (B+1 valid rows, lr.cpp:308-354 gather == train window):
//   k_lr_forward   one thread per row: s = sum w_i*x_i (fp32, feature order),
//                  p = 1/(1+exp(-s)), e = y - p; one gradient record e*x_i per
//                  nonzero, keyed by the feature's vid   (lr.cpp:358-375)
//   radix sort     records by vid (stable: row order, then feature order)
//   run-length     unique vids + counts of the batch = the pushed key set
//   k_lr_push      per key: fp32 sum in record order, mean = sum/count
//                  (lr.cpp:32-38), AdaGrad fp32 (lr.cpp:68-75) on the shard row
// Every weight read in a batch belongs to that batch's key set, which the
// reference pulls at the start of the batch and the server only changes at the
// push: reading the shard rows directly is the same snapshot, so no copy.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <limits>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "swps_internal.h"

using namespace swps;

namespace {

__global__ void k_lr_forward(const uint64_t *__restrict__ row_off, const int32_t *__restrict__ fvid,
                             const float *__restrict__ fval, const float *__restrict__ label, uint64_t r0, uint64_t nr,
                             const uint32_t *__restrict__ vid_row, const float *__restrict__ rows,
                             float *__restrict__ contrib, uint32_t *__restrict__ keys, uint32_t *__restrict__ idx,
                             float *__restrict__ err2, uint64_t nz0) {
  uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nr) return;
  const uint64_t r = r0 + j;
  const uint64_t a = row_off[r], b = row_off[r + 1];
  float sum = 0;
  for (uint64_t i = a; i < b; i++) {
    const float w = rows[(uint64_t)vid_row[fvid[i]] * 2];
    const float prod = w * fval[i];
    sum += prod;
  }
  const float predict = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
  const float error = label[r] - predict;
  for (uint64_t i = a; i < b; i++) {
    contrib[i - nz0] = error * fval[i];
    keys[i - nz0] = (uint32_t)fvid[i];
    idx[i - nz0] = (uint32_t)(i - nz0);
  }
  err2[r] = error * error;
}

__global__ void k_lr_push(const uint32_t *__restrict__ uniq, const uint32_t *__restrict__ cnt,
                          const uint32_t *__restrict__ off, const uint32_t *__restrict__ nruns,
                          const uint32_t *__restrict__ sidx, const float *__restrict__ contrib,
                          const uint32_t *__restrict__ vid_row, float *__restrict__ rows, float lr, float fudge) {
  const uint32_t R = *nruns;
  for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < R; r += gridDim.x * blockDim.x) {
    const uint32_t o = off[r], c = cnt[r];
    float s = 0;
    for (uint32_t i = o; i < o + c; i++) s += contrib[sidx[i]];
    const float m = float(s / c);
    float *row = rows + (uint64_t)vid_row[uniq[r]] * 2;
    const float g2 = row[1] + m * m;
    row[1] = g2;
    const float step = lr * m;
    row[0] = row[0] + step / sqrtf(g2 + fudge);
  }
}

__global__ void k_lr_predict(const uint64_t *__restrict__ row_off, const int32_t *__restrict__ fvid,
                             const float *__restrict__ fval, uint64_t nr, const uint32_t *__restrict__ vid_row,
                             const float *__restrict__ rows, float *__restrict__ pred) {
  uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nr) return;
  float sum = 0;
  for (uint64_t i = row_off[r]; i < row_off[r + 1]; i++) {
    const float prod = rows[(uint64_t)vid_row[fvid[i]] * 2] * fval[i];
    sum += prod;
  }
  pred[r] = (float)(1. / (1. + (double)(float)exp((double)(-sum))));
}

inline unsigned nblk(uint64_t n, unsigned bs = 256) { return (unsigned)std::max<uint64_t>(1, (n + bs - 1) / bs); }

struct LTimer {
  bool on = false;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
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
  void resolve() {
    for (auto &q : pending) {
      float t = 0;
      (void)hipEventElapsedTime(&t, q.second.first, q.second.second);
      ms[q.first] += t;
      cnt[q.first]++;
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
  std::vector<uint64_t> vocab_keys;  // vid order = first-pull order
  bool loaded = false, inited = false;
  uint64_t cursor = 0, nbatches = 0;
  DevMem d_label, d_row_off, d_fvid, d_fval, d_vid_row, d_contrib, d_keys, d_idx, d_keys_s, d_idx_s, d_uniq, d_cnt,
      d_off, d_nruns, d_err2, d_tmp, d_pred;
  uint32_t *h_small = nullptr;
  LTimer timer;
  int B1() const { return cfg.minibatch + 1; }
};

namespace {

// lr.cpp:161-166: the first gather collects every feature of every valid row
// into `_local_keys` (std::unordered_set<unsigned>); the first pull visits it
// in iteration order, initialising each miss with global_random().gen_float().
int lr_ingest(swps_lr *l, std::vector<uint32_t> &&feat) {
  std::unordered_set<uint32_t> K0;
  for (auto f : feat) K0.insert(f);
  l->vocab_keys.assign(K0.begin(), K0.end());
  std::unordered_map<uint32_t, int32_t> vid;
  vid.reserve(K0.size() * 2);
  for (size_t i = 0; i < l->vocab_keys.size(); i++) vid[(uint32_t)l->vocab_keys[i]] = (int32_t)i;
  l->fvid.resize(feat.size());
  for (size_t i = 0; i < feat.size(); i++) l->fvid[i] = vid[feat[i]];
  const uint64_t nr = l->label.size();
  l->nbatches = nr ? (nr + l->B1() - 1) / l->B1() : 0;
  hipStream_t s = l->s;
  SWPS_TRY(upload(l->d_label, l->label, s));
  SWPS_TRY(upload(l->d_row_off, l->row_off, s));
  SWPS_TRY(upload(l->d_fvid, l->fvid, s));
  SWPS_TRY(upload(l->d_fval, l->fval, s));
  SWPS_TRY(l->d_vid_row.ensure(std::max<size_t>(1, l->vocab_keys.size()) * 4));
  SWPS_TRY(l->d_err2.ensure(std::max<uint64_t>(1, nr) * 4));
  SWPS_HIP(hipStreamSynchronize(s));
  l->loaded = true;
  return SWPS_OK;
}

int lr_batch(swps_lr *l) {
  const uint64_t nr = l->label.size();
  const uint64_t bi = l->cursor % l->nbatches;
  const uint64_t r0 = bi * l->B1(), r1 = std::min<uint64_t>(nr, r0 + l->B1());
  const uint64_t nz0 = l->row_off[r0], nnz = l->row_off[r1] - nz0;
  hipStream_t s = l->s;
  float *rows = l->t->rows.as<float>();
  l->cursor++;
  if (nnz == 0) return SWPS_OK;
  SWPS_TRY(l->d_contrib.ensure(nnz * 4));
  SWPS_TRY(l->d_keys.ensure(nnz * 4));
  SWPS_TRY(l->d_idx.ensure(nnz * 4));
  SWPS_TRY(l->d_keys_s.ensure(nnz * 4));
  SWPS_TRY(l->d_idx_s.ensure(nnz * 4));
  SWPS_TRY(l->d_uniq.ensure(nnz * 4));
  SWPS_TRY(l->d_cnt.ensure((nnz + 1) * 4));
  SWPS_TRY(l->d_off.ensure((nnz + 1) * 4));
  SWPS_TRY(l->d_nruns.ensure(16));
  hipEvent_t e0 = l->timer.begin(s);
  k_lr_forward<<<nblk(r1 - r0), 256, 0, s>>>(l->d_row_off.as<uint64_t>(), l->d_fvid.as<int32_t>(),
                                             l->d_fval.as<float>(), l->d_label.as<float>(), r0, r1 - r0,
                                             l->d_vid_row.as<uint32_t>(), rows, l->d_contrib.as<float>(),
                                             l->d_keys.as<uint32_t>(), l->d_idx.as<uint32_t>(), l->d_err2.as<float>(),
                                             nz0);
  SWPS_HIP(hipGetLastError());
  l->timer.end(0, e0, s);
  int bits = 1;
  while ((1ULL << bits) <= l->vocab_keys.size()) bits++;
  hipEvent_t e1 = l->timer.begin(s);
  size_t b1 = 0, b2 = 0, b3 = 0;
  SWPS_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, b1, l->d_keys.as<uint32_t>(), l->d_keys_s.as<uint32_t>(),
                                              l->d_idx.as<uint32_t>(), l->d_idx_s.as<uint32_t>(), (int)nnz, 0, bits,
                                              s));
  SWPS_HIP(hipcub::DeviceRunLengthEncode::Encode(nullptr, b2, l->d_keys_s.as<uint32_t>(), l->d_uniq.as<uint32_t>(),
                                                 l->d_cnt.as<uint32_t>(), l->d_nruns.as<uint32_t>(), (int)nnz, s));
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, b3, l->d_cnt.as<uint32_t>(), l->d_off.as<uint32_t>(),
                                            (int)nnz, s));
  SWPS_TRY(l->d_tmp.ensure(std::max(b1, std::max(b2, b3))));
  size_t tb = l->d_tmp.bytes;
  SWPS_HIP(hipcub::DeviceRadixSort::SortPairs(l->d_tmp.p, tb, l->d_keys.as<uint32_t>(), l->d_keys_s.as<uint32_t>(),
                                              l->d_idx.as<uint32_t>(), l->d_idx_s.as<uint32_t>(), (int)nnz, 0, bits,
                                              s));
  tb = l->d_tmp.bytes;
  SWPS_HIP(hipcub::DeviceRunLengthEncode::Encode(l->d_tmp.p, tb, l->d_keys_s.as<uint32_t>(), l->d_uniq.as<uint32_t>(),
                                                 l->d_cnt.as<uint32_t>(), l->d_nruns.as<uint32_t>(), (int)nnz, s));
  tb = l->d_tmp.bytes;
  SWPS_HIP(hipcub::DeviceScan::ExclusiveSum(l->d_tmp.p, tb, l->d_cnt.as<uint32_t>(), l->d_off.as<uint32_t>(),
                                            (int)nnz, s));
  l->timer.end(1, e1, s);
  hipEvent_t e3 = l->timer.begin(s);
  k_lr_push<<<(unsigned)std::min<uint64_t>(nblk(nnz), 4096), 256, 0, s>>>(
      l->d_uniq.as<uint32_t>(), l->d_cnt.as<uint32_t>(), l->d_off.as<uint32_t>(), l->d_nruns.as<uint32_t>(),
      l->d_idx_s.as<uint32_t>(), l->d_contrib.as<float>(), l->d_vid_row.as<uint32_t>(), rows,
      l->t->cfg.learning_rate, l->t->cfg.fudge);
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
  if (t->cfg.dtype != SWPS_F32) return fail(SWPS_E_UNSUPPORTED, "LR runs in the reference's fp32 (SWPS_F32)");
  if (cfg->minibatch <= 0) return fail(SWPS_E_CFG, "minibatch must be positive");
  SWPS_HIP(hipSetDevice(t->cfg.device));
  swps_lr *l = new swps_lr();
  l->t = t;
  l->cfg = *cfg;
  l->s = t->stream;
  l->timer.on = cfg->profile != 0;
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
  l->timer.resolve();
  if (l->h_small) (void)hipHostFree(l->h_small);
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
  return lr_ingest(l, std::move(feat));
}

int swps_lr_load_csr(swps_lr *l, const float *labels, uint64_t nrows, const uint64_t *row_off, const uint32_t *feat,
                     const float *vals) {
  if (row_off[0] != 0) return fail(SWPS_E_CFG, "row_off[0] must be 0");
  l->label.assign(labels, labels + nrows);
  l->row_off.assign(row_off, row_off + nrows + 1);
  const uint64_t nnz = row_off[nrows];
  l->fval.assign(vals, vals + nnz);
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  return lr_ingest(l, std::vector<uint32_t>(feat, feat + nnz));
}

int swps_lr_init(swps_lr *l) {
  if (!l->loaded) return fail(SWPS_E_STATE, "load data first");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  const uint64_t V = l->vocab_keys.size();
  DevMem dk;
  SWPS_TRY(upload(dk, l->vocab_keys, l->s));
  SWPS_TRY(table_find_or_insert(l->t, dk.as<uint64_t>(), V, l->d_vid_row.as<uint32_t>(), l->s));
  if (l->cfg.init_ref) {
    // LRPullAccessMethod::init_param (lr.cpp:48-50): w = gen_float() per miss
    std::vector<float> rows(V * 2, 0.f);
    uint64_t y = std::numeric_limits<unsigned long>::max() / 2;
    for (uint64_t i = 0; i < V; i++) {
      y = y * kFlcgA + kLcgC;
      rows[2 * i] = flcg_value(y);
    }
    DevMem dr;
    SWPS_TRY(upload(dr, rows, l->s));
    SWPS_TRY(table_set_rows(l->t, l->d_vid_row.as<uint32_t>(), V, dr.p, l->s));
    SWPS_HIP(hipStreamSynchronize(l->s));
  }
  l->inited = true;
  return SWPS_OK;
}

int swps_lr_train_batches(swps_lr *l, uint64_t count) {
  if (!l->inited) return fail(SWPS_E_STATE, "call swps_lr_init first");
  if (l->nbatches == 0) return SWPS_OK;
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  for (uint64_t i = 0; i < count; i++) SWPS_TRY(lr_batch(l));
  return SWPS_OK;
}

// lr.cpp:175-236: per epoch the mean of (y-p)^2 over the trained rows,
// accumulated in row order in double like `total_error`.
int swps_lr_train(swps_lr *l, int32_t niters, double *err_out) {
  if (l->cursor % std::max<uint64_t>(1, l->nbatches)) return fail(SWPS_E_STATE, "not at an epoch boundary");
  const uint64_t nr = l->label.size();
  std::vector<float> e2(nr);
  for (int it = 0; it < niters; it++) {
    SWPS_TRY(swps_lr_train_batches(l, l->nbatches));
    if (err_out) {
      SWPS_HIP(hipMemcpyAsync(e2.data(), l->d_err2.p, nr * 4, hipMemcpyDeviceToHost, l->s));
      SWPS_HIP(hipStreamSynchronize(l->s));
      double tot = 0;
      for (uint64_t r = 0; r < nr; r++) tot += e2[r];
      err_out[it] = nr ? tot / (double)nr : 0.0;
    }
  }
  return swps_lr_sync(l);
}

int swps_lr_sync(swps_lr *l) {
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  SWPS_HIP(hipStreamSynchronize(l->s));
  l->timer.resolve();
  return SWPS_OK;
}

// LR::predict_instance (lr.cpp:376-385) with the shard's current weights.
int swps_lr_predict(swps_lr *l, float *pred_out, float *target_out, uint64_t cap) {
  const uint64_t nr = l->label.size();
  if (cap < nr) return fail(SWPS_E_CFG, "buffer too small");
  SWPS_HIP(hipSetDevice(l->t->cfg.device));
  SWPS_TRY(l->d_pred.ensure(std::max<uint64_t>(1, nr) * 4));
  k_lr_predict<<<nblk(nr), 256, 0, l->s>>>(l->d_row_off.as<uint64_t>(), l->d_fvid.as<int32_t>(), l->d_fval.as<float>(),
                                            nr, l->d_vid_row.as<uint32_t>(), l->t->rows.as<float>(),
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

int swps_lr_info(swps_lr *l, uint64_t *o) {
  o[0] = l->label.size();
  o[1] = l->vocab_keys.size();
  o[2] = l->nbatches;
  o[3] = l->row_off.empty() ? 0 : l->row_off.back();
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

}  // extern "C"
