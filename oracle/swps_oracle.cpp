// =============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A plain-C++ (g++) CPU restatement of SwiftMPI's data-parallel hot path,
// written from the reference's behaviour (reference @ /root/reference/src,
// read as text; no reference source is compiled into this file).  It is the
// checker for the MI355X product in swiftmpi_amd/: only tests/,
// __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may load it.
// The product never links, loads or calls anything under oracle/.
//
// Parity pinning:
//   * LCG / float-LCG streams: pinned bit-exactly against the reference's own
//     utils/random.h compiled unmodified (oracle/ref_harness -> oracle/_ref),
//     fixture tests/golden/lcg_seed2008.json.
//   * LR end-to-end: pinned against the reference binary's recorded outputs on
//     its bundled data.txt (log-loss/accuracy after 20 and 100
//     epochs), fixture tests/golden/lr_reference_quality.json.
//   * BKDR, fmix64, hash-frag map, exp table, unigram table, CBOW-NS step and
//     AdaGrad: restated from the cited lines; known answers derived from the
//     code (no reference test asserts values — unittest/utils/common_test.h
//     only logs).  Those rows are "pinned by construction", not by execution.
//
// Precision modes: storage_f32 = 0 keeps every parameter in fp64 exactly like
// the reference (Vec::value_type = double, utils/vec1.h:8).  storage_f32 = 1
// rounds the stored server/cache values to fp32 after every write while all
// arithmetic stays fp64 — the exact semantics of the product's fp32 tables.
// =============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

extern "C" {

// ---- hashing ---------------------------------------------------------------
// utils/string.h:130-137  BKDRHash<size_t>(str, seed=13131); `char` is signed
// on x86-64, so bytes >= 0x80 contribute sign-extended negative values.
uint64_t orc_bkdr(const char *s) {
  uint64_t h = 0;
  while (*s) {
    h = h * 13131ULL + (uint64_t)(int64_t)(signed char)(*s++);
  }
  return h;
}

// utils/HashFunction.h:16-24  MurmurHash3 fmix64.
uint64_t orc_fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

// cluster/hashfrag.h:33-49  BasicHashFrag::init; node ids are 1..num_nodes.
// Returns -1 when frag_num < num_nodes (the reference divides by zero).
int orc_hashfrag_table(int frag_num, int num_nodes, uint32_t *out) {
  if (num_nodes <= 0 || frag_num <= 0) return -1;
  int each = int(frag_num / num_nodes);
  if (each == 0) return -1;
  for (int i = 0; i < frag_num; i++) {
    int id = int(uint32_t(i / each)) + 1;
    if (id < 1) id = 1;
    if (id > num_nodes) id = num_nodes;
    out[i] = (uint32_t)id;
  }
  return 0;
}

// cluster/hashfrag.h:51-56  to_node_id = map_table[fmix64(key) % frag_num].
int orc_to_node_id(uint64_t key, int frag_num, const uint32_t *table) {
  int frag = (int)(orc_fmix64(key) % (uint64_t)frag_num);
  return (int)table[frag];
}

// parameter/sparsetable.h:143  in-server shard id.
int orc_shard_id(uint64_t key, int shard_num) {
  return (int)(orc_fmix64(key) % (uint64_t)shard_num);
}

// ---- RNG: utils/random.h:25-47 --------------------------------------------
static inline uint64_t lcg_next(uint64_t &x) {
  x = x * 25214903917ULL + 11ULL;
  return x;
}
static inline float flcg_next(uint64_t &y) {
  y = y * 4903917ULL + 11ULL;
  return (float)y / (float)std::numeric_limits<unsigned long>::max();
}

void orc_lcg_sequence(uint64_t seed, uint64_t n, uint64_t *out) {
  uint64_t x = seed;
  for (uint64_t i = 0; i < n; i++) out[i] = lcg_next(x);
}

void orc_float_lcg_sequence(uint64_t n, uint64_t *states, float *out) {
  uint64_t y = std::numeric_limits<unsigned long>::max() / 2;
  for (uint64_t i = 0; i < n; i++) {
    out[i] = flcg_next(y);
    states[i] = y;
  }
}

// ---- ExpTable: apps/word2vec/word2vec_global.h:240-272 ----------------------
// t[i] = e/(e+1) with e = (float)exp((double)((i/1000.f*2-1)*6)).
void orc_exptable(float *out) {
  for (int i = 0; i < 1000; i++) {
    float x = (i / (float)1000 * 2 - 1) * 6;
    float e = (float)::exp((double)x);
    out[i] = e / (e + 1);
  }
}

// glibc rand() — the oracle calls libc itself (the function the reference's
// Vec::randInit uses, utils/vec1.h:229-232).
void orc_libc_rand_sequence(unsigned seed, uint64_t skip, uint64_t n, int32_t *out) {
  srand(seed);
  for (uint64_t i = 0; i < skip; i++) (void)rand();
  for (uint64_t i = 0; i < n; i++) out[i] = rand();
}

}  // extern "C"

// =============================================================================
// word2vec CBOW-NS, reference semantics of apps/word2vec/word2vec_global.h
// with nthreads = 1 (the deterministic configuration).
// =============================================================================
namespace {

thread_local std::string g_err;

struct Line {
  std::vector<uint64_t> words;
  bool valid = false;
};

// split(line, " ") — utils/string.h:34-48: only ' ' delimits.
static std::vector<std::string> split_space(const std::string &s) {
  std::vector<std::string> cols;
  size_t start = s.find_first_not_of(' ', 0);
  while (start != std::string::npos) {
    size_t last = s.find_first_of(' ', start);
    if (last == std::string::npos) {
      cols.push_back(s.substr(start));
    } else {
      cols.push_back(s.substr(start, last - start));
    }
    if (last == std::string::npos) break;
    start = s.find_first_not_of(' ', last);
  }
  return cols;
}

// LineFileReader::getline semantics (utils/string.h:91-120): split on '\n',
// strip the delimiter, a final fragment without '\n' is still a line.
static bool read_lines(const char *path, std::vector<std::string> &lines) {
  FILE *f = fopen(path, "rb");
  if (!f) return false;
  char *buf = nullptr;
  size_t cap = 0;
  ssize_t n;
  while ((n = getdelim(&buf, &cap, '\n', f)) >= 0) {
    if (n >= 1 && buf[n - 1] == '\n') buf[--n] = 0;
    lines.emplace_back(buf);  // NUL-terminated like std::string(cline)
  }
  free(buf);
  fclose(f);
  return true;
}

struct W2VCfg {
  int32_t dim, window, negative, min_sentence_length, minibatch, storage_f32;
  float sample, alpha, lr;
  uint64_t table_size;
  int32_t key_mode;        // 0 = BKDR (word2vec_global.h:205), 1 = atoi (word2vec.h:206)
  int32_t minibatch_vocab; // 1 = word2vec.h's MiniBatch (w2v_local.cpp): per-minibatch vocab + table
};

struct Row {
  std::vector<double> h, v;
};
struct SParam {
  std::vector<double> h, v, h2, v2;
};
struct Grad {
  std::vector<double> hg, vg;
  int hc = 0, vc = 0;
  std::vector<double> hp, vp;  // orc_diag_round bit 2: the current 128-record chunk's partial
};

// Diagnostic only (scripts/diag_fast.py): emulate one fp32 rounding of the
// GPU's fp32-intermediate kernels at a time, to attribute their distance from
// this oracle.  bit 0: g*neu1 formed from neu1 rounded to fp32; bit 1: neu1e
// rounded to fp32 before accu_v; bit 2: every 128-record chunk of a (key,
// kind) run summed alone and rounded to fp32 (k_gather_t partials; a run of
// <= 128 records is one chunk); bit 3: the mean rounded to fp32; bit 4: bits
// 0 and 1 keep a bf16 residual (x = fp32 hi + bf16 lo, the hi/lo storage).
// 0 = the reference's arithmetic.
static int orc_diag_round = 0;
static inline double diag_bf16(float x) {  // round to nearest even bf16
  uint32_t u;
  memcpy(&u, &x, 4);
  u = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xFFFF0000u;
  float y;
  memcpy(&y, &u, 4);
  return (double)y;
}
static inline double diag_r(double x, int bit) {
  if (!((orc_diag_round >> bit) & 1)) return x;
  const float hi = (float)x;
  if (bit <= 1 && (orc_diag_round & 16)) return (double)hi + diag_bf16((float)(x - (double)hi));
  if (bit <= 1 && (orc_diag_round & 32) && hi != 0.f) {  // int16 residual in units of ulp(hi) / 2^16
    int e;
    std::frexp(hi, &e);
    const double u = std::ldexp(1.0, e - 24 - 16);
    double q = std::nearbyint((x - (double)hi) / u);
    q = std::max(-32768.0, std::min(32767.0, q));
    return (double)hi + q * u;
  }
  return (double)hi;
}
// a whole neu1 / neu1e row: bit 6 = int16 residual in units of 2^-16 ulp of the row's largest
// element (one scale per row; bit 7: int8, 2^-8 ulp), else element-wise diag_r
static inline void diag_row(const std::vector<double> &x, std::vector<double> &out, int bit) {
  out = x;
  if (!((orc_diag_round >> bit) & 1)) return;
  if (orc_diag_round & (256 | 512 | 1024)) {  // bits 8 / 9 / 10: block floating point, int32 / int40 / int24
                                                // mantissas, one exponent
    double mx = 0;
    for (double v : x) mx = std::max(mx, std::fabs(v));
    if (mx == 0) return;
    int e;
    std::frexp(mx, &e);
    const int mb = (orc_diag_round & 256) ? 31 : (orc_diag_round & 1024) ? 23 : 39;
    const double u = std::ldexp(1.0, e - mb);
    for (size_t i = 0; i < x.size(); i++) out[i] = std::nearbyint(x[i] / u) * u;
    return;
  }
  if (!(orc_diag_round & 64)) {
    for (auto &v : out) v = diag_r(v, bit);
    return;
  }
  int emax = -1000;
  for (double v : x) {
    const float hi = (float)v;
    if (hi != 0.f) {
      int e;
      std::frexp(hi, &e);
      emax = std::max(emax, e);
    }
  }
  const int rb = (orc_diag_round & 128) ? 8 : 16;  // bit 7: an int8 residual instead of int16
  const double u = std::ldexp(1.0, std::max(emax - 24 - rb, -149));
  const double qm = rb == 8 ? 127.0 : 32767.0;
  for (size_t i = 0; i < x.size(); i++) {
    const float hi = (float)x[i];
    double q = std::nearbyint((x[i] - (double)hi) / u);
    q = std::max(-qm, std::min(qm, q));
    out[i] = (double)hi + q * u;
  }
}

static inline double store_round(double x, bool f32) { return f32 ? (double)(float)x : x; }

struct W2V {
  W2VCfg cfg;
  std::vector<Line> lines;
  std::map<uint64_t, int> word_freq;
  std::unordered_set<uint64_t> local_keys;  // global minibatch key set
  std::vector<uint64_t> wordids;
  size_t train_words = 0;
  std::vector<uint32_t> table;  // unigram table as indices into wordids
  std::unordered_map<uint64_t, SParam> server;
  std::unordered_map<uint64_t, SParam> *srv = &server;  // the multi-rank oracle shares one server
  std::unordered_map<uint64_t, Row> cache;
  std::unordered_map<uint64_t, Grad> grads;
  std::unordered_map<uint64_t, uint32_t> vid;
  uint64_t rng = 2008;                                              // random.h:44-47
  uint64_t frng = std::numeric_limits<unsigned long>::max() / 2;    // random.h:40-41
  float exptab[1000];
  // stats
  uint64_t kept = 0, pushes = 0, pulls = 0, actual_train_words = 0;
  double error_sum = 0;
  uint64_t error_cnt = 0;
  // optional trace of negative draws (vids) for the first `trace_cap` draws
  std::vector<int64_t> neg_trace;
  size_t trace_cap = 0;
  // word2vec.h MiniBatch state (minibatch_vocab): the minibatch's counts in
  // std::map order, its unigram table (keys), and `_num_words`, which
  // gather_keys increments for every gathered word and nothing resets
  // 
  std::map<uint64_t, int> bfreq;
  std::vector<uint64_t> btable;
  size_t num_words = 0;

  int D() const { return cfg.dim; }
  bool f32() const { return cfg.storage_f32 != 0; }

  uint64_t key_of(const std::string &w) const {
    if (cfg.key_mode == 1) return (uint64_t)(int64_t)std::atoi(w.c_str());
    return orc_bkdr(w.c_str());
  }

  // word2vec_global.h:215-227 parse_instance
  void parse(const std::string &s, Line &ln) const {
    ln.words.clear();
    for (auto &w : split_space(s)) ln.words.push_back(key_of(w));
    ln.valid = (int)ln.words.size() >= cfg.min_sentence_length;
  }

  // word2vec_global.h:385-444 gather_keys(file, nlines) with nthreads = 1
  void gather_all() {
    for (auto &ln : lines) {
      if (!ln.valid) continue;
      train_words += ln.words.size();
      for (auto k : ln.words) {
        auto it = word_freq.find(k);
        if (it != word_freq.end())
          it->second++;
        else {
          word_freq[k] = 1;
          local_keys.insert(k);
        }
      }
    }
  }

  // word2vec_global.h:467-497 gen_unigram_table (literal 1e8-entry loop)
  void gen_unigram_table() {
    for (auto k : local_keys) wordids.push_back(k);
    for (size_t i = 0; i < wordids.size(); i++) vid[wordids[i]] = (uint32_t)i;
    const uint64_t T = cfg.table_size;
    table.assign(T, 0);
    double pw = 0, power = 0.75;
    for (auto &it : word_freq) pw += std::pow(it.second, power);
    size_t i = 0;
    double d1 = std::pow(word_freq[wordids[i]], power) / (double)pw;
    for (uint64_t a = 0; a < T; a++) {
      table[a] = (uint32_t)i;
      if ((int64_t)a / (double)T > d1) {
        i++;
        if (i >= wordids.size()) throw std::runtime_error("unigram table walked past the vocab (reference UB)");
        d1 += std::pow(word_freq[wordids[i]], power) / (double)pw;
      }
      if (i >= word_freq.size()) i = word_freq.size() - 1;
    }
  }

  // WParam() random init, utils/vec1.h:229-232: (rand()/(float)RAND_MAX-0.5)/D
  void init_row_rand(std::vector<double> &x) {
    for (int i = 0; i < D(); i++) {
      float r = rand() / (float)RAND_MAX;
      x[i] = store_round(((double)r - 0.5) / (double)(size_t)D(), f32());
    }
  }

  // The first full pull (word2vec_global.h:557-562): every vocab key misses on
  // the server in `_local_keys` iteration order; each WParam() draws D rand()
  // for h then D for v.  rand_offset = rand() calls made before (port binds).
  void init_params_rand(unsigned seed, uint64_t rand_offset) {
    srand(seed);
    for (uint64_t i = 0; i < rand_offset; i++) (void)rand();
    for (auto k : local_keys) {
      SParam p;
      p.h.assign(D(), 0);
      p.v.assign(D(), 0);
      p.h2.assign(D(), 0);
      p.v2.assign(D(), 0);
      init_row_rand(p.h);
      init_row_rand(p.v);
      server[k] = p;
    }
    full_pull_to_cache();
  }

  void full_pull_to_cache() {
    for (auto k : local_keys) {
      auto &p = (*srv)[k];
      cache[k] = Row{p.h, p.v};
      Grad g;
      g.hg.assign(D(), 0);
      g.vg.assign(D(), 0);
      grads[k] = g;
    }
  }

  // float-LCG keep test, word2vec_global.h:725-731
  bool to_sample(uint64_t word) {
    if (cfg.sample < 0) return true;
    auto it = word_freq.find(word);
    if (it == word_freq.end()) throw std::runtime_error("word outside the vocab reached to_sample (reference UB)");
    float freq = float(it->second) / (float)train_words;
    float ran = (float)(1 - std::sqrt((double)(cfg.sample / freq)));
    return flcg_next(frng) > ran;
  }

  // word2vec.h:621-629 to_sample: freq over the minibatch's counts and the
  // never-reset `_num_words` (an int in the reference)
  bool to_sample_local(uint64_t word) {
    if (cfg.sample < 0) return true;
    auto it = bfreq.find(word);
    if (it == bfreq.end()) throw std::runtime_error("trained word outside the minibatch vocab (reference UB)");
    const int tw = (int)num_words;
    float freq = float(it->second) / tw;
    float ran = (float)(1 - std::sqrt((double)(cfg.sample / freq)));
    return flcg_next(frng) > ran;
  }

  // word2vec.h:398-425 gen_unigram_table over the minibatch vocab (_wordids
  // and the normaliser both in std::map key order), literal T-entry loop
  void gen_batch_table() {
    std::vector<uint64_t> ids;
    for (auto &kv : bfreq) ids.push_back(kv.first);
    const uint64_t T = cfg.table_size;
    btable.assign(T, 0);
    double pw = 0, power = 0.75;
    for (auto &kv : bfreq) pw += std::pow(kv.second, power);
    size_t i = 0;
    double d1 = std::pow(bfreq[ids[i]], power) / (double)pw;
    for (uint64_t a = 0; a < T; a++) {
      btable[a] = ids[i];
      if ((int64_t)a / (double)T > d1) {
        i++;
        if (i >= ids.size()) throw std::runtime_error("unigram table walked past the vocab (reference UB)");
        d1 += std::pow(bfreq[ids[i]], power) / (double)pw;
      }
      if (i >= bfreq.size()) i = bfreq.size() - 1;
    }
  }

  Row &cache_row(uint64_t k) {
    auto it = cache.find(k);
    if (it == cache.end()) {  // dense_hash_map::operator[] inserts zeros
      Row r;
      r.h.assign(D(), 0);
      r.v.assign(D(), 0);
      it = cache.emplace(k, r).first;
    }
    return it->second;
  }
  std::vector<double> &chunk_part(std::vector<double> &p) {
    if (p.empty()) p.assign(D(), 0);
    return p;
  }
  static void flush_part(std::vector<double> &p, std::vector<double> &tot) {
    for (size_t i = 0; i < p.size(); i++) {
      tot[i] += (double)(float)p[i];
      p[i] = 0;
    }
  }
  Grad &grad_row(uint64_t k) {
    auto it = grads.find(k);
    if (it == grads.end()) {
      Grad g;
      g.hg.assign(D(), 0);
      g.vg.assign(D(), 0);
      it = grads.emplace(k, g).first;
    }
    return it->second;
  }

  float exp_lookup(float f) const { return exptab[(int)((f + 6) * (1000 / 6 / 2))]; }

  // word2vec_global.h:654-719 learn_instance (CBOW, negative sampling)
  void learn_instance(const std::vector<uint64_t> &w) {
    const int W = cfg.window, N = cfg.negative, Dd = D();
    int b = (int)(lcg_next(rng) % (uint64_t)W);
    (void)b;
    int n = (int)w.size();
    std::vector<double> neu1(Dd), neu1e(Dd), tmp(Dd), n1r, n1er;
    const bool local = cfg.minibatch_vocab != 0;
    for (int pos = 0; pos < n; pos++) {
      uint64_t word = w[pos];
      if (!(local ? to_sample_local(word) : to_sample(word))) continue;
      kept++;
      std::fill(neu1.begin(), neu1.end(), 0.0);
      std::fill(neu1e.begin(), neu1e.end(), 0.0);
      b = (int)(lcg_next(rng) % (uint64_t)W);
      for (int a = b; a < W * 2 + 1 - b; a++) {
        if (a == W) continue;
        int c = pos - W + a;
        if (c < 0 || c >= n) continue;
        Row &r = cache_row(w[c]);
        for (int i = 0; i < Dd; i++) neu1[i] += r.v[i];
      }
      diag_row(neu1, n1r, 0);
      for (int d = 0; d < N + 1; d++) {
        uint64_t target;
        int label;
        if (d == 0) {
          target = word;
          label = 1;
        } else {
          uint64_t ti = (lcg_next(rng) >> 16) % cfg.table_size;
          target = local ? btable[ti] : wordids[table[ti]];
          if (target == 0) {
            ti = (lcg_next(rng) >> 16) % cfg.table_size;
            target = local ? btable[ti] : wordids[table[ti]];
          }
          if (neg_trace.size() < trace_cap) neg_trace.push_back(local ? (int64_t)vid[target] : (int64_t)table[ti]);
          if (target == word) continue;
          label = 0;
        }
        Row &t = cache_row(target);
        double dot = 0;
        for (int i = 0; i < Dd; i++) dot += neu1[i] * t.h[i];
        float f = 0;
        f += dot;
        float g;
        if (f > 6)
          g = (label - 1) * cfg.alpha;
        else if (f < -6)
          g = (label - 0) * cfg.alpha;
        else
          g = (label - exp_lookup(f)) * cfg.alpha;
        error_sum += 10000 * g * g;
        error_cnt++;
        for (int i = 0; i < Dd; i++) {
          tmp[i] = (double)g * t.h[i];
          neu1e[i] += tmp[i];
        }
        Grad &gr = grad_row(target);
        gr.hc++;
        std::vector<double> &hacc = (orc_diag_round & 4) ? chunk_part(gr.hp) : gr.hg;
        for (int i = 0; i < Dd; i++) {
          double p = (double)g * n1r[i];
          hacc[i] += p;
        }
        if ((orc_diag_round & 4) && gr.hc % 128 == 0) flush_part(gr.hp, gr.hg);
      }
      diag_row(neu1e, n1er, 1);
      for (int a = b; a < W * 2 + 1 - b; a++) {
        if (a == W) continue;
        int c = pos - W + a;
        if (c < 0 || c >= n) continue;
        Grad &gr = grad_row(w[c]);
        gr.vc++;
        std::vector<double> &vacc = (orc_diag_round & 4) ? chunk_part(gr.vp) : gr.vg;
        for (int i = 0; i < Dd; i++) vacc[i] += n1er[i];
        if ((orc_diag_round & 4) && gr.vc % 128 == 0) flush_part(gr.vp, gr.vg);
      }
    }
  }

  // gather_keys(file, line_id, B, 3) — next B+3 valid lines after `start`
  std::unordered_set<uint64_t> gather_window(size_t start) {
    std::unordered_set<uint64_t> K;
    int count = 0;
    size_t li = start;
    for (int task = 0; task < 3; task++) {
      while (li < lines.size()) {
        const Line &ln = lines[li++];
        if (!ln.valid) continue;
        for (auto k : ln.words) K.insert(k);
        count++;
        if (count > cfg.minibatch) break;
      }
    }
    return K;
  }

  // global_pull_access.h:80-101 callback + server.h:131-151 handler
  void pull(const std::unordered_set<uint64_t> &K) {
    pulls++;
    for (auto k : K) {
      auto it = srv->find(k);
      if (it == srv->end()) throw std::runtime_error("pull of a key the full pull never inserted");
      cache[k] = Row{it->second.h, it->second.v};
      Grad g;
      g.hg.assign(D(), 0);
      g.vg.assign(D(), 0);
      grads[k] = g;
    }
  }

  // global_push_access.h:48-67 + word2vec_global.h:122-134 (mean) +
  // word2vec_global.h:176-185 (AdaGrad, fp64)
  void push(const std::unordered_set<uint64_t> &K) {
    pushes++;
    const double lr = (double)cfg.lr;
    const double fudge = (double)1e-6f;
    const bool rf = f32();
    for (auto k : K) {
      auto git = grads.find(k);
      if (git == grads.end()) continue;
      Grad &g = git->second;
      if (orc_diag_round & 4) {
        if (g.hc % 128) flush_part(g.hp, g.hg);
        if (g.vc % 128) flush_part(g.vp, g.vg);
      }
      std::vector<double> hg = g.hg, vg = g.vg;
      if (g.hc > 0)
        for (auto &x : hg) x = diag_r(x / g.hc, 3);
      if (g.vc > 0)
        for (auto &x : vg) x = diag_r(x / g.vc, 3);
      std::fill(g.hg.begin(), g.hg.end(), 0.0);
      std::fill(g.vg.begin(), g.vg.end(), 0.0);
      g.hc = g.vc = 0;
      auto sit = srv->find(k);
      if (sit == srv->end()) throw std::runtime_error("push of an unknown key");
      SParam &p = sit->second;
      for (int i = 0; i < D(); i++) {
        double h2 = p.h2[i] + hg[i] * hg[i];
        double v2 = p.v2[i] + vg[i] * vg[i];
        double hn = p.h[i] + (hg[i] * lr) / std::sqrt(h2 + fudge);
        double vn = p.v[i] + (vg[i] * lr) / std::sqrt(v2 + fudge);
        p.h2[i] = store_round(h2, rf);
        p.v2[i] = store_round(v2, rf);
        p.h[i] = store_round(hn, rf);
        p.v[i] = store_round(vn, rf);
      }
    }
  }

  // word2vec.h:496-538 train_iter with nthreads = 1 (w2v_local.cpp): per
  // minibatch, gather_keys reads the next B+1 valid lines (counts, keys,
  // `_num_words`) and seeks back; fewer than 5 keys ends the epoch; pull;
  // the minibatch table; then B+1 lines (valid or not) are trained; push all
  // gathered keys; clear.
  void train_iter_local() {
    actual_train_words = 0;
    size_t p = 0;
    const int B = cfg.minibatch;
    while (true) {
      bfreq.clear();
      std::unordered_set<uint64_t> K;
      int count = 0;
      for (size_t q = p; q < lines.size();) {
        const Line &ln = lines[q++];
        if (!ln.valid) continue;
        for (auto k : ln.words) {
          num_words++;
          if (bfreq.find(k) == bfreq.end()) K.insert(k);
          bfreq[k]++;
        }
        if (++count > B) break;
      }
      if (K.size() < 5) break;
      pull(K);
      gen_batch_table();
      int lc = 0;
      while (p < lines.size()) {
        const Line &ln = lines[p++];
        learn_instance(ln.words);
        actual_train_words += ln.words.size();
        if (++lc > B) break;
      }
      push(K);
      for (auto k : K) {  // MiniBatch::clear (word2vec.h:386-391)
        cache.erase(k);
        grads.erase(k);
      }
    }
  }

  // The batches of one train_iter epoch as steps (the GPU schedule's
  // batches): step 0 = line 1, trained on the stale cache with no key set;
  // step j >= 1 = pull K_j, the lines up to the next minibatch boundary (or
  // the early stop), push K_j.
  struct Step {
    size_t l0, l1;
    bool hasK;
    std::unordered_set<uint64_t> K;
  };
  std::vector<Step> epoch_steps() {
    std::vector<Step> out;
    int line_counter = 0;
    size_t cur = 0, li = 0, start = 0;
    bool hasK = false;
    std::unordered_set<uint64_t> K;
    auto emit = [&](size_t end) {
      out.push_back(Step{start, end, hasK, hasK ? K : std::unordered_set<uint64_t>()});
      start = end;
    };
    while (li < lines.size()) {
      cur += lines[li++].words.size();
      line_counter++;
      if (line_counter == 1) {
        emit(li);
        K = gather_window(li);
        hasK = true;
      }
      if (line_counter % cfg.minibatch == 0) {
        emit(li);
        K = gather_window(li);
      }
      if (cur > train_words) break;
    }
    emit(li);
    return out;
  }
  // one step of a lockstep multi-rank run, in three phases
  void step_pull(const Step &st) {
    if (st.hasK) pull(st.K);
  }
  void step_learn(const Step &st) {
    for (size_t l = st.l0; l < st.l1; l++) {
      learn_instance(lines[l].words);
      actual_train_words += lines[l].words.size();
    }
  }
  void step_push(const Step &st) {
    if (st.hasK) push(st.K);
  }

  // word2vec_global.h:591-651 TrainModelThread(0) with nthreads = 1
  void train_iter() {
    actual_train_words = 0;
    int line_counter = 0;
    size_t cur_train_words = 0;
    std::unordered_set<uint64_t> K;
    size_t li = 0;
    while (li < lines.size()) {
      const Line &ln = lines[li++];
      learn_instance(ln.words);
      cur_train_words += ln.words.size();
      actual_train_words += ln.words.size();
      line_counter++;
      if (line_counter == 1) {
        K = gather_window(li);
        pull(K);
      }
      if (line_counter > 0 && line_counter % cfg.minibatch == 0) {
        push(K);
        K = gather_window(li);
        pull(K);
      }
      if (cur_train_words > train_words / 1) break;
    }
    push(K);
  }
};

}  // namespace

extern "C" {

typedef struct {
  int32_t dim, window, negative, min_sentence_length, minibatch, storage_f32;
  float sample, alpha, lr;
  uint64_t table_size;
  int32_t key_mode;
  int32_t minibatch_vocab;
} orc_w2v_cfg;

const char *orc_last_error(void) { return g_err.c_str(); }

void *orc_w2v_create(const char *corpus_path, const orc_w2v_cfg *c) {
  try {
    W2V *m = new W2V();
    m->cfg = W2VCfg{c->dim,    c->window, c->negative,   c->min_sentence_length, c->minibatch,
                    c->storage_f32, c->sample, c->alpha, c->lr, c->table_size, c->key_mode, c->minibatch_vocab};
    std::vector<std::string> raw;
    if (!read_lines(corpus_path, raw)) {
      g_err = "cannot open corpus";
      delete m;
      return nullptr;
    }
    m->lines.resize(raw.size());
    for (size_t i = 0; i < raw.size(); i++) m->parse(raw[i], m->lines[i]);
    m->gather_all();
    m->num_words = m->train_words;  // the first gather_keys(file, nlines) (word2vec.h:467-471)
    if (m->local_keys.size() < 5) {  // word2vec_global.h:556: train() returns
      g_err = "fewer than 5 keys";
      delete m;
      return nullptr;
    }
    m->gen_unigram_table();
    orc_exptable(m->exptab);
    return m;
  } catch (std::exception &e) {
    g_err = e.what();
    return nullptr;
  }
}

void orc_w2v_destroy(void *h) { delete (W2V *)h; }
void orc_set_diag_round(int bits) { orc_diag_round = bits; }

uint64_t orc_w2v_vocab_size(void *h) { return ((W2V *)h)->wordids.size(); }
uint64_t orc_w2v_train_words(void *h) { return ((W2V *)h)->train_words; }

// vocab in `_wordids` order (unordered_set iteration order) with counts
void orc_w2v_vocab(void *h, uint64_t *keys, int32_t *counts) {
  W2V *m = (W2V *)h;
  for (size_t i = 0; i < m->wordids.size(); i++) {
    keys[i] = m->wordids[i];
    counts[i] = m->word_freq[m->wordids[i]];
  }
}

// unigram table entries (as vids = index into the vocab order) at given slots
void orc_w2v_table_at(void *h, const uint64_t *idx, uint64_t n, uint32_t *out) {
  W2V *m = (W2V *)h;
  for (uint64_t i = 0; i < n; i++) out[i] = m->table[idx[i]];
}

// run-length form of the unigram table: start slot of every vid (V+1 entries)
int orc_w2v_table_starts(void *h, uint64_t *starts) {
  W2V *m = (W2V *)h;
  size_t V = m->wordids.size();
  size_t cur = 0;
  starts[0] = 0;
  for (uint64_t a = 1; a < m->table.size(); a++) {
    if (m->table[a] != m->table[a - 1]) {
      if (m->table[a] != m->table[a - 1] + 1) return -1;
      cur = m->table[a];
      starts[cur] = a;
    }
  }
  for (size_t i = cur + 1; i <= V; i++) starts[i] = m->table.size();
  return 0;
}

int orc_w2v_init_rand(void *h, unsigned seed, uint64_t rand_offset) {
  try {
    ((W2V *)h)->init_params_rand(seed, rand_offset);
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}

// set server params (and the full-pull cache) for vocab vids 0..V-1; each row
// is [h(D) | v(D)] in the given precision (double).
void orc_w2v_set_params(void *hh, const double *hv) {
  W2V *m = (W2V *)hh;
  int D = m->D();
  for (size_t i = 0; i < m->wordids.size(); i++) {
    SParam p;
    p.h.assign(hv + i * 2 * D, hv + i * 2 * D + D);
    p.v.assign(hv + i * 2 * D + D, hv + i * 2 * D + 2 * D);
    for (auto &x : p.h) x = store_round(x, m->f32());
    for (auto &x : p.v) x = store_round(x, m->f32());
    p.h2.assign(D, 0);
    p.v2.assign(D, 0);
    m->server[m->wordids[i]] = p;
  }
  m->full_pull_to_cache();
}

// get server params per vid: [h | v | h2 | v2] (4·D doubles per row)
void orc_w2v_get_params(void *hh, double *out) {
  W2V *m = (W2V *)hh;
  int D = m->D();
  for (size_t i = 0; i < m->wordids.size(); i++) {
    SParam &p = m->server[m->wordids[i]];
    double *o = out + i * 4 * D;
    std::copy(p.h.begin(), p.h.end(), o);
    std::copy(p.v.begin(), p.v.end(), o + D);
    std::copy(p.h2.begin(), p.h2.end(), o + 2 * D);
    std::copy(p.v2.begin(), p.v2.end(), o + 3 * D);
  }
}

void orc_w2v_trace_negatives(void *h, uint64_t cap) { ((W2V *)h)->trace_cap = cap; }
uint64_t orc_w2v_negatives(void *h, int64_t *out, uint64_t cap) {
  W2V *m = (W2V *)h;
  uint64_t n = std::min<uint64_t>(cap, m->neg_trace.size());
  std::copy(m->neg_trace.begin(), m->neg_trace.begin() + n, out);
  return n;
}

int orc_w2v_train(void *h, int niters) {
  try {
    W2V *m = (W2V *)h;
    for (int i = 0; i < niters; i++) {
      if (m->cfg.minibatch_vocab)
        m->train_iter_local();
      else
        m->train_iter();
    }
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}

// stats: [kept, pushes, pulls, actual_train_words, rng, frng]
void orc_w2v_stats(void *h, uint64_t *out) {
  W2V *m = (W2V *)h;
  out[0] = m->kept;
  out[1] = m->pushes;
  out[2] = m->pulls;
  out[3] = m->actual_train_words;
  out[4] = m->rng;
  out[5] = m->frng;
}

}  // extern "C"

// =============================================================================
// Sparse logistic regression — apps/logistic/lr.cpp with nthreads = 1.
// =============================================================================
namespace {

struct LRIns {
  float target;
  std::vector<std::pair<uint32_t, float>> feas;
};

// lr.cpp:103-131 parse_instance2 (blank / '#' lines are skipped; the
// reference's read past the NUL of an empty line is not reproduced).
static bool lr_parse(const std::string &line, LRIns &ins) {
  const char *p = line.c_str();
  ins.feas.clear();
  while (*p == ' ') p++;
  if (*p == 0 || *p == '#') return false;
  float value;
  int nchar, feature;
  if (std::sscanf(p, "%f%n", &value, &nchar) >= 1) {
    p += nchar;
    ins.target = value;
    while (std::sscanf(p, "%d:%f%n", &feature, &value, &nchar) >= 2) {
      p += nchar;
      ins.feas.emplace_back((uint32_t)feature, value);
    }
    return true;
  }
  throw std::runtime_error("cannot parse line");
}

struct LRParam {
  float val = 0, g2 = 0;
};
struct LRGrad {
  float val = 0;
  double val64 = 0;  // sum_f64: the same terms summed in fp64 (the rebuild's fast_sums definition)
  int count = 0;
};

struct LR {
  int minibatch = 200;
  float lr = 0.05f;
  // not the reference: each key's mean from an fp64 sum of its fp32 terms,
  // mean = float(sum / count) — what the rebuild's fast_sums computes (up to
  // summation order); the distance between the two oracle modes is the
  // reference's own fp32-chain rounding
  bool sum_f64 = false;
  std::vector<std::string> raw;
  std::vector<LRIns> ins;  // valid lines only
  std::unordered_set<uint32_t> all_keys;
  std::unordered_map<uint32_t, LRParam> server;
  std::unordered_map<uint32_t, float> cache;
  std::unordered_map<uint32_t, LRGrad> grads;
  uint64_t frng = std::numeric_limits<unsigned long>::max() / 2;
  std::vector<double> epoch_err;
  uint64_t batches = 0;

  // lr.cpp:45-56: init w = global_random().gen_float() on a miss
  void pull(const std::unordered_set<uint32_t> &K) {
    for (auto k : K) {
      auto it = server.find(k);
      if (it == server.end()) {
        LRParam p;
        p.val = flcg_next(frng);
        it = server.emplace(k, p).first;
      }
      cache[k] = it->second.val;
      grads[k] = LRGrad();
    }
  }
  // lr.cpp:32-38 (mean) + lr.cpp:68-75 (AdaGrad fp32)
  void push(const std::unordered_set<uint32_t> &K) {
    for (auto k : K) {
      auto it = grads.find(k);
      if (it == grads.end()) continue;
      LRGrad g = it->second;
      it->second = LRGrad();
      if (g.count == 0) throw std::runtime_error("zero-count push (reference stream desync, lr.cpp:34-35)");
      float m = sum_f64 ? float(g.val64 / (double)g.count) : float(g.val / g.count);
      LRParam &p = server[k];
      p.g2 += m * m;
      p.val += lr * m / float(std::sqrt(p.g2 + 1e-6f));
    }
  }
  // lr.cpp:358-375
  float learn(const LRIns &x) {
    float sum = 0;
    for (auto &f : x.feas) {
      float w = cache[f.first];
      float prod = w * f.second;
      sum += prod;
    }
    float predict = 1. / (1. + std::exp(-sum));
    float error = x.target - predict;
    for (auto &f : x.feas) {
      float grad = error * f.second;
      LRGrad &g = grads[f.first];
      g.val += grad;
      g.val64 += (double)grad;
      g.count++;
    }
    return error * error;
  }
  void train(int niters) {
    // lr.cpp:161-166 first full gather + pull
    std::unordered_set<uint32_t> K0;
    for (auto &x : ins)
      for (auto &f : x.feas) K0.insert(f.first);
    for (auto k : K0) {
      cache[k] = 0;
      grads[k] = LRGrad();
    }
    pull(K0);
    for (int it = 0; it < niters; it++) {
      double total = 0;
      int nrec = 0;
      size_t li = 0;
      while (true) {
        // gather_keys(file, B): next B+1 valid lines
        std::unordered_set<uint32_t> K;
        size_t end = std::min(ins.size(), li + (size_t)minibatch + 1);
        for (size_t j = li; j < end; j++)
          for (auto &f : ins[j].feas) K.insert(f.first);
        if (K.empty()) throw std::runtime_error("empty minibatch: the reference hangs here (global_pull_access.h:33-42)");
        cache.clear();
        grads.clear();
        for (auto k : K) {
          cache[k] = 0;
          grads[k] = LRGrad();
        }
        pull(K);
        for (size_t j = li; j < end; j++) {
          total += learn(ins[j]);
          nrec++;
        }
        push(K);
        batches++;
        li = end;
        if (li >= ins.size()) break;
      }
      epoch_err.push_back(total / nrec);
    }
  }
};

}  // namespace

extern "C" {

void orc_lr_set_sum_f64(void *h, int on) { ((LR *)h)->sum_f64 = on != 0; }

void *orc_lr_create(const char *path, int minibatch, float lr) {
  try {
    LR *m = new LR();
    m->minibatch = minibatch;
    m->lr = lr;
    if (!read_lines(path, m->raw)) {
      g_err = "cannot open dataset";
      delete m;
      return nullptr;
    }
    for (auto &s : m->raw) {
      LRIns x;
      if (lr_parse(s, x)) m->ins.push_back(x);
    }
    return m;
  } catch (std::exception &e) {
    g_err = e.what();
    return nullptr;
  }
}
// the same instances from CSR arrays (bench.py's CPU baseline: no text round trip of millions
// of synthetic rows; the training is lr.cpp's either way)
void *orc_lr_create_csr(const float *labels, uint64_t nrows, const uint64_t *row_off, const uint32_t *feat,
                        const float *vals, int minibatch, float lr) {
  try {
    LR *m = new LR();
    m->minibatch = minibatch;
    m->lr = lr;
    m->ins.resize(nrows);
    for (uint64_t r = 0; r < nrows; r++) {
      m->ins[r].target = labels[r];
      for (uint64_t j = row_off[r]; j < row_off[r + 1]; j++) m->ins[r].feas.emplace_back(feat[j], vals[j]);
    }
    return m;
  } catch (std::exception &e) {
    g_err = e.what();
    return nullptr;
  }
}
void orc_lr_destroy(void *h) { delete (LR *)h; }
uint64_t orc_lr_num_instances(void *h) { return ((LR *)h)->ins.size(); }

int orc_lr_train(void *h, int niters, double *epoch_err) {
  try {
    LR *m = (LR *)h;
    m->train(niters);
    for (int i = 0; i < niters; i++) epoch_err[i] = m->epoch_err[m->epoch_err.size() - niters + i];
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}

uint64_t orc_lr_num_keys(void *h) { return ((LR *)h)->server.size(); }
// keys (ascending) with their weight and AdaGrad accumulator
void orc_lr_params(void *h, uint32_t *keys, float *w, float *g2) {
  LR *m = (LR *)h;
  std::vector<uint32_t> ks;
  for (auto &kv : m->server) ks.push_back(kv.first);
  std::sort(ks.begin(), ks.end());
  for (size_t i = 0; i < ks.size(); i++) {
    keys[i] = ks[i];
    w[i] = m->server[ks[i]].val;
    g2[i] = m->server[ks[i]].g2;
  }
}

// lr.cpp:376-385 predict_instance with the current server weights; targets out
void orc_lr_predict(void *h, float *pred, float *target) {
  LR *m = (LR *)h;
  for (size_t i = 0; i < m->ins.size(); i++) {
    float sum = 0;
    for (auto &f : m->ins[i].feas) {
      auto it = m->server.find(f.first);
      float w = it == m->server.end() ? 0.f : it->second.val;
      float prod = w * f.second;
      sum += prod;
    }
    pred[i] = 1. / (1. + std::exp(-sum));
    target[i] = m->ins[i].target;
  }
}

// ClusterServer::load (server.h:49-62) of an LR dump (LRParam operator>>, lr.cpp:28-31): the
// dumped keys get their values, grad2sum 0, and nothing is drawn (init_param is not called)
void orc_lr_load(void *h, const uint32_t *keys, const float *vals, uint64_t n) {
  LR *m = (LR *)h;
  for (uint64_t i = 0; i < n; i++) {
    LRParam p;
    p.val = vals[i];
    m->server[keys[i]] = p;
  }
}

// lr.cpp:240-295 predict mode (after load_param, no training): per minibatch the keys of the next
// B+1 valid lines (gather_keys(file, minibatch), lr.cpp:308-351) are pulled — a key the server
// lacks gets init_param's gen_float() draw, in the key set's iteration order (lr.cpp:45-50) — and
// those lines are predicted from the pulled values (predict_instance, lr.cpp:376-385)
void orc_lr_predict_mode(void *h, float *pred) {
  LR *m = (LR *)h;
  size_t li = 0;
  while (li < m->ins.size()) {
    std::unordered_set<uint32_t> K;
    size_t end = std::min(m->ins.size(), li + (size_t)m->minibatch + 1);
    for (size_t j = li; j < end; j++)
      for (auto &f : m->ins[j].feas) K.insert(f.first);
    m->cache.clear();
    m->grads.clear();
    for (auto k : K) m->cache[k] = 0;
    m->pull(K);
    for (size_t j = li; j < end; j++) {
      float sum = 0;
      for (auto &f : m->ins[j].feas) {
        float w = m->cache[f.first];
        float prod = w * f.second;
        sum += prod;
      }
      pred[j] = 1. / (1. + std::exp(-sum));
    }
    li = end;
  }
}

// order in which the first full pull visits keys (unordered_set iteration)
uint64_t orc_lr_pull_order(void *h, uint32_t *out, uint64_t cap) {
  LR *m = (LR *)h;
  std::unordered_set<uint32_t> K0;
  for (auto &x : m->ins)
    for (auto &f : x.feas) K0.insert(f.first);
  uint64_t n = 0;
  for (auto k : K0)
    if (n < cap) out[n++] = k;
  return n;
}

}  // extern "C"

// =============================================================================
// Multi-rank lockstep restatement.  R workers — each a
// reference MPI rank with its own corpus, vocab, unigram table, RNG streams
// (global_random() is per process, random.h:44-47) and worker cache — and ONE
// server map standing for the union of the key-sharded servers.  A key is
// initialised on the first pull that reaches its owner by the hash rule of the
// product's sharded tables (SWPS_INIT_HASH: the reference's rand() order would
// depend on message arrival).  Step s of an epoch: every rank pulls its batch-s
// key set (so every pull sees every push of steps < s), every rank learns its
// batch-s lines, then every rank's mean-gradient push is applied as its own
// AdaGrad step in rank order — cluster/server.h:156-176 applies each worker's
// push request as it arrives; the lockstep order fixes the arrival order.
// Ranks with fewer batches per epoch idle in the later steps.
// =============================================================================
namespace {

static inline uint64_t orc_splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}
// u in [0, 1) from (seed, key, element) — the sharded tables' init hash
static inline float orc_unit_hash(uint64_t seed, uint64_t key, uint64_t i) {
  uint64_t z = orc_splitmix64(seed ^ orc_splitmix64(key + 0x632be59bd9b4e019ULL * (i + 1)));
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

struct W2VMulti {
  std::vector<W2V *> ranks;
  std::unordered_map<uint64_t, SParam> server;
  uint64_t seed = 0;
  ~W2VMulti() {
    for (auto *m : ranks) delete m;
  }
  void init_key(uint64_t k, int D, bool f32) {
    if (server.count(k)) return;
    SParam p;
    p.h.assign(D, 0);
    p.v.assign(D, 0);
    p.h2.assign(D, 0);
    p.v2.assign(D, 0);
    for (int e = 0; e < 2 * D; e++) {
      double x = store_round(((double)orc_unit_hash(seed, k, e) - 0.5) / (double)D, f32);
      (e < D ? p.h[e] : p.v[e - D]) = x;
    }
    server[k] = p;
  }
  void full_pulls() {  // every rank's first full pull (word2vec_global.h:557-562)
    for (auto *m : ranks) {
      for (auto k : m->local_keys) init_key(k, m->D(), m->f32());
      m->full_pull_to_cache();
    }
  }
  std::vector<std::vector<W2V::Step>> st;
  size_t maxs = 0, cursor = 0;  // steps per epoch (the longest rank's), global step
  void plan() {
    if (!st.empty()) return;
    for (auto *m : ranks) {
      st.push_back(m->epoch_steps());
      maxs = std::max(maxs, st.back().size());
    }
  }
  void train_steps(size_t n) {  // the next n lockstep steps, epochs wrapping
    plan();
    for (size_t k = 0; k < n; k++, cursor++) {
      const size_t s = cursor % maxs;
      if (s == 0)
        for (auto *m : ranks) m->actual_train_words = 0;
      for (size_t r = 0; r < ranks.size(); r++)
        if (s < st[r].size()) ranks[r]->step_pull(st[r][s]);
      for (size_t r = 0; r < ranks.size(); r++)
        if (s < st[r].size()) ranks[r]->step_learn(st[r][s]);
      for (size_t r = 0; r < ranks.size(); r++)
        if (s < st[r].size()) ranks[r]->step_push(st[r][s]);
    }
  }
  void train(int niters) {
    plan();
    train_steps((size_t)niters * maxs);
  }
};

// sparse LR, the same lockstep over R workers (lr.cpp:157-238 per rank, one
// server map, hash init w = u on the first pull, AdaGrad per source in rank order)
struct LRMulti {
  std::vector<LR *> ranks;
  std::unordered_map<uint32_t, LRParam> server;
  uint64_t seed = 0;
  ~LRMulti() {
    for (auto *m : ranks) delete m;
  }
  // a rank's batches of an epoch: B+1 valid lines each (lr.cpp:308-354)
  static std::vector<std::pair<size_t, size_t>> batches(const LR &m) {
    std::vector<std::pair<size_t, size_t>> out;
    for (size_t li = 0; li < m.ins.size();) {
      size_t end = std::min(m.ins.size(), li + (size_t)m.minibatch + 1);
      out.emplace_back(li, end);
      li = end;
    }
    return out;
  }
  void pull(LR &m, const std::unordered_set<uint32_t> &K) {
    for (auto k : K) {
      auto it = server.find(k);
      if (it == server.end()) {
        LRParam p;
        p.val = orc_unit_hash(seed, k, 0);
        it = server.emplace(k, p).first;
      }
      m.cache[k] = it->second.val;
      m.grads[k] = LRGrad();
    }
  }
  void push(LR &m, const std::unordered_set<uint32_t> &K) {
    for (auto k : K) {
      auto it = m.grads.find(k);
      if (it == m.grads.end()) continue;
      LRGrad g = it->second;
      it->second = LRGrad();
      if (g.count == 0) continue;
      float mg = float(g.val / g.count);
      LRParam &p = server[k];
      p.g2 += mg * mg;
      p.val += m.lr * mg / float(std::sqrt(p.g2 + 1e-6f));
    }
  }
  void train(int niters) {
    std::vector<std::vector<std::pair<size_t, size_t>>> bs;
    size_t maxs = 0;
    for (auto *m : ranks) {
      std::unordered_set<uint32_t> K0;
      for (auto &x : m->ins)
        for (auto &f : x.feas) K0.insert(f.first);
      pull(*m, K0);
      bs.push_back(batches(*m));
      maxs = std::max(maxs, bs.back().size());
    }
    std::vector<std::unordered_set<uint32_t>> K(ranks.size());
    for (int it = 0; it < niters; it++)
      for (size_t s = 0; s < maxs; s++) {
        for (size_t r = 0; r < ranks.size(); r++) {
          if (s >= bs[r].size()) continue;
          LR &m = *ranks[r];
          K[r].clear();
          for (size_t j = bs[r][s].first; j < bs[r][s].second; j++)
            for (auto &f : m.ins[j].feas) K[r].insert(f.first);
          m.cache.clear();
          m.grads.clear();
          pull(m, K[r]);
        }
        for (size_t r = 0; r < ranks.size(); r++)
          if (s < bs[r].size())
            for (size_t j = bs[r][s].first; j < bs[r][s].second; j++) ranks[r]->learn(ranks[r]->ins[j]);
        for (size_t r = 0; r < ranks.size(); r++)
          if (s < bs[r].size()) push(*ranks[r], K[r]);
      }
  }
};

}  // namespace

extern "C" {

void *orc_w2vm_create(const char **paths, int R, const orc_w2v_cfg *c, uint64_t seed) {
  W2VMulti *mm = new W2VMulti();
  mm->seed = seed;
  for (int r = 0; r < R; r++) {
    W2V *m = (W2V *)orc_w2v_create(paths[r], c);
    if (!m) {
      delete mm;
      return nullptr;
    }
    m->srv = &mm->server;
    mm->ranks.push_back(m);
  }
  try {
    mm->full_pulls();
  } catch (std::exception &e) {
    g_err = e.what();
    delete mm;
    return nullptr;
  }
  return mm;
}
void orc_w2vm_destroy(void *h) { delete (W2VMulti *)h; }
int orc_w2vm_train(void *h, int niters) {
  try {
    ((W2VMulti *)h)->train(niters);
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}
int orc_w2vm_train_steps(void *h, uint64_t n) {
  try {
    ((W2VMulti *)h)->train_steps(n);
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}
uint64_t orc_w2vm_num_keys(void *h) { return ((W2VMulti *)h)->server.size(); }
// every server key (ascending) with its row [h | v | h2 | v2]
void orc_w2vm_params(void *h, uint64_t *keys, double *rows) {
  W2VMulti *mm = (W2VMulti *)h;
  std::vector<uint64_t> ks;
  for (auto &kv : mm->server) ks.push_back(kv.first);
  std::sort(ks.begin(), ks.end());
  const int D = mm->ranks[0]->D();
  for (size_t i = 0; i < ks.size(); i++) {
    keys[i] = ks[i];
    const SParam &p = mm->server[ks[i]];
    double *o = rows + i * 4 * D;
    std::copy(p.h.begin(), p.h.end(), o);
    std::copy(p.v.begin(), p.v.end(), o + D);
    std::copy(p.h2.begin(), p.h2.end(), o + 2 * D);
    std::copy(p.v2.begin(), p.v2.end(), o + 3 * D);
  }
}
// per-rank [kept, pushes, pulls, actual_train_words, rng, frng]
void orc_w2vm_rank_stats(void *h, int r, uint64_t *out) { orc_w2v_stats(((W2VMulti *)h)->ranks[r], out); }

void *orc_lrm_create(const char **paths, int R, int minibatch, float lr, uint64_t seed) {
  LRMulti *mm = new LRMulti();
  mm->seed = seed;
  for (int r = 0; r < R; r++) {
    LR *m = (LR *)orc_lr_create(paths[r], minibatch, lr);
    if (!m) {
      delete mm;
      return nullptr;
    }
    mm->ranks.push_back(m);
  }
  return mm;
}
void orc_lrm_destroy(void *h) { delete (LRMulti *)h; }
int orc_lrm_train(void *h, int niters) {
  try {
    ((LRMulti *)h)->train(niters);
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}
uint64_t orc_lrm_num_keys(void *h) { return ((LRMulti *)h)->server.size(); }
void orc_lrm_params(void *h, uint32_t *keys, float *w, float *g2) {
  LRMulti *mm = (LRMulti *)h;
  std::vector<uint32_t> ks;
  for (auto &kv : mm->server) ks.push_back(kv.first);
  std::sort(ks.begin(), ks.end());
  for (size_t i = 0; i < ks.size(); i++) {
    keys[i] = ks[i];
    w[i] = mm->server[ks[i]].val;
    g2[i] = mm->server[ks[i]].g2;
  }
}

}  // extern "C"

// =============================================================================
// sent2vec — apps/sent2vec/sent2vec.cpp (Sent2Vec) on apps/word2vec/word2vec.h's
// MiniBatch, nthreads = 1.
//   * word vectors: ClusterServer::load (cluster/server.h:49-62) of a text
//     dump "key\tv...\th..." — one WParam (2·D rand()) is constructed before
//     the loop; never updated afterwards (WordMiniBatch has no push);
//   * per minibatch: gather the next B+1 valid lines (word2vec.h:323-377:
//     atoi keys, std::map counts, `_local_keys` a persistent unordered_set
//     that is cleared, not rebuilt), pull (server.h:129-154: a WParam — 2·D
//     rand() — per pulled key, misses inserted), a table_size-slot unigram
//     table in std::map key order (word2vec.h:398-425);
//   * then B+1 lines (valid or not) are read; each valid line gets
//     sent_id = BKDR(line), a fresh sentence vector (Vec::random: D rand(),
//     utils/vec1.h:229-232) and `niters` learn_instance passes
//     (sent2vec.cpp:109-181): neu1 = sent + sum of context v, positive +
//     negatives from the minibatch table, neu1e += g*h, sent += alpha*neu1e.
// `rand_insert_extra` = rand() calls consumed per new server key beyond the
// WParam that is stored (google::dense_hash_map::operator[] default-constructs
// the mapped WParam, 2·D, when the key is new: sparsetable.h:45-48); 0 models
// a map that does not.
// =============================================================================
namespace {

struct S2VCfg {
  int32_t dim, window, negative, min_sentence_length, minibatch, niters, storage_f32;
  float alpha;
  uint64_t table_size;
  uint32_t rand_seed;
  uint64_t rand_offset;
  uint64_t rand_insert_extra;
};

struct S2V {
  S2VCfg cfg;
  std::vector<std::string> raw;
  std::vector<Line> lines;
  std::unordered_map<uint64_t, Row> server;
  std::unordered_set<uint64_t> local_keys;  // MiniBatch::_local_keys (one object for the run)
  std::map<uint64_t, int> word_freq;
  std::vector<uint64_t> wordids;
  std::vector<uint64_t> table;  // keys
  std::unordered_map<uint64_t, Row> cache;
  uint64_t rng = 2008;
  float exptab[1000];
  uint64_t rand_calls = 0, batches = 0, pulled = 0, misses = 0, draws = 0;
  float err_data = 0;
  std::vector<uint64_t> ids;
  std::vector<double> vecs;
  std::vector<float> errs;

  int D() const { return cfg.dim; }
  bool f32() const { return cfg.storage_f32 != 0; }

  int32_t R() {
    rand_calls++;
    return rand();
  }
  // Vec::randInit (utils/vec1.h:229-232)
  void rand_vec(std::vector<double> &x) {
    x.assign(D(), 0.0);
    for (int i = 0; i < D(); i++) {
      float r = R() / (float)RAND_MAX;
      x[i] = ((double)r - 0.5) / (double)(size_t)D();
    }
  }
  // SparseTableShard::assign (sparsetable.h:45-48) of a key new to the server
  void insert(uint64_t k, const Row &p) {
    for (uint64_t i = 0; i < cfg.rand_insert_extra; i++) (void)R();
    Row r = p;
    for (auto &x : r.h) x = store_round(x, f32());
    for (auto &x : r.v) x = store_round(x, f32());
    server[k] = r;
  }

  // ClusterServer::load (server.h:49-62), one server: every key is owned.
  void load(const char *path) {
    std::ifstream file(path);
    if (!file.is_open()) throw std::runtime_error("cannot open word vectors");
    Row param;  // `param_t param;` — WParam(): h then v
    rand_vec(param.h);
    rand_vec(param.v);
    unsigned long key = 0;
    bool have = false;
    while (!file.eof()) {
      file >> key;  // on failure at EOF `key` keeps the last value
      have = have || !file.fail();
      for (int i = 0; i < D(); i++) file >> param.v[i];  // WParam operator>>: v then h
      for (int i = 0; i < D(); i++) file >> param.h[i];
      if (!have) break;  // empty file: the reference would assign an uninitialised key
      if (server.find(key) == server.end()) {
        insert(key, param);
      } else {
        Row r = param;
        for (auto &x : r.h) x = store_round(x, f32());
        for (auto &x : r.v) x = store_round(x, f32());
        server[key] = r;
      }
    }
  }

  // word2vec.h:398-425 (std::map order, literal table_size walk)
  void gen_unigram_table() {
    wordids.clear();
    for (auto &it : word_freq) wordids.push_back(it.first);
    const uint64_t T = cfg.table_size;
    table.assign(T, 0);
    double pw = 0, power = 0.75;
    for (auto &it : word_freq) pw += std::pow(it.second, power);
    size_t i = 0;
    double d1 = std::pow(word_freq[wordids[i]], power) / (double)pw;
    for (uint64_t a = 0; a < T; a++) {
      table[a] = wordids[i];
      if ((int64_t)a / (double)T > d1) {
        i++;
        if (i >= wordids.size()) throw std::runtime_error("unigram table walked past the vocab (reference UB)");
        d1 += std::pow(word_freq[wordids[i]], power) / (double)pw;
      }
      if (i >= word_freq.size()) i = word_freq.size() - 1;
    }
  }

  float exp_lookup(float f) const { return exptab[(int)((f + 6) * (1000 / 6 / 2))]; }

  // sent2vec.cpp:109-181
  float learn_instance(const std::vector<uint64_t> &w, std::vector<double> &sent) {
    const int W = cfg.window, N = cfg.negative, Dd = D();
    int b = (int)(lcg_next(rng) % (uint64_t)W);
    draws++;
    const int n = (int)w.size();
    float g = 0, f;
    std::vector<double> neu1(Dd), neu1e(Dd);
    for (int pos = 0; pos < n; pos++) {
      const uint64_t word = w[pos];
      std::fill(neu1e.begin(), neu1e.end(), 0.0);
      b = (int)(lcg_next(rng) % (uint64_t)W);
      draws++;
      neu1 = sent;
      for (int a = b; a < W * 2 + 1 - b; a++) {
        if (a == W) continue;
        int c = pos - W + a;
        if (c < 0 || c >= n) continue;
        const Row &r = cache.at(w[c]);
        for (int i = 0; i < Dd; i++) neu1[i] += r.v[i];
      }
      for (int d = 0; d < N + 1; d++) {
        uint64_t target;
        int label;
        if (d == 0) {
          target = word;
          label = 1;
        } else {
          target = table[(lcg_next(rng) >> 16) % cfg.table_size];
          draws++;
          if (target == 0) {
            target = table[(lcg_next(rng) >> 16) % cfg.table_size];
            draws++;
          }
          if (target == word) continue;
          label = 0;
        }
        const Row &t = cache.at(target);
        double dot = 0;
        for (int i = 0; i < Dd; i++) dot += neu1[i] * t.h[i];
        f = 0;
        f += dot;
        if (f > 6)
          g = (label - 1) * cfg.alpha;
        else if (f < -6)
          g = (label - 0) * cfg.alpha;
        else
          g = (label - exp_lookup(f)) * cfg.alpha;
        for (int i = 0; i < Dd; i++) {
          double p = t.h[i] * (double)g;
          neu1e[i] += p;
        }
      }
      for (int i = 0; i < Dd; i++) {
        double p = neu1e[i] * (double)cfg.alpha;
        sent[i] += p;
      }
    }
    return g * g;
  }

  // Sent2Vec::train (sent2vec.cpp:37-106)
  void train() {
    const int B = cfg.minibatch;
    const size_t nl = lines.size();
    size_t li = 0;
    while (true) {
      // MiniBatch::gather_keys(file, line_id, B) (word2vec.h:323-377) after clear()
      local_keys.clear();
      word_freq.clear();
      cache.clear();
      int cnt = 0;
      for (size_t j = li; j < nl;) {
        const Line &ln = lines[j++];
        if (!ln.valid) continue;
        for (auto k : ln.words) {
          auto it = word_freq.find(k);
          if (it != word_freq.end())
            it->second++;
          else {
            word_freq[k] = 1;
            local_keys.insert(k);
          }
        }
        if (++cnt > B) break;
      }
      if (local_keys.size() < 5) break;
      // MiniBatch::pull (word2vec.h:303-310) -> server.h:143-150 per key
      for (auto k : local_keys) {
        Row p;
        rand_vec(p.h);
        rand_vec(p.v);
        auto it = server.find(k);
        if (it == server.end()) {
          insert(k, p);
          it = server.find(k);
          misses++;
        }
        cache[k] = it->second;
        pulled++;
      }
      gen_unigram_table();
      // the training handler (sent2vec.cpp:48-93)
      int lc = 0;
      while (true) {
        if (lc > B) break;
        if (li >= nl) break;
        const size_t l = li++;
        lc++;
        if (!lines[l].valid) continue;
        const uint64_t sent_id = orc_bkdr(raw[l].c_str());
        std::vector<double> sent;
        rand_vec(sent);
        float error = 0;
        for (int it = 0; it < cfg.niters; it++) error = learn_instance(lines[l].words, sent);
        err_data += error;
        ids.push_back(sent_id);
        vecs.insert(vecs.end(), sent.begin(), sent.end());
        errs.push_back(error);
        if (lc > B) break;
      }
      batches++;
    }
  }
};

}  // namespace

extern "C" {

typedef struct {
  int32_t dim, window, negative, min_sentence_length, minibatch, niters, storage_f32;
  float alpha;
  uint64_t table_size;
  uint32_t rand_seed;
  uint64_t rand_offset;
  uint64_t rand_insert_extra;
} orc_s2v_cfg;

void *orc_s2v_create(const char *corpus_path, const orc_s2v_cfg *c) {
  try {
    S2V *m = new S2V();
    m->cfg = S2VCfg{c->dim,        c->window,     c->negative,  c->min_sentence_length,
                    c->minibatch,  c->niters,     c->storage_f32, c->alpha,
                    c->table_size, c->rand_seed,  c->rand_offset, c->rand_insert_extra};
    if (!read_lines(corpus_path, m->raw)) {
      g_err = "cannot open corpus";
      delete m;
      return nullptr;
    }
    m->lines.resize(m->raw.size());
    for (size_t i = 0; i < m->raw.size(); i++) {  // word2vec.h:212-224 (atoi keys)
      Line &ln = m->lines[i];
      for (auto &w : split_space(m->raw[i])) ln.words.push_back((uint64_t)(int64_t)std::atoi(w.c_str()));
      ln.valid = (int)ln.words.size() >= c->min_sentence_length;
    }
    orc_exptable(m->exptab);
    srand(c->rand_seed);
    for (uint64_t i = 0; i < c->rand_offset; i++) (void)m->R();
    return m;
  } catch (std::exception &e) {
    g_err = e.what();
    return nullptr;
  }
}

void orc_s2v_destroy(void *h) { delete (S2V *)h; }

int orc_s2v_load_words(void *h, const char *path) {
  try {
    ((S2V *)h)->load(path);
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}

int orc_s2v_train(void *h) {
  try {
    ((S2V *)h)->train();
    return 0;
  } catch (std::exception &e) {
    g_err = e.what();
    return -1;
  }
}

uint64_t orc_s2v_num_docs(void *h) { return ((S2V *)h)->ids.size(); }

// sentence ids, vectors [n][D] and per-sentence learn_instance return values
void orc_s2v_docs(void *h, uint64_t *ids, double *vecs, float *errs) {
  S2V *m = (S2V *)h;
  std::copy(m->ids.begin(), m->ids.end(), ids);
  std::copy(m->vecs.begin(), m->vecs.end(), vecs);
  std::copy(m->errs.begin(), m->errs.end(), errs);
}

// [minibatches, pulled keys, inserted keys, rand() calls, LCG draws, LCG state,
//  server keys, Error::data as float bits]
void orc_s2v_stats(void *h, uint64_t *out) {
  S2V *m = (S2V *)h;
  out[0] = m->batches;
  out[1] = m->pulled;
  out[2] = m->misses;
  out[3] = m->rand_calls;
  out[4] = m->draws;
  out[5] = m->rng;
  out[6] = m->server.size();
  uint32_t bits;
  std::memcpy(&bits, &m->err_data, 4);
  out[7] = bits;
}

// server rows [h | v] of the given keys (0 and return -1 for unknown keys)
int orc_s2v_word_rows(void *h, const uint64_t *keys, uint64_t n, double *out) {
  S2V *m = (S2V *)h;
  int rc = 0;
  const int D = m->D();
  for (uint64_t i = 0; i < n; i++) {
    auto it = m->server.find(keys[i]);
    double *o = out + i * 2 * D;
    if (it == m->server.end()) {
      std::fill(o, o + 2 * D, 0.0);
      rc = -1;
      continue;
    }
    std::copy(it->second.h.begin(), it->second.h.end(), o);
    std::copy(it->second.v.begin(), it->second.v.end(), o + D);
  }
  return rc;
}

}  // extern "C"
