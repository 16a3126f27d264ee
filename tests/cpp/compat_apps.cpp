// C++11 drivers over include/swiftmpi_compat.h — what the reference's app
// mains (apps/word2vec/w2v.cpp, apps/sent2vec/sent2vec.cpp,
// apps/logistic/lr.cpp) become when they link libswps instead of the
// MPI/ZeroMQ parameter server.  Used by tests/test_compat_gpu.py.
//
//   compat_apps w2v    -config C -data D -niters N -output O
//   compat_apps s2v    -config C -data D -niters N -wordvec W -output O
//   compat_apps lr     -config C -data D -niters N -output O [-param P]
//                      (per-epoch MSE; -param: the trained shard's dump, lr.cpp:488-492)
//   compat_apps lrpredict -config C -data D -param P -output O  (lr.cpp:498-504)
//   compat_apps ps     -config C                               (PS-level client)
//   compat_apps rules  -config C -case K   (access-method rule resolution)
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>

#include "swiftmpi_compat.h"

using namespace swift_snails;

// ---- the PS-level value types of word2vec_global.h:50-100, restated ------
static int g_dim = 0;
struct WLocalParam {
  std::vector<double> h, v;
  WLocalParam() : h(g_dim, 0.0), v(g_dim, 0.0) {}
};
struct WLocalGrad {
  std::vector<double> h_grad, v_grad;
  int h_count = 0, v_count = 0;
  WLocalGrad() : h_grad(g_dim, 0.0), v_grad(g_dim, 0.0) {}
  void accu_h(const std::vector<double> &g) {
    h_count++;
    for (int i = 0; i < g_dim; i++) h_grad[i] += g[i];
  }
  void accu_v(const std::vector<double> &g) {
    v_count++;
    for (int i = 0; i < g_dim; i++) v_grad[i] += g[i];
  }
};
namespace swift_snails {
template <> struct PullCodec<WLocalParam> {
  typedef double wire_t;
  static const int32_t layout = SWPS_LAYOUT_W2V;
  static int elems() { return 2 * g_dim; }
  static void decode(const double *w, WLocalParam &p) {
    p.h.assign(w, w + g_dim);
    p.v.assign(w + g_dim, w + 2 * g_dim);
  }
};
template <> struct PushCodec<WLocalGrad> {  // the mean, word2vec_global.h:122-134
  static void encode(WLocalGrad &g, double *w) {
    for (int i = 0; i < g_dim; i++) {
      w[i] = g.h_count > 0 ? g.h_grad[i] / g.h_count : g.h_grad[i];
      w[g_dim + i] = g.v_count > 0 ? g.v_grad[i] / g.v_count : g.v_grad[i];
    }
    g = WLocalGrad();
  }
};
}  // namespace swift_snails

typedef LocalParamCache<uint64_t, WLocalParam, WLocalGrad> cache_t;

// the reference app's access-method classes keep their shape
// (word2vec_global.h:158-191); the device applies the rule they select
class WPullAccessMethod : public PullAccessMethod<uint64_t, WLocalParam, WLocalParam> {};
class WPushAccessMethod : public PushAccessMethod<uint64_t, WLocalParam, WLocalGrad> {};
typedef ClusterServer<uint64_t, WLocalParam, WLocalParam, WLocalGrad, WPullAccessMethod, WPushAccessMethod> server_t;

// access methods with their own host bodies (word2vec_global.h:158-191 shape)
class BodyPushAccessMethod : public PushAccessMethod<uint64_t, WLocalParam, WLocalGrad> {
 public:
  void apply_push_value(const uint64_t &, WLocalParam &, const WLocalGrad &) {}
};
class DeclaredPushAccessMethod : public PushAccessMethod<uint64_t, WLocalParam, WLocalGrad> {
 public:
  static const int32_t push_rule = SWPS_PUSH_ADAGRAD;  // what its body computes
  void apply_push_value(const uint64_t &, WLocalParam &, const WLocalGrad &) {}
};
class UnknownPushAccessMethod : public PushAccessMethod<uint64_t, WLocalParam, WLocalGrad> {
 public:
  static const int32_t push_rule = 7;  // a rule the library lacks
};
class BodyPullAccessMethod : public PullAccessMethod<uint64_t, WLocalParam, WLocalParam> {
 public:
  void init_param(const uint64_t &, WLocalParam &) {}
};

// rule resolution of a ClusterServer: prints the resolved rules (errors exit 3)
template <class PullM, class PushM> static int rules_of() {
  typedef ClusterServer<uint64_t, WLocalParam, WLocalParam, WLocalGrad, PullM, PushM> s_t;
  std::printf("init_mode=%d push_rule=%d\n", (int)s_t::init_mode(), (int)s_t::push_rule());
  g_dim = global_config().get("word2vec", "len_vec").to_int32();
  Cluster<ClusterWorker, s_t, uint64_t> cluster(64);
  cluster.finalize();
  return 0;
}
static int rules(const std::string &k) {
  if (k == "plain") return rules_of<WPullAccessMethod, WPushAccessMethod>();
  if (k == "push_body") return rules_of<WPullAccessMethod, BodyPushAccessMethod>();
  if (k == "push_declared") return rules_of<WPullAccessMethod, DeclaredPushAccessMethod>();
  if (k == "push_unknown") return rules_of<WPullAccessMethod, UnknownPushAccessMethod>();
  if (k == "pull_body") return rules_of<BodyPullAccessMethod, WPushAccessMethod>();
  return 2;
}

// rank r's keys: overlapping sets, so owners see several sources per key
static bool has_key(uint64_t i, int r) { return (i + (uint64_t)r) % 3 != 0; }
static uint64_t key_of(uint64_t i) { return i * 2654435761ULL; }
static void grads_of(uint64_t k, int r, std::vector<double> &g1, std::vector<double> &g2, std::vector<double> &g3) {
  for (int i = 0; i < g_dim; i++) {
    g1[i] = std::sin((double)(k % 97) + i + r);
    g2[i] = std::cos((double)(k % 89) * i - r);
    g3[i] = 0.25 * i - 1.0 + 0.1 * r;
  }
}

// PS-level client (the reference apps' pull / learn / push cycle with a
// host learn step): on one rank, or key-sharded over several (RANK /
// WORLD_SIZE; every rank's push is its own AdaGrad step, in rank order)
static int ps_client() {
  g_dim = global_config().get("word2vec", "len_vec").to_int32();
  const double lr = global_config().get("server", "initial_learning_rate").to_float();
  Cluster<ClusterWorker, server_t, uint64_t> cluster(4096, SWPS_F64);
  cluster.initialize();
  const int rank = cluster.rank(), world = cluster.world();
  std::unordered_set<uint64_t> keys;
  for (uint64_t i = 1; i <= 300; i++)
    if (has_key(i, rank)) keys.insert(key_of(i));
  cache_t cache, again;
  cache.init_keys(keys);
  global_pull_access<uint64_t, WLocalParam, WLocalGrad>().pull_with_barrier(keys, cache);
  again.init_keys(keys);
  global_pull_access<uint64_t, WLocalParam, WLocalGrad>().pull_with_barrier(keys, again);
  for (auto k : keys) {
    const WLocalParam &a = cache.params()[k], &b = again.params()[k];
    for (int i = 0; i < g_dim; i++)
      if (a.h[i] != b.h[i] || a.v[i] != b.v[i] || std::fabs(a.h[i]) > 0.5 / g_dim) {
        std::printf("FAIL pull k=%llu\n", (unsigned long long)k);
        return 1;
      }
  }
  // accumulate two gradients per key, push the mean
  std::vector<double> g1(g_dim), g2(g_dim), g3(g_dim);
  for (auto k : keys) {
    grads_of(k, rank, g1, g2, g3);
    cache.grads()[k].accu_h(g1);
    cache.grads()[k].accu_h(g2);
    cache.grads()[k].accu_v(g3);
  }
  global_push_access<uint64_t, WLocalParam, WLocalGrad>().push_with_barrier(keys, cache);
  cache_t after;
  after.init_keys(keys);
  global_pull_access<uint64_t, WLocalParam, WLocalGrad>().pull_with_barrier(keys, after);
  // expected: word2vec_global.h:176-185 from h2 = v2 = 0, one step per rank
  // holding the key, ranks in order
  const double fudge = (double)1e-6f;
  double worst = 0;
  for (uint64_t ii = 1; ii <= 300; ii++) {
    if (!has_key(ii, rank)) continue;
    const uint64_t k = key_of(ii);
    for (int i = 0; i < g_dim; i++) {
      double h = again.params()[k].h[i], v = again.params()[k].v[i], h2 = 0, v2 = 0;
      for (int r = 0; r < world; r++) {
        if (!has_key(ii, r)) continue;
        grads_of(k, r, g1, g2, g3);
        const double a = (g1[i] + g2[i]) / 2, b = g3[i];
        h2 = h2 + a * a;
        v2 = v2 + b * b;
        h = h + (a * lr) / std::sqrt(h2 + fudge);
        v = v + (b * lr) / std::sqrt(v2 + fudge);
      }
      worst = std::fmax(worst, std::fabs(after.params()[k].h[i] - h));
      worst = std::fmax(worst, std::fabs(after.params()[k].v[i] - v));
    }
    if (cache.grads()[k].h_count != 0) {
      std::printf("FAIL grads not reset\n");
      return 1;
    }
  }
  // the last rank keeps working after the others finished: their shards
  // still serve it (swps_finish)
  if (world > 1 && rank == world - 1) {
    cache_t late;
    late.init_keys(keys);
    global_pull_access<uint64_t, WLocalParam, WLocalGrad>().pull_with_barrier(keys, late);
    for (auto k : keys)
      for (int i = 0; i < g_dim; i++)
        if (late.params()[k].h[i] != after.params()[k].h[i]) {
          std::printf("FAIL late pull\n");
          return 1;
        }
  }
  cluster.finalize();
  std::printf("ps ok rank=%d world=%d routed=%d keys=%zu max|diff|=%.3g\n", rank, world, (int)cluster.routed(),
              keys.size(), worst);
  return worst < 1e-12 ? 0 : 1;
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const std::string mode = argv[1];
  std::map<std::string, std::string> a;
  for (int i = 2; i + 1 < argc; i += 2) a[argv[i]] = argv[i + 1];
  try {
    global_config().load_conf(a["-config"]);
    global_config().parse();
    if (mode == "ps") return ps_client();
    if (mode == "rules") return rules(a["-case"]);
    const int niters = std::atoi(a["-niters"].c_str());
    if (mode == "w2v") {  // apps/word2vec/w2v.cpp:5-61
      Cluster<ClusterWorker, W2VServer, uint64_t> cluster;
      cluster.initialize();
      Word2VecApp w2v(a["-data"], niters);
      w2v.train();
      const std::string out = a["-output"] + "-" + std::to_string(cluster.rank()) + ".txt";  // w2v.cpp:54
      cluster.finalize(out);
    } else if (mode == "s2v") {  // apps/sent2vec/sent2vec.cpp:198-257
      Cluster<ClusterWorker, W2VServer, uint64_t> cluster;
      cluster.initialize();
      Sent2VecApp s2v(a["-data"], a["-output"], niters);
      s2v.load_word_vector(a["-wordvec"]);
      s2v.train();
    } else if (mode == "lr") {  // apps/logistic/lr.cpp:413-509 (train mode)
      Cluster<ClusterWorker, LRServer, uint32_t> cluster;
      cluster.initialize();
      LRApp lr(a["-data"]);
      std::vector<double> err = lr.train(niters);
      FILE *f = std::fopen(a["-output"].c_str(), "w");
      for (double e : err) std::fprintf(f, "%.17g\n", e);
      std::fclose(f);
      cluster.finalize(a["-param"]);  // lr.cpp:488-492 (no dump when -param is absent)
    } else if (mode == "lrpredict") {  // apps/logistic/lr.cpp:498-504 (predict mode)
      Cluster<ClusterWorker, LRServer, uint32_t> cluster;
      cluster.initialize();
      LRApp lr(a["-data"]);
      lr.load_param(a["-param"]);
      lr.predict(a["-data"], a["-output"]);
      cluster.finalize();
    } else {
      return 2;
    }
  } catch (SwpsError &e) {
    std::fprintf(stderr, "error %d: %s\n", e.code, e.what());
    return 3;
  }
  std::printf("%s ok\n", mode.c_str());
  return 0;
}
