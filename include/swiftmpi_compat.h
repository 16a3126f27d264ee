/*
 * swiftmpi_compat.h — C++11 host-side drop-in for SwiftMPI's parameter-server
 * key-value API (src/parameter) and its app entry points (src/apps), over the
 * C ABI of libswps.so (swps.h).  Header-only; needs no MPI, ZeroMQ, glog or
 * sparsehash.  Link with -lswps.
 *
 * Reference interfaces mirrored (paths relative to logicxin/SwiftMPI src/):
 *   ConfigParser / global_config()     utils/ConfigParser.h:25-133
 *   LocalParamCache<Key,Param,Grad>    parameter/param.h:13-68
 *   GlobalPullAccess<Key,Val,Grad>     parameter/global_pull_access.h:15-118
 *   GlobalPushAccess<Key,Val,Grad>     parameter/global_push_access.h:15-106
 *   Cluster<Worker,Server,Key>         cluster/cluster.h:9-140 (initialize/finalize)
 *   ClusterServer<Key,Param,PullVal,Grad,PullM,PushM>  cluster/server.h:20-101
 *   PullAccessMethod / PushAccessMethod parameter/accessmethod.h:7-35
 *   Word2VecApp                        apps/word2vec/word2vec_global.h:541-748 + w2v.cpp
 *   Sent2VecApp                        apps/sent2vec/sent2vec.cpp:14-257
 *   LRApp                              apps/logistic/lr.cpp:133-509
 *
 * Two levels, as in swps.h:
 *   * PS level: an app keeps its own learn_instance on the host and calls
 *     pull_with_barrier / push_with_barrier exactly as before; keys and
 *     values cross into the HBM shard through swps_pull_h / swps_push_h.
 *     A PullCodec / PushCodec specialisation states how the app's value
 *     types map onto the reference's wire layouts (word2vec_global.h:122-156,
 *     lr.cpp:32-43) — the role BinaryBuffer operator<< / >> play there.
 *   * App level: the whole minibatch loop runs on the GPU (swps_w2v_*,
 *     swps_s2v_*, swps_lr_*); the classes below read the same config keys
 *     as the reference's app constructors.
 * Errors: the reference CHECK-aborts; here every failure throws SwpsError
 * carrying swps_last_error().
 */
#ifndef SWIFTMPI_COMPAT_H_
#define SWIFTMPI_COMPAT_H_

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <type_traits>
#include <limits>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "swps.h"

namespace swift_snails {

struct SwpsError : std::runtime_error {
  int code;
  SwpsError(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

inline void swps_check(int rc) {
  if (rc != SWPS_OK) throw SwpsError(rc, swps_last_error());
}

/* ---- utils/ConfigParser.h ------------------------------------------------ */
class ConfigValue {
 public:
  ConfigValue() {}
  explicit ConfigValue(const std::string &s) : _s(s) {}
  int to_int32() const { return std::atoi(_s.c_str()); }
  float to_float() const { return (float)std::atof(_s.c_str()); }
  std::string to_string() const { return _s; }
  bool empty() const { return _s.empty(); }

 private:
  std::string _s;
};

/* "[section]" headers, "key: value" lines, '#' comments, "import path";
 * the first definition of a key wins (std::map::insert); get() of a missing
 * key throws (the reference CHECK-fails, ConfigParser.h:64-69). */
class ConfigParser {
 public:
  void load_conf(const std::string &path) { _path = path; }
  void parse() { parse_file(_path); }
  ConfigValue get(const std::string &section, const std::string &key) const {
    auto s = _data.find(section);
    if (s != _data.end()) {
      auto k = s->second.find(key);
      if (k != s->second.end()) return ConfigValue(k->second);
    }
    throw SwpsError(SWPS_E_CFG, "no such key:\t[" + section + "]\t" + key);
  }
  bool has(const std::string &section, const std::string &key) const {
    auto s = _data.find(section);
    return s != _data.end() && s->second.count(key);
  }

 private:
  static std::string trim(const std::string &s) {
    const size_t a = s.find_first_not_of(" \t\n\r");
    if (a == std::string::npos) return std::string();
    const size_t b = s.find_last_not_of(" \t\n\r");
    return s.substr(a, b - a + 1);
  }
  void parse_file(const std::string &path) {
    std::ifstream f(path.c_str());
    if (!f) throw SwpsError(SWPS_E_IO, "conf can not open: " + path);
    std::string line, cur;
    while (std::getline(f, line)) {
      line = trim(line);
      if (line.empty() || line[0] == '#') continue;
      if (line.compare(0, 6, "import") == 0) {
        const std::string p = trim(line.substr(line.find(' ') + 1));
        if (p == path) throw SwpsError(SWPS_E_CFG, "recursive import");
        parse_file(p);
        continue;
      }
      if (line[0] == '[' && line[line.size() - 1] == ']') {
        cur = trim(line.substr(1, line.size() - 2));
        continue;
      }
      const size_t c = line.find(':');
      if (c == std::string::npos) throw SwpsError(SWPS_E_CFG, "bad config line: " + line);
      _data[cur].insert(std::make_pair(trim(line.substr(0, c)), trim(line.substr(c + 1))));
    }
  }
  std::string _path;
  std::map<std::string, std::map<std::string, std::string> > _data;
};

inline ConfigParser &global_config() {
  static ConfigParser c;
  return c;
}

/* ---- utils/Buffer.h BinaryBuffer ------------------------------------------
 * The byte buffer the reference's apps serialise their pull values and
 * gradients into (operator<< / >> of basic types, Buffer.h:169-230): the
 * generic codecs below run an app's own operator<< (BinaryBuffer&, Grad&) /
 * operator>> to produce and consume the wire values. */
class BinaryBuffer {
 public:
  BinaryBuffer() {}
  BinaryBuffer(const char *p, size_t n) : _b(p, p + n) {}
#define SWPS_BB_POD(T)                        \
  BinaryBuffer &operator<<(const T &x) {      \
    const char *p = (const char *)&x;         \
    _b.insert(_b.end(), p, p + sizeof(T));    \
    return *this;                             \
  }                                           \
  BinaryBuffer &operator>>(T &x) {            \
    if (_r + sizeof(T) > _b.size())           \
      throw SwpsError(SWPS_E_IO, "BinaryBuffer: read past the end"); \
    std::memcpy(&x, &_b[_r], sizeof(T));      \
    _r += sizeof(T);                          \
    return *this;                             \
  }
  SWPS_BB_POD(int16_t)
  SWPS_BB_POD(uint16_t)
  SWPS_BB_POD(int32_t)
  SWPS_BB_POD(uint32_t)
  SWPS_BB_POD(long)
  SWPS_BB_POD(unsigned long)
  SWPS_BB_POD(long long)
  SWPS_BB_POD(unsigned long long)
  SWPS_BB_POD(float)
  SWPS_BB_POD(double)
  SWPS_BB_POD(bool)
  SWPS_BB_POD(char)
#undef SWPS_BB_POD
  bool read_finished() const { return _r >= _b.size(); }
  size_t size() const { return _b.size(); }
  char *buffer() { return _b.empty() ? nullptr : &_b[0]; }
  const char *buffer() const { return _b.empty() ? nullptr : &_b[0]; }
  void clear() {
    _b.clear();
    _r = 0;
  }

 private:
  std::vector<char> _b;
  size_t _r = 0;
};

/* ---- utils/random.h Random / global_random() -------------------------------
 * The reference's two LCGs (random.h:25-37): operator() and gen_float().
 * A table whose init rule is SWPS_INIT_FLCG continues this float stream on
 * the device from the state it had when the shard was created. */
struct Random {
  explicit Random(unsigned long long seed) : next_random(seed) {}
  unsigned long long operator()() {
    next_random = next_random * (unsigned long long)25214903917 + 11;
    return next_random;
  }
  float gen_float() {
    next_float_random = next_float_random * (unsigned long)4903917 + 11;
    return float(next_float_random) / std::numeric_limits<unsigned long>::max();
  }
  unsigned long float_state() const { return next_float_random; }

 private:
  unsigned long long next_random = 0;
  unsigned long next_float_random = std::numeric_limits<unsigned long>::max() / 2;
};
inline Random &global_random() {
  static Random r(2008);
  return r;
}

/* ---- the reference process's libc rand() stream -------------------------------
 * Vec::randInit and the server's WParam draw glibc rand() after the default srand(1)
 * (vec1.h:229-232, word2vec.h:38-44).  In this process the ROCm runtime calls srand() and rand()
 * itself (libhsa-runtime64 imports both, at HIP initialisation and later), which would reseed and
 * advance that stream under the app at run-dependent points.  The apps' draws therefore come from
 * this copy of it: glibc's TYPE_3 additive generator — r[i] = r[i-31] + r[i-3] (mod 2^32) seeded
 * by the 16807 LCG, r[31..33] = r[0..2], 310 outputs discarded, each output r >> 1 — which returns
 * what rand() returns in a process that calls nothing else (tests/test_compat.py checks it against
 * libc).  One stream per process, like rand(); not thread-safe, like the reference's nthreads = 1. */
class ProcessRand {
 public:
  explicit ProcessRand(uint32_t seed = 1) {
    int32_t w = seed ? (int32_t)seed : 1;
    _r[0] = (uint32_t)w;
    for (int i = 1; i < 31; i++) {
      const int32_t hi = w / 127773, lo = w % 127773;
      w = 16807 * lo - 2836 * hi;
      if (w < 0) w += 2147483647;
      _r[i] = (uint32_t)w;
    }
    for (int i = 31; i < 34; i++) _r[i] = _r[i - 31];
    _i = 34;
    for (int k = 0; k < 310; k++) next_raw();
  }
  int operator()() { return (int)(next_raw() >> 1); }

 private:
  uint32_t next_raw() {
    const uint32_t v = _r[(_i - 31) % 34] + _r[(_i - 3) % 34];
    _r[_i % 34] = v;
    _i++;
    return v;
  }
  uint32_t _r[34];
  uint64_t _i;
};
inline ProcessRand &process_rand() {
  static ProcessRand r(1);
  return r;
}

/* ---- wire codecs ----------------------------------------------------------
 * Typed form (a specialisation states the wire directly):
 *   PullCodec<Val>:  typedef wire_t (double for word2vec, float for LR);
 *                    static int elems();  static void decode(const wire_t*, Val&)
 *   PushCodec<Grad>: static void encode(Grad&, wire_t*)  — writes the MEAN
 *                    gradient the reference's serializer sends and resets it
 *                    (word2vec_global.h:122-134, lr.cpp:32-38).
 * Generic form (no specialisation — what an unchanged reference app gets):
 * the app's own BinaryBuffer operators, exactly as its messages carried the
 * values (global_pull_access.h:88-97, global_push_access.h:86-90): a pull
 * value is read with `bb >> val`, a gradient written with `bb << grad` (a
 * gradient that writes nothing — lr.cpp:34-35 with count 0 — is not pushed)
 * and then reset with its reset() (global_push_access.h:49, 64) or to
 * Grad().  Layout: a scalar pull value is the LR layout, anything else the
 * word2vec one (its wire interleaves h[i], v[i]; the library's value blocks
 * are converted). */
namespace detail {
template <class V> struct is_generic_layout {
  static const int32_t value = std::is_arithmetic<V>::value ? SWPS_LAYOUT_LR : SWPS_LAYOUT_W2V;
};
}  // namespace detail
template <class Val> struct PullCodec {
  static const bool generic = true;
  static const int32_t layout = detail::is_generic_layout<Val>::value;
};
template <class Grad> struct PushCodec {
  static const bool generic = true;
};

namespace detail {
template <class C> struct is_generic {
  template <class U> static char test(decltype(&U::generic));
  template <class U> static long test(...);
  static const bool value = sizeof(test<C>(nullptr)) == 1;
};
template <class G> struct has_reset {
  template <class U> static char test(decltype(&U::reset));
  template <class U> static long test(...);
  static const bool value = sizeof(test<G>(nullptr)) == 1;
};
template <class G> void reset_grad(G &g, std::true_type) { g.reset(); }
template <class G> void reset_grad(G &g, std::false_type) { g = G(); }
template <class G> void reset_grad(G &g) { reset_grad(g, std::integral_constant<bool, has_reset<G>::value>()); }
/* the library's W2V value blocks [a(D) | b(D)] <-> the reference wire's a[i], b[i] pairs */
inline void interleave(const char *blk, char *wire, size_t keys, int D, size_t es) {
  for (size_t k = 0; k < keys; k++)
    for (int i = 0; i < D; i++) {
      std::memcpy(wire + ((k * D + i) * 2) * es, blk + (k * 2 * D + i) * es, es);
      std::memcpy(wire + ((k * D + i) * 2 + 1) * es, blk + (k * 2 * D + D + i) * es, es);
    }
}
inline void deinterleave(const char *wire, char *blk, size_t keys, int D, size_t es) {
  for (size_t k = 0; k < keys; k++)
    for (int i = 0; i < D; i++) {
      std::memcpy(blk + (k * 2 * D + i) * es, wire + ((k * D + i) * 2) * es, es);
      std::memcpy(blk + (k * 2 * D + D + i) * es, wire + ((k * D + i) * 2 + 1) * es, es);
    }
}
inline size_t wire_bytes(int32_t layout) { return layout == SWPS_LAYOUT_W2V ? 8 : 4; }
}  // namespace detail

/* The shard this process serves and pulls from (one GPU = one shard). */
inline swps_table *&global_swps_table() {
  static swps_table *t = nullptr;
  return t;
}
/* The multi-rank job's communicator (null on one rank), its frag_num, and
 * the shard's configuration (Cluster sets them). */
inline swps_comm *&global_swps_comm() {
  static swps_comm *c = nullptr;
  return c;
}
inline int &global_frag_num() {
  static int f = 1000;
  return f;
}
inline swps_table_cfg &global_swps_cfg() {
  static swps_table_cfg c;
  return c;
}
/* BasicHashFrag node id of this rank's shard (rank + 1, hashfrag.h:33-56) and the node count */
inline std::pair<int, int> &global_node() {
  static std::pair<int, int> n(1, 1);
  return n;
}

/* ---- parameter/accessmethod.h ---------------------------------------------
 * The reference's server runs the app's access-method objects per key on
 * the CPU (accessmethod.h:16-33); here the owner GPU applies one of the
 * library's device rules to whole batches.  An app's access-method classes
 * keep their reference shape and select the device rule through two
 * constants:
 *   PullM::init_mode = SWPS_INIT_HASH or SWPS_INIT_ZERO       (init_param)
 *   PushM::push_rule = SWPS_PUSH_ADAGRAD or SWPS_PUSH_SGD     (apply_push_value)
 * A class that leaves them unset inherits "unspecified", which resolves to
 * the rule every reference app implements (AdaGrad, word2vec_global.h:
 * 176-185 / lr.cpp:68-75; hashed random init) — unless the class defines its
 * own init_param / get_pull_value / apply_push_value body: the library cannot
 * run host bodies on the device, so such a class must state the rule its
 * body computes (one line, e.g. `static const int32_t push_rule =
 * SWPS_PUSH_ADAGRAD;` in the reference's WPushAccessMethod), and creating
 * its ClusterServer otherwise throws SwpsError(SWPS_E_UNSUPPORTED).  A rule
 * value the library lacks fails the same way (swps_table_create). */
const int32_t SWPS_RULE_UNSPECIFIED = -1;

template <typename Key, typename Param, typename PullVal> class PullAccessMethod {
 public:
  typedef Key key_t;
  typedef Param param_t;
  typedef PullVal pull_t;
  static const int32_t init_mode = SWPS_RULE_UNSPECIFIED;
  virtual ~PullAccessMethod() {}
};
template <typename Key, typename Param, typename Grad> class PushAccessMethod {
 public:
  typedef Key key_t;
  typedef Param param_t;
  typedef Grad grad_t;
  static const int32_t push_rule = SWPS_RULE_UNSPECIFIED;
  virtual ~PushAccessMethod() {}
};

namespace detail {
/* does M (or a base between it and the library's) define a host body? */
template <class M> struct has_init_param {
  template <class U> static char test(decltype(&U::init_param));
  template <class U> static long test(...);
  static const bool value = sizeof(test<M>(nullptr)) == 1;
};
template <class M> struct has_get_pull_value {
  template <class U> static char test(decltype(&U::get_pull_value));
  template <class U> static long test(...);
  static const bool value = sizeof(test<M>(nullptr)) == 1;
};
template <class M> struct has_apply_push_value {
  template <class U> static char test(decltype(&U::apply_push_value));
  template <class U> static long test(...);
  static const bool value = sizeof(test<M>(nullptr)) == 1;
};
inline int32_t resolve_rule(int32_t declared, bool host_body, int32_t dflt, const char *what) {
  if (declared != SWPS_RULE_UNSPECIFIED) return declared;
  if (host_body)
    throw SwpsError(SWPS_E_UNSUPPORTED, std::string("the access method defines its own ") + what +
                                            " body, which the library cannot run on the device: declare the rule "
                                            "it computes (see swiftmpi_compat.h, parameter/accessmethod.h)");
  return dflt;
}
inline SwpsError unrecognised(const char *what) {
  return SwpsError(SWPS_E_UNSUPPORTED, std::string("the access method's ") + what +
                                           " body computes none of the library's device rules: declare the rule "
                                           "it computes (see swiftmpi_compat.h, parameter/accessmethod.h)");
}
template <class G> struct has_bb_read {
  template <class U>
  static char test(typename std::remove_reference<decltype(std::declval<BinaryBuffer &>() >> std::declval<U &>())>::type *);
  template <class U> static long test(...);
  static const bool value = sizeof(test<G>(nullptr)) == 1;
};
inline bool near(float x, float e) { return std::fabs(x - e) <= 1e-6f * std::fmax(1.f, std::fabs(e)); }

/* Recognising an unchanged app's host bodies (an app whose access methods
 * keep the reference's shape, lr.cpp:45-80, and declare nothing): for a
 * scalar pull value the bodies are RUN once on the host against probe values
 * and matched to a device rule — they are never the rule that trains.
 *   init_param:        twice: 0, 0 -> SWPS_INIT_ZERO; the next two
 *                      global_random().gen_float() draws -> SWPS_INIT_FLCG
 *                      (global_random() is left as it was)
 *   apply_push_value:  two steps from Param(), read back through
 *                      get_pull_value, = AdaGrad (fudge 1e-6f) or SGD with
 *                      [server] initial_learning_rate
 * Anything else, or a value type that is not a scalar, fails as before. */
template <class Key, class Param, class PullVal, class Grad, class PullM, class PushM, bool Scalar =
                                                                                           std::is_arithmetic<PullVal>::value &&
                                                                                           has_get_pull_value<PullM>::value>
struct RuleProbe {
  static int32_t init_mode() { throw unrecognised("init_param / get_pull_value"); }
  static int32_t push_rule() { throw unrecognised("apply_push_value"); }
};
template <class Key, class Param, class PullVal, class Grad, class PullM, class PushM>
struct RuleProbe<Key, Param, PullVal, Grad, PullM, PushM, true> {
  static PullVal read(PullM &m, const Param &p) {
    PullVal v = PullVal();
    m.get_pull_value(Key(), p, v);
    return v;
  }
  static int32_t init_mode() { return init_mode(std::integral_constant<bool, has_init_param<PullM>::value>()); }
  static int32_t init_mode(std::false_type) { return SWPS_INIT_ZERO; }  // Param() as it is
  static int32_t init_mode(std::true_type) {
    PullM m;
    Param p = Param(), q = Param();
    const Random saved = global_random();
    Random next = saved;
    const float d1 = next.gen_float(), d2 = next.gen_float();  // two draws: the stream's first is 0.5
    m.init_param(Key(), p);
    m.init_param(Key(), q);
    global_random() = saved;
    const float v1 = (float)read(m, p), v2 = (float)read(m, q);
    if (v1 == 0.f && v2 == 0.f) return SWPS_INIT_ZERO;
    if (v1 == d1 && v2 == d2) return SWPS_INIT_FLCG;
    throw unrecognised("init_param");
  }
  static int32_t push_rule() { return push_rule(std::integral_constant<bool, has_bb_read<Grad>::value>()); }
  static int32_t push_rule(std::false_type) { throw unrecognised("apply_push_value"); }
  static Grad grad_of(float x) {  // what the server deserialises from the wire (global_push_access.h:86-90)
    BinaryBuffer bb;
    bb << x;
    Grad g = Grad();
    bb >> g;
    return g;
  }
  static int32_t push_rule(std::true_type) {
    PushM m;
    PullM pm;
    const float lr = global_config().get("server", "initial_learning_rate").to_float();
    const float fudge = 1e-6f, a = 0.5f, b = -0.25f;
    Param p = Param();
    const float v0 = (float)read(pm, p);
    m.apply_push_value(Key(), p, grad_of(a));
    const float v1 = (float)read(pm, p);
    m.apply_push_value(Key(), p, grad_of(b));
    const float v2 = (float)read(pm, p);
    const float g2a = a * a, g2b = g2a + b * b;
    const float ada1 = v0 + lr * a / float(std::sqrt(g2a + fudge));
    if (near(v1, ada1) && near(v2, ada1 + lr * b / float(std::sqrt(g2b + fudge)))) return SWPS_PUSH_ADAGRAD;
    if (near(v1, v0 + lr * a) && near(v2, v0 + lr * a + lr * b)) return SWPS_PUSH_SGD;
    throw unrecognised("apply_push_value");
  }
};
}  // namespace detail

/* ---- cluster/server.h ClusterServer --------------------------------------
 * The server half of a rank: its HBM shard's layout comes from the pull
 * value's codec (PullCodec<PullVal>::layout), its miss initialisation and
 * push rule from the access methods.  Cluster<Worker, ClusterServer<...>,
 * Key> creates the shard; load() assigns the dump's keys this rank owns
 * (server.h:49-62), global_server<server_t>().load(path) as in lr.cpp:297-300. */
template <typename Key, typename Param, typename PullVal, typename Grad, typename PullM, typename PushM>
class ClusterServer {
 public:
  typedef Key key_t;
  typedef Param param_t;
  typedef PullVal pull_t;
  typedef Grad grad_t;
  typedef PullM pull_access_t;
  typedef PushM push_access_t;
  typedef detail::RuleProbe<Key, Param, PullVal, Grad, PullM, PushM> probe_t;
  static int32_t layout() { return PullCodec<PullVal>::layout; }
  static int32_t init_mode() {
    const bool body = detail::has_init_param<PullM>::value || detail::has_get_pull_value<PullM>::value;
    if (PullM::init_mode == SWPS_RULE_UNSPECIFIED && body && std::is_arithmetic<PullVal>::value)
      return probe_t::init_mode();  // an unchanged reference app's bodies (see detail::RuleProbe)
    return detail::resolve_rule(PullM::init_mode, body, SWPS_INIT_HASH, "init_param / get_pull_value");
  }
  /* SWPS_INIT_FLCG continues global_random()'s float stream from here */
  static uint64_t init_seed() { return init_mode() == SWPS_INIT_FLCG ? global_random().float_state() : 0; }
  static int32_t push_rule() {
    const bool body = detail::has_apply_push_value<PushM>::value;
    if (PushM::push_rule == SWPS_RULE_UNSPECIFIED && body && std::is_arithmetic<PullVal>::value)
      return probe_t::push_rule();
    return detail::resolve_rule(PushM::push_rule, body, SWPS_PUSH_ADAGRAD, "apply_push_value");
  }
  void load(const std::string &path);  // defined after Cluster's globals
};

/* ---- parameter/param.h ---------------------------------------------------- */
template <typename Key, typename Param, typename Grad> class LocalParamCache {
 public:
  typedef Key key_t;
  typedef Param param_t;
  typedef Grad grad_t;

  void init_keys(const std::unordered_set<key_t> &keys) {
    for (const auto &key : keys) {
      _params[key] = param_t();
      _grads[key] = grad_t();
    }
  }
  void clear() {
    _params.clear();
    _grads.clear();
  }
  size_t size() const { return _params.size(); }
  std::unordered_map<key_t, param_t> &params() { return _params; }
  std::unordered_map<key_t, grad_t> &grads() { return _grads; }

 private:
  std::unordered_map<key_t, param_t> _params;
  std::unordered_map<key_t, grad_t> _grads;
};

/* ---- parameter/global_pull_access.h --------------------------------------
 * pull_with_barrier: params[key] = pulled value, grads[key] reset
 * (global_pull_access.h:88-97).  Keys new to the shard are initialised by it
 * (accessmethod.h:63-70).  On a multi-rank Cluster the keys go to their
 * BasicHashFrag owners inside the library (swps_table_route): every rank
 * calls pull / push in the same sequence, an empty key set included (the
 * reference blocks forever on one, global_pull_access.h:33-42; here it
 * joins the exchange and returns). */
template <typename Key, typename Val, typename Grad> class GlobalPullAccess {
 public:
  typedef LocalParamCache<Key, Val, Grad> param_cache_t;

  explicit GlobalPullAccess(swps_table *t = nullptr) : _t(t) {}

  void pull_with_barrier(const std::unordered_set<Key> &keys, param_cache_t &cache) {
    swps_table *t = _t ? _t : global_swps_table();
    if (!t) throw SwpsError(SWPS_E_STATE, "no shard: create a Cluster first");
    std::vector<uint64_t> k;
    k.reserve(keys.size());
    for (const auto &key : keys) k.push_back((uint64_t)key);
    pull(t, k, cache, std::integral_constant<bool, detail::is_generic<PullCodec<Val> >::value>());
  }

 private:
  static void pull(swps_table *t, const std::vector<uint64_t> &k, param_cache_t &cache, std::false_type) {
    typedef typename PullCodec<Val>::wire_t wire_t;
    const int P = PullCodec<Val>::elems();
    std::vector<wire_t> vals(k.size() * (size_t)P);
    swps_check(swps_pull_h(t, k.data(), k.size(), vals.data()));
    for (size_t i = 0; i < k.size(); i++) {
      const Key key = (Key)k[i];
      PullCodec<Val>::decode(&vals[i * P], cache.params()[key]);
      cache.grads()[key] = Grad();
    }
  }
  static void pull(swps_table *t, const std::vector<uint64_t> &k, param_cache_t &cache, std::true_type) {
    int32_t row = 0, P = 0, push = 0;
    swps_check(swps_table_row_elems(t, &row, &P, &push));
    const int32_t layout = PullCodec<Val>::layout;
    const size_t es = detail::wire_bytes(layout), stride = (size_t)P * es;
    std::vector<char> raw(k.size() * stride + 1), wire;
    swps_check(swps_pull_h(t, k.data(), k.size(), &raw[0]));
    const char *src = &raw[0];
    if (layout == SWPS_LAYOUT_W2V) {  // the reference's wire: h[i], v[i] pairs
      wire.resize(raw.size());
      detail::interleave(&raw[0], &wire[0], k.size(), P / 2, es);
      src = &wire[0];
    }
    for (size_t i = 0; i < k.size(); i++) {
      const Key key = (Key)k[i];
      BinaryBuffer bb(src + i * stride, stride);
      bb >> cache.params()[key];  // the app's own deserialiser (global_pull_access.h:88-97)
      cache.grads()[key] = Grad();
    }
  }
  swps_table *_t;
};

/* ---- parameter/global_push_access.h --------------------------------------
 * push_with_barrier: the mean gradient of every key present in the cache's
 * grads is applied by the shard's push rule (AdaGrad, word2vec_global.h:
 * 176-185 / lr.cpp:68-75) and the local gradient is reset
 * (global_push_access.h:48-67). */
template <typename Key, typename Val, typename Grad> class GlobalPushAccess {
 public:
  typedef LocalParamCache<Key, Val, Grad> param_cache_t;

  explicit GlobalPushAccess(swps_table *t = nullptr) : _t(t) {}

  void push_with_barrier(const std::unordered_set<Key> &keys, param_cache_t &cache) {
    swps_table *t = _t ? _t : global_swps_table();
    if (!t) throw SwpsError(SWPS_E_STATE, "no shard: create a Cluster first");
    int32_t row = 0, pull = 0, push = 0;
    swps_check(swps_table_row_elems(t, &row, &pull, &push));
    push_(t, keys, cache, push, std::integral_constant<bool, detail::is_generic<PushCodec<Grad> >::value>());
  }

 private:
  static void push_(swps_table *t, const std::unordered_set<Key> &keys, param_cache_t &cache, int32_t push,
                    std::false_type) {
    typedef typename PullCodec<Val>::wire_t wire_t;
    std::vector<uint64_t> k;
    std::vector<wire_t> g;
    for (const auto &key : keys) {
      auto it = cache.grads().find(key);
      if (it == cache.grads().end()) continue;
      k.push_back((uint64_t)key);
      g.resize(k.size() * (size_t)push);
      PushCodec<Grad>::encode(it->second, &g[(k.size() - 1) * push]);
    }
    swps_check(swps_push_h(t, k.data(), k.size(), g.data()));  // n = 0 still joins a routed exchange
  }
  static void push_(swps_table *t, const std::unordered_set<Key> &keys, param_cache_t &cache, int32_t push,
                    std::true_type) {
    const int32_t layout = PullCodec<Val>::layout;
    const size_t es = detail::wire_bytes(layout), stride = (size_t)push * es;
    std::vector<uint64_t> k;
    BinaryBuffer bb;
    for (const auto &key : keys) {
      auto it = cache.grads().find(key);
      if (it == cache.grads().end()) continue;
      const size_t before = bb.size();
      bb << it->second;  // the app's own serialiser: the mean gradient (lr.cpp:32-38)
      detail::reset_grad(it->second);
      const size_t nb = bb.size() - before;
      if (nb == 0) continue;  // nothing to push for this key
      if (nb != stride)
        throw SwpsError(SWPS_E_UNSUPPORTED, "a gradient serialises to " + std::to_string(nb) +
                                                " bytes; the shard's push value is " + std::to_string(stride));
      k.push_back((uint64_t)key);
    }
    std::vector<char> blk(bb.size() + 1);
    if (layout == SWPS_LAYOUT_W2V)
      detail::deinterleave(bb.buffer(), &blk[0], k.size(), push / 2, es);
    else if (bb.size())
      std::memcpy(&blk[0], bb.buffer(), bb.size());
    swps_check(swps_push_h(t, k.data(), k.size(), &blk[0]));  // n = 0 still joins a routed exchange
  }
  swps_table *_t;
};

template <class Key, class Val, class Grad> GlobalPullAccess<Key, Val, Grad> &global_pull_access() {
  static GlobalPullAccess<Key, Val, Grad> a;
  return a;
}
template <class Key, class Val, class Grad> GlobalPushAccess<Key, Val, Grad> &global_push_access() {
  static GlobalPushAccess<Key, Val, Grad> a;
  return a;
}

/* ---- cluster/cluster.h ----------------------------------------------------
 * One process per GPU.  Rank / world / device from the launcher's
 * environment (torchrun: RANK, WORLD_SIZE, LOCAL_RANK; mpirun:
 * OMPI_COMM_WORLD_RANK / _SIZE / _LOCAL_RANK) instead of MPI_Comm_rank.
 * With world > 1 (or SWPS_ROUTE=1) the shard is key-sharded over a
 * communicator (swps_table_route): RCCL over xGMI, its unique id
 * bootstrapped over TCP at MASTER_ADDR:SWPS_BOOTSTRAP_PORT (default
 * MASTER_PORT + 1), or SWPS_TRANSPORT=tcp for the library's TCP star
 * (several ranks on one GPU).  frag_num = [server] frag_num (the
 * reference's hash-frag size; 1000 when absent).  The shard's shape:
 * [word2vec] len_vec (W2V layout) and [server] initial_learning_rate. */
struct W2VServer {
  static int32_t layout() { return SWPS_LAYOUT_W2V; }
  static int32_t init_mode() { return SWPS_INIT_HASH; }
  static uint64_t init_seed() { return 0; }
  static int32_t push_rule() { return SWPS_PUSH_ADAGRAD; }
};
struct LRServer {
  static int32_t layout() { return SWPS_LAYOUT_LR; }
  static int32_t init_mode() { return SWPS_INIT_HASH; }
  static uint64_t init_seed() { return 0; }
  static int32_t push_rule() { return SWPS_PUSH_ADAGRAD; }
};
struct ClusterWorker {};

inline int env_int(const char *a, const char *b, int dflt) {
  const char *v = std::getenv(a);
  if (!v && b) v = std::getenv(b);
  return v ? std::atoi(v) : dflt;
}

template <class WorkerT, class ServerT, class KeyT> class Cluster {
 public:
  /* capacity: keys this rank's shard holds (SWPS_CAPACITY overrides the default) */
  explicit Cluster(uint64_t capacity = 0, int32_t dtype = SWPS_F32) {
    if (!capacity) capacity = (uint64_t)env_int("SWPS_CAPACITY", nullptr, 1 << 22);
    _rank = env_int("RANK", "OMPI_COMM_WORLD_RANK", 0);
    _world = env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", 1);
    const int dev = env_int("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", 0);
    swps_table_cfg c;
    c.device = dev;
    c.layout = ServerT::layout();
    c.dtype = dtype;
    c.dim = c.layout == SWPS_LAYOUT_W2V ? global_config().get("word2vec", "len_vec").to_int32() : 1;
    c.capacity = capacity;
    c.learning_rate = global_config().get("server", "initial_learning_rate").to_float();
    c.fudge = 1e-6f;
    c.init_mode = ServerT::init_mode();
    c.seed = ServerT::init_seed();
    c.push_rule = ServerT::push_rule();
    swps_check(swps_table_create(&c, &_t));
    global_swps_table() = _t;
    global_swps_cfg() = c;
    global_node() = std::make_pair(_rank + 1, _world);
    global_frag_num() = global_config().has("server", "frag_num") ? global_config().get("server", "frag_num").to_int32()
                                                                  : 1000;
    if (_world > 1 || env_int("SWPS_ROUTE", nullptr, 0)) {
      const char *addr = std::getenv("MASTER_ADDR");
      const int port = env_int("SWPS_BOOTSTRAP_PORT", nullptr, env_int("MASTER_PORT", nullptr, 29500) + 1);
      const int timeout = env_int("SWPS_BOOTSTRAP_TIMEOUT_MS", nullptr, 120000);
      const char *tr = std::getenv("SWPS_TRANSPORT");
      if (tr && std::string(tr) == "tcp") {
        swps_check(swps_comm_create_tcp(addr ? addr : "127.0.0.1", port, _rank, _world, dev, timeout, &_comm));
      } else {
        std::vector<uint8_t> id(SWPS_COMM_ID_BYTES);
        swps_check(swps_comm_bootstrap_tcp(addr ? addr : "127.0.0.1", port, _rank, _world, timeout, id.data()));
        swps_check(swps_comm_create_rccl(id.data(), _rank, _world, dev, &_comm));
      }
      // SWPS_COMM_IPC=1: the exchanges' payloads device to device through IPC-mapped peer
      // inboxes (swps_comm_enable_ipc; the ranks of one node)
      if (_world > 1 && env_int("SWPS_COMM_IPC", nullptr, 0)) swps_check(swps_comm_enable_ipc(_comm, 0));
      swps_check(swps_table_route(_t, _comm, global_frag_num()));
      global_swps_comm() = _comm;
    }
  }
  ~Cluster() {
    if (global_swps_table() == _t) global_swps_table() = nullptr;
    if (global_swps_comm() == _comm) global_swps_comm() = nullptr;
    swps_table_destroy(_t);
    swps_comm_destroy(_comm);
  }
  /* the reference's initialize binds its transfer's listeners to random ports: one rand() per
   * bind, two binds (common.h:92-96 via Listener.h:83) — the process's rand() stream moves by 2
   * before an app draws, as SWPS_W2V_INIT_REF's rand_offset = 2 assumes */
  void initialize() {
    (void)process_rand()();
    (void)process_rand()();
  }
  /* The worker is done: keep serving the other ranks until all are
   * (swps_finish), then SparseTable::output (sparsetable.h:127-132) of this
   * rank's shard to exactly `path` (cluster.h:41-50; the reference's mains
   * make it per rank themselves, w2v.cpp:54-56). */
  void finalize(const std::string &path = "") {
    swps_check(swps_finish(_t));
    if (path.empty()) return;
    swps_check(swps_dump(_t, path.c_str()));
  }
  swps_table *table() { return _t; }
  int rank() const { return _rank; }
  int world() const { return _world; }
  bool routed() const { return _comm != nullptr; }

 private:
  Cluster(const Cluster &);
  Cluster &operator=(const Cluster &);
  swps_table *_t = nullptr;
  swps_comm *_comm = nullptr;
  int _rank = 0, _world = 1;
};

/* server.h:49-62: every "key param" record of the dump whose BasicHashFrag
 * node is this rank's is assigned to the shard (the others are skipped). */
template <typename Key, typename Param, typename PullVal, typename Grad, typename PullM, typename PushM>
void ClusterServer<Key, Param, PullVal, Grad, PullM, PushM>::load(const std::string &path) {
  swps_table *t = global_swps_table();
  if (!t) throw SwpsError(SWPS_E_STATE, "no shard: create a Cluster first");
  // server.h:49-62 constructs one `param_t param;` before reading the dump: word2vec's WParam
  // draws h then v from libc rand() (word2vec.h:36-44, Vec::randInit) — the process's rand()
  // stream moves by 2·D as the reference's did (LRParam draws nothing)
  if (layout() == SWPS_LAYOUT_W2V) {
    int32_t row = 0;
    swps_check(swps_table_row_elems(t, &row, nullptr, nullptr));
    for (int32_t i = 0; i < row / 2; i++) (void)process_rand()();
  }
  swps_check(swps_load(t, path.c_str(), global_frag_num(), global_node().second, global_node().first));
}
template <class ServerT> ServerT &global_server() {
  static ServerT s;
  return s;
}

/* ---- app level ------------------------------------------------------------ */

/* Word2Vec<MiniBatch> (word2vec_global.h:541-748, w2v.cpp): train() = the
 * first full pull + niters epochs of the minibatch loop, all on the GPU.
 * local = true: word2vec.h's Word2Vec<MiniBatch> (w2v_local.cpp) — atoi keys,
 * per-minibatch vocab and unigram table.  On a multi-rank Cluster each rank
 * trains its own corpus file and the library runs the key-sharded exchange
 * (swps_w2v_shard_comm; the owners initialise keys, SWPS_INIT_HASH). */
class Word2VecApp {
 public:
  Word2VecApp(const std::string &path, int niters, swps_table *t = nullptr, int fp64_intermediates = 1,
              bool local = false)
      : _path(path), _niters(niters) {
    swps_w2v_cfg c;
    c.window = global_config().get("word2vec", "window").to_int32();
    c.negative = global_config().get("word2vec", "negative").to_int32();
    c.min_sentence_length = global_config().get("word2vec", "min_sentence_length").to_int32();
    c.minibatch = global_config().get("worker", "minibatch").to_int32();
    c.sample = global_config().get("word2vec", "sample").to_float();
    c.alpha = global_config().get("word2vec", "learning_rate").to_float();
    c.unigram_size = 100000000ULL;
    c.key_mode = local ? SWPS_KEY_ATOI : SWPS_KEY_BKDR;
    c.init_mode = SWPS_W2V_INIT_REF;
    c.rand_seed = 1;
    c.rand_offset = 2;
    c.fp64_intermediates = fp64_intermediates;
    c.profile = 0;
    c.minibatch_vocab = local ? 1 : 0;
    c.sampler = SWPS_SAMPLER_TABLE;
    c.host_ingest = 0;
    _comm = t ? nullptr : global_swps_comm();
    if (_comm) c.init_mode = SWPS_W2V_INIT_TABLE;
    swps_check(swps_w2v_create(t ? t : global_swps_table(), &c, &_w));
  }
  ~Word2VecApp() { swps_w2v_destroy(_w); }
  void train() {
    swps_check(swps_w2v_load_text(_w, _path.c_str()));
    if (_comm) swps_check(swps_w2v_shard_comm(_w, _comm, global_frag_num()));
    swps_check(swps_w2v_init(_w));
    swps_check(swps_w2v_train_epochs(_w, _niters));
  }
  swps_w2v *handle() { return _w; }

 private:
  Word2VecApp(const Word2VecApp &);
  Word2VecApp &operator=(const Word2VecApp &);
  std::string _path;
  int _niters;
  swps_w2v *_w = nullptr;
  swps_comm *_comm = nullptr;
};

/* Sent2Vec (sent2vec.cpp:14-195): load_word_vector then train(); the
 * sentence vectors go to `out_path` in the reference's format.  On a
 * multi-rank Cluster: replicas — every rank loads the whole (read-only) word
 * table into a local copy and trains the documents BasicHashFrag gives it
 * (swps_s2v_shard); its sentence vectors go to exactly `out_path`, as the
 * reference's Sent2Vec writes them (sent2vec.cpp:24,46). */
class Sent2VecApp {
 public:
  Sent2VecApp(const std::string &path, const std::string &out_path, int niters, swps_table *t = nullptr)
      : _path(path), _out(out_path), _t(t ? t : global_swps_table()) {
    _comm = t ? nullptr : global_swps_comm();
    if (_comm) {  // a local replica of the word table
      swps_table_cfg c = global_swps_cfg();
      swps_check(swps_table_create(&c, &_own));
      _t = _own;
      swps_check(swps_comm_info(_comm, &_rank, &_world));
    }
    _c.window = global_config().get("word2vec", "window").to_int32();
    _c.negative = global_config().get("word2vec", "negative").to_int32();
    _c.min_sentence_length = global_config().get("word2vec", "min_sentence_length").to_int32();
    _c.minibatch = global_config().get("worker", "minibatch").to_int32();
    _c.niters = niters;
    _c.alpha = global_config().get("word2vec", "learning_rate").to_float();
    _c.unigram_size = 100000000ULL;
    _c.rand_seed = 1;
    _c.rand_offset = 2;
    _c.rand_insert_extra = 0;
    _c.profile = 0;
  }
  ~Sent2VecApp() {
    if (_s) swps_s2v_destroy(_s);
    if (_own) swps_table_destroy(_own);
  }
  /* ClusterServer::load (server.h:49-62) + the WParam it constructs first */
  void load_word_vector(const std::string &path) {
    uint64_t before = 0, after = 0;
    swps_check(swps_table_size(_t, &before));
    swps_check(swps_load(_t, path.c_str(), 1000, 1, 0));
    swps_check(swps_table_size(_t, &after));
    int32_t row = 0;
    swps_check(swps_table_row_elems(_t, &row, nullptr, nullptr));
    _c.rand_offset += (uint64_t)row / 2 + _c.rand_insert_extra * (after - before);
  }
  void train() {
    swps_check(swps_s2v_create(_t, &_c, &_s));
    if (_comm) swps_check(swps_s2v_shard(_s, _rank, _world, global_frag_num()));
    swps_check(swps_s2v_load_text(_s, _path.c_str()));
    swps_check(swps_s2v_train(_s));
    if (!_out.empty()) swps_check(swps_s2v_dump(_s, _out.c_str()));
  }
  swps_s2v *handle() { return _s; }

 private:
  Sent2VecApp(const Sent2VecApp &);
  Sent2VecApp &operator=(const Sent2VecApp &);
  std::string _path, _out;
  swps_table *_t;
  swps_s2v_cfg _c;
  swps_s2v *_s = nullptr;
  swps_comm *_comm = nullptr;
  swps_table *_own = nullptr;
  int32_t _rank = 0, _world = 1;
};

/* LR (lr.cpp:133-411): train(niters) returns the per-epoch mean squared
 * error the reference logs (lr.cpp:231); predict() the probabilities.  As in
 * the reference the first pull happens at the first train / predict, so a
 * load_param (lr.cpp:297-300: ClusterServer::load of a dump) before it leaves
 * the loaded keys as they are and initialises only the others (gen_float in
 * first-pull order, lr.cpp:48-50) — the predict mode of lr.cpp:498-504.  On
 * a multi-rank Cluster the library runs the key-sharded exchange
 * (swps_lr_shard_comm): train / predict are collective, errors are this
 * rank's rows'. */
class LRApp {
 public:
  LRApp(const std::string &path, swps_table *t = nullptr) : _t(t ? t : global_swps_table()) {
    swps_comm *comm = t ? nullptr : global_swps_comm();
    swps_lr_cfg c;
    c.minibatch = global_config().get("worker", "minibatch").to_int32();
    c.init_ref = comm ? 0 : 1;
    c.profile = 0;
    c.fast_sums = 0;
    c.plan = SWPS_LR_PLAN_STEP;
    swps_check(swps_lr_create(_t, &c, &_l));
    swps_check(swps_lr_load_text(_l, path.c_str()));
    if (comm) swps_check(swps_lr_shard_comm(_l, comm, global_frag_num()));
  }
  ~LRApp() { swps_lr_destroy(_l); }
  /* lr.cpp:297-300: the dump's keys this rank owns (server.h:49-62) */
  void load_param(const std::string &path) {
    if (_inited) throw SwpsError(SWPS_E_STATE, "load_param after the first pull");
    swps_check(swps_load(_t, path.c_str(), global_frag_num(), global_node().second, global_node().first));
  }
  std::vector<double> train(int niters) {
    init();
    std::vector<double> err((size_t)niters);
    swps_check(swps_lr_train(_l, niters, err.data()));
    return err;
  }
  std::vector<float> predict() {
    init();
    uint64_t info[4];
    swps_check(swps_lr_info(_l, info));
    std::vector<float> p(info[0] ? info[0] : 1);
    swps_check(swps_lr_predict(_l, p.data(), nullptr, p.size()));
    p.resize(info[0]);
    return p;
  }
  /* lr.cpp:240-295: one probability per line (`outfile << predict <<
   * std::endl`, ostream precision 6).  Like the reference (it reads _path,
   * lr.cpp:247) the rows are the context's own data; `dataset` is unused. */
  void predict(const std::string &dataset, const std::string &out) {
    (void)dataset;
    const std::vector<float> p = predict();
    std::ofstream f(out.c_str());
    if (!f) throw SwpsError(SWPS_E_IO, "cannot open " + out);
    for (float x : p) f << x << std::endl;
  }

 private:
  void init() {
    if (!_inited) swps_check(swps_lr_init(_l));
    _inited = true;
  }
  LRApp(const LRApp &);
  LRApp &operator=(const LRApp &);
  swps_table *_t;
  swps_lr *_l = nullptr;
  bool _inited = false;
};

}  // namespace swift_snails

#endif /* SWIFTMPI_COMPAT_H_ */
