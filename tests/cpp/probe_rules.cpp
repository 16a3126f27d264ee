// Host-body rule recognition (swiftmpi_compat.h detail::RuleProbe): access
// methods in the reference's shape that declare nothing, their bodies run on
// probe values and matched to a device rule.  Prints "<case> init=<m> push=<r>"
// or "<case> error <code>".  Used by tests/test_compat.py (CPU: no GPU call).
#include <cmath>
#include <cstdio>

#include "swiftmpi_compat.h"

using namespace swift_snails;

struct Row {
  float w = 0, acc = 0;
};
struct Delta {
  float sum = 0;
  int n = 0;
};
BinaryBuffer &operator<<(BinaryBuffer &bb, Delta &d) {
  if (d.n) bb << float(d.sum / d.n);
  return bb;
}
BinaryBuffer &operator>>(BinaryBuffer &bb, Delta &d) {
  bb >> d.sum;
  d.n = 1;
  return bb;
}

template <bool Draw> class InitM : public PullAccessMethod<unsigned, Row, float> {
 public:
  void init_param(const unsigned &, Row &r) { r.w = Draw ? global_random().gen_float() : 0.f; }
  void get_pull_value(const unsigned &, const Row &r, float &v) { v = r.w; }
};
class HalfInit : public PullAccessMethod<unsigned, Row, float> {
 public:
  void init_param(const unsigned &, Row &r) { r.w = 0.5f; }
  void get_pull_value(const unsigned &, const Row &r, float &v) { v = r.w; }
};
class AdaM : public PushAccessMethod<unsigned, Row, Delta> {
 public:
  AdaM() : lr(global_config().get("server", "initial_learning_rate").to_float()) {}
  void apply_push_value(const unsigned &, Row &r, const Delta &d) {
    r.acc += d.sum * d.sum;
    r.w += lr * d.sum / float(std::sqrt(r.acc + 1e-6f));
  }
  float lr;
};
class SgdM : public PushAccessMethod<unsigned, Row, Delta> {
 public:
  void apply_push_value(const unsigned &, Row &r, const Delta &d) {
    r.w += global_config().get("server", "initial_learning_rate").to_float() * d.sum;
  }
};
class MomentumM : public PushAccessMethod<unsigned, Row, Delta> {  // no device rule
 public:
  void apply_push_value(const unsigned &, Row &r, const Delta &d) {
    r.acc = 0.9f * r.acc + d.sum;
    r.w += 0.1f * r.acc;
  }
};

template <class PullM, class PushM> static void show(const char *name) {
  typedef ClusterServer<unsigned, Row, float, Delta, PullM, PushM> s_t;
  const float before = Random(global_random()).gen_float();
  try {
    const int m = s_t::init_mode(), r = s_t::push_rule();
    std::printf("%s init=%d push=%d seed_ok=%d\n", name, m, r,
                (int)(Random(global_random()).gen_float() == before));  // probing draws nothing
  } catch (SwpsError &e) {
    std::printf("%s error %d\n", name, e.code);
  }
}

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  global_config().load_conf(argv[1]);
  global_config().parse();
  show<InitM<true>, AdaM>("flcg_adagrad");
  show<InitM<false>, SgdM>("zero_sgd");
  show<HalfInit, AdaM>("half_adagrad");
  show<InitM<true>, MomentumM>("flcg_momentum");
  return 0;
}
