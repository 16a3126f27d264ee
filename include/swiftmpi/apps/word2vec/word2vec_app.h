/*
 * The word2vec app types of apps/word2vec/word2vec_global.h (and word2vec.h,
 * the local-vocabulary variant) under their reference names, over
 * libswps.so: an unchanged w2v.cpp / w2v_local.cpp compiles against them
 * (swiftmpi/swiftmpi.h explains the include order).
 *
 *   w2v_key_t, WLocalParam, WLocalGrad, WParam      word2vec_global.h:30-156
 *   WPullAccessMethod / WPushAccessMethod           :158-191 (the device's hashed init and AdaGrad)
 *   server_t, pull_access_t, push_access_t          :229-232
 *   MiniBatch                                       :284-515 (the minibatch loop runs on the GPU)
 *   Word2Vec<MiniBatch>(path, niters).train()       :534-748 (Word2VecApp)
 *
 * Precision of the device loop: [gpu] intermediates = parity (fp64 neu1 /
 * neu1e and sums, the default: the reference's arithmetic within 1e-5),
 * bfp32, bfp40 or fast; the shard is fp32.
 */
#ifndef SWIFTMPI_WORD2VEC_APP_H_
#define SWIFTMPI_WORD2VEC_APP_H_

#include <functional>

#include "swiftmpi/swiftmpi.h"

using namespace swift_snails;

typedef size_t w2v_key_t;

inline int len_vec() {
  static int d = 0;
  if (d == 0) {
    d = global_config().get("word2vec", "len_vec").to_int32();
    CHECK_GT(d, 0);
  }
  return d;
}

/* the server-side row [h | v | h2sum | v2sum] lives in the HBM shard */
struct WParam {};

/* PS-level values, as the reference's GlobalPullAccess / GlobalPushAccess carry them
 * (word2vec.h:50-100: zero-initialised Vecs) */
struct WLocalParam {
  Vec h, v;
  WLocalParam() : h(len_vec()), v(len_vec()) {}
};
struct WLocalGrad {
  Vec h_grad, v_grad;
  int h_count = 0, v_count = 0;
  WLocalGrad() : h_grad(len_vec()), v_grad(len_vec()) {}
  void accu_h(const Vec &g) {
    h_count++;
    h_grad += g;
  }
  void accu_v(const Vec &g) {
    v_count++;
    v_grad += g;
  }
  void reset() { *this = WLocalGrad(); }
};
namespace swift_snails {
template <> struct PullCodec<WLocalParam> {
  typedef double wire_t;
  static const int32_t layout = SWPS_LAYOUT_W2V;
  static int elems() { return 2 * len_vec(); }
  static void decode(const double *w, WLocalParam &p) {
    const int D = len_vec();
    p.h.init(D);
    p.v.init(D);
    for (int i = 0; i < D; i++) {
      p.h[i] = w[i];
      p.v[i] = w[D + i];
    }
  }
};
template <> struct PushCodec<WLocalGrad> {  // the mean gradient, word2vec_global.h:122-134
  static void encode(WLocalGrad &g, double *w) {
    const int D = len_vec();
    for (int i = 0; i < D; i++) {
      w[i] = g.h_count > 0 ? g.h_grad[i] / g.h_count : g.h_grad[i];
      w[D + i] = g.v_count > 0 ? g.v_grad[i] / g.v_count : g.v_grad[i];
    }
    g.reset();
  }
};
}  // namespace swift_snails

class WPullAccessMethod : public PullAccessMethod<w2v_key_t, WParam, WLocalParam> {
 public:
  static const int32_t init_mode = SWPS_INIT_HASH;
};
class WPushAccessMethod : public PushAccessMethod<w2v_key_t, WParam, WLocalGrad> {
 public:
  static const int32_t push_rule = SWPS_PUSH_ADAGRAD;  // word2vec_global.h:176-185
};
typedef ClusterServer<w2v_key_t, WParam, WLocalParam, WLocalGrad, WPullAccessMethod, WPushAccessMethod> server_t;
typedef GlobalPullAccess<w2v_key_t, WLocalParam, WLocalGrad> pull_access_t;
typedef GlobalPushAccess<w2v_key_t, WLocalParam, WLocalGrad> push_access_t;

namespace swift_snails {
inline int w2v_intermediates() {
  if (!global_config().has("gpu", "intermediates")) return 1;
  const std::string m = global_config().get("gpu", "intermediates").to_string();
  if (m == "parity") return 1;
  if (m == "fast") return 0;
  if (m == "bfp40") return SWPS_INTER_BFP40;
  if (m == "bfp32") return SWPS_INTER_BFP32;
  throw SwpsError(SWPS_E_CFG, "[gpu] intermediates: parity, bfp32, bfp40 or fast, not " + m);
}

/* Word2Vec<MiniBatch>: the first full pull and `niters` epochs on the GPU of this rank's shard;
 * on a multi-rank Cluster the library runs the key-sharded exchange (Word2VecApp) */
template <typename MiniBatchT, bool Local> class Word2VecT {
 public:
  Word2VecT(const std::string &path, int niters) : _app(path, niters, nullptr, w2v_intermediates(), Local) {}
  void train() { _app.train(); }
  swps_w2v *handle() { return _app.handle(); }

 private:
  Word2VecApp _app;
};
}  // namespace swift_snails

#endif /* SWIFTMPI_WORD2VEC_APP_H_ */
