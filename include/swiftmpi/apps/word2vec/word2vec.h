/* apps/word2vec/word2vec.h under its reference name: the local variant (atoi keys, each minibatch
 * its own vocabulary and unigram table, word2vec.h:281-629).  Two users:
 *   w2v_local.cpp — Word2Vec<MiniBatch>(path, niters).train(): the library's device loop
 *                   (word2vec_app.h, swps_w2v_cfg.minibatch_vocab = 1);
 *   sent2vec.cpp  — derives WordMiniBatch from MiniBatch and trains its sentence vectors on the
 *                   host with the reference's own learn_instance; MiniBatch below is the
 *                   reference's host worker (gather_keys / pull / table / param / clear) over the
 *                   PS API (GlobalPullAccess -> swps_pull_h on the HBM shard).
 * Restated here (paths relative to logicxin/SwiftMPI src/apps/word2vec/word2vec.h):
 *   EXP_TABLE_SIZE, MAX_EXP, table_size   :6-8
 *   Instance, hash_fn, hash_fn2           :192-209
 *   parse_instance                        :210-225 (atoi keys, min_sentence_length)
 *   global_channel                        :232-236
 *   ExpTable / exptable                   :238-266
 *   MiniBatch                             :277-440
 *   Error                                 :442-457 */
#ifndef SWIFTMPI_WORD2VEC_LOCAL_H_
#define SWIFTMPI_WORD2VEC_LOCAL_H_
#include "swiftmpi/apps/word2vec/word2vec_app.h"

#define EXP_TABLE_SIZE 1000
#define MAX_EXP 6
const int table_size = 1e8;

struct Instance {
  std::vector<w2v_key_t> words;
  void clear() { words.clear(); }
};

inline w2v_key_t hash_fn(const char *key) noexcept { return BKDRHash<w2v_key_t>(key); }
inline w2v_key_t hash_fn2(const char *key) noexcept { return std::atoi(key); }

/* a line's words as atoi keys; valid when it has at least [word2vec] min_sentence_length words */
inline bool parse_instance(const std::string &line, Instance &ins) noexcept {
  ins.clear();
  static int min_length = 0;
  if (min_length == 0) min_length = global_config().get("word2vec", "min_sentence_length").to_int32();
  for (const auto &word : split(line, " ")) ins.words.push_back(hash_fn2(word.c_str()));
  return (int)ins.words.size() >= min_length;
}

inline std::shared_ptr<AsynExec::channel_t> &global_channel() {
  static AsynExec async(global_config().get("worker", "nthreads").to_int32());
  static std::shared_ptr<AsynExec::channel_t> channel = async.open();
  return channel;
}

/* sigmoid lookup: e / (e + 1) with e = exp((i / 1000 * 2 - 1) * 6) in float, the argument's
 * exp in double (the overload the reference resolves), index (f + 6) * 83 */
class ExpTable {
 public:
  typedef float real_t;
  ExpTable() : _t(EXP_TABLE_SIZE + 1, 0.f) {
    for (int i = 0; i < EXP_TABLE_SIZE; i++) {
      _t[i] = exp((i / (real_t)EXP_TABLE_SIZE * 2 - 1) * MAX_EXP);
      _t[i] = _t[i] / (_t[i] + 1);
    }
  }
  real_t operator()(real_t f) const noexcept { return _t[(int)((f + MAX_EXP) * (EXP_TABLE_SIZE / MAX_EXP / 2))]; }

 private:
  std::vector<real_t> _t;
};
static ExpTable exptable;

struct Error {
  float data = 0;
  size_t counter = 0;
  void accu(float e) noexcept {
    data += e;
    counter++;
  }
  float norm() noexcept {
    const float error = data / counter;
    data = 0;
    counter = 0;
    return error;
  }
};

/* the minibatch's unigram^0.75 table (word2vec.h:398-425) in run-length form: word i of the
 * std::map-ordered vocabulary owns slots [start[i], start[i+1]) of the table_size-slot walk
 * (swps_unigram_starts: the literal loop's boundaries, bit for bit); t[a] finds a's word */
class UnigramTable {
 public:
  void build(const std::map<w2v_key_t, int> &freq) {
    _ids.clear();
    std::vector<uint64_t> keys;
    std::vector<int32_t> counts;
    for (const auto &kv : freq) {
      _ids.push_back(kv.first);
      keys.push_back((uint64_t)kv.first);
      counts.push_back(kv.second);
    }
    _start.assign(_ids.size() + 1, 0);
    if (!_ids.empty())
      swps_check(swps_unigram_starts(keys.data(), counts.data(), _ids.size(), (uint64_t)table_size, _start.data()));
  }
  w2v_key_t operator[](size_t a) const {
    const size_t i = (size_t)(std::upper_bound(_start.begin(), _start.end(), (uint64_t)a) - _start.begin());
    return _ids[std::min(i ? i - 1 : 0, _ids.size() - 1)];
  }

 private:
  std::vector<w2v_key_t> _ids;
  std::vector<uint64_t> _start;
};

/* The reference's host minibatch worker: negative sampling within a minibatch.
 *   gather_keys(file, line_id, B)  the next B + 1 valid lines' words: counts in a std::map and the
 *                                  `_local_keys` set (first occurrence), file position restored
 *   pull()                         init_keys + pull_with_barrier of `_local_keys`, then the
 *                                  minibatch's unigram table
 *   push()                         push_with_barrier of the accumulated gradients, then clear()
 * One rank is worker and server of its own shard (the reference runs both in the process): the
 * server's pull handler constructs a WParam — h then v, Vec::randInit: 2·D rand() — for every
 * requested key (accessmethod.h:63-70, server.h:143-150) and inserts it for a key its table
 * lacks, so pull() moves the process's rand() stream by 2·D per pulled key, in request order, and
 * gives a key new to the shard those draws (swps_table_find_h / swps_assign_h).  Multi-rank
 * (routed) shards initialise new keys on their owners (SWPS_INIT_HASH) instead.  Single-threaded
 * (the reference's nthreads = 1, its only deterministic setting). */
class MiniBatch {
 public:
  typedef LocalParamCache<w2v_key_t, WLocalParam, WLocalGrad> param_cache_t;
  MiniBatch()
      : _minibatch(global_config().get("worker", "minibatch").to_int32()),
        _nthreads(global_config().get("worker", "nthreads").to_int32()),
        _pull_access(global_pull_access<w2v_key_t, WLocalParam, WLocalGrad>()),
        _push_access(global_push_access<w2v_key_t, WLocalParam, WLocalGrad>()) {
    CHECK_GT(_minibatch, 0);
    CHECK_GT(_nthreads, 0);
  }
  virtual ~MiniBatch() {}

  void pull() {
    _param_cache.init_keys(_local_keys);
    server_side_params();
    _pull_access.pull_with_barrier(_local_keys, _param_cache);
    gen_unigram_table();
  }
  void push() {
    _push_access.push_with_barrier(_local_keys, _param_cache);
    clear();
  }
  size_t gather_keys(FILE *file, int &line_id, int minibatch = 0) {
    const long cur_pos = ftell(file);
    int line_count = 0;
    line_id = 0;
    _local_keys.clear();
    LineFileReader line_reader;
    Instance ins;
    while (!feof(file)) {
      char *cline = line_reader.getline(file);
      if (!cline) continue;
      if (!parse_instance(std::string(cline), ins)) continue;
      for (const auto &item : ins.words) {
        _num_words++;  // never reset (word2vec.h:385-392, 624)
        auto it = _word_freq.find(item);
        if (it != _word_freq.end()) {
          it->second++;
        } else {
          _word_freq[item] = 1;
          _local_keys.insert(item);
        }
      }
      line_count++;
      line_id++;
      if (minibatch > 0 && line_count > minibatch) break;
    }
    RAW_LOG(INFO, "collect %lu keys", (unsigned long)_local_keys.size());
    fseek(file, cur_pos, SEEK_SET);
    return _local_keys.size();
  }
  param_cache_t &param() noexcept { return _param_cache; }
  const std::map<w2v_key_t, int> &word_freq() noexcept { return _word_freq; }
  const UnigramTable &table() noexcept { return _table; }
  virtual void clear() noexcept {
    _local_keys.clear();
    _word_freq.clear();
    _param_cache.clear();
  }
  size_t num_words() noexcept { return _num_words; }

 protected:
  void gen_unigram_table() {
    CHECK_GT(_word_freq.size(), 0) << "word_freq should be inited before";
    _table.build(_word_freq);
  }
  void server_side_params() {
    swps_table *t = global_swps_table();
    if (!t || global_swps_comm()) return;
    std::vector<uint64_t> keys;
    keys.reserve(_local_keys.size());
    for (const auto &k : _local_keys) keys.push_back((uint64_t)k);
    std::vector<uint8_t> present(keys.size() + 1, 0);
    swps_check(swps_table_find_h(t, keys.data(), keys.size(), present.data()));
    int32_t row = 0;
    swps_check(swps_table_row_elems(t, &row, nullptr, nullptr));
    const int D = len_vec();
    std::vector<uint64_t> miss;
    std::vector<double> rows;
    Vec h(D), v(D);
    for (size_t i = 0; i < keys.size(); i++) {
      h.random();
      v.random();
      if (present[i]) continue;
      miss.push_back(keys[i]);
      const size_t o = rows.size();
      rows.resize(o + (size_t)row, 0.0);  // [h | v | h2sum = 0 | v2sum = 0]
      for (int e = 0; e < D; e++) {
        rows[o + e] = h[e];
        rows[o + D + e] = v[e];
      }
    }
    swps_check(swps_assign_h(t, miss.data(), miss.size(), rows.data()));
  }

  std::unordered_set<w2v_key_t> _local_keys;
  std::map<w2v_key_t, int> _word_freq;
  int _minibatch = 0;
  int _nthreads = 0;
  pull_access_t &_pull_access;
  push_access_t &_push_access;
  param_cache_t _param_cache;
  size_t _num_words = 0;
  UnigramTable _table;
};

template <typename MiniBatchT> using Word2Vec = swift_snails::Word2VecT<MiniBatchT, true>;
#endif
