/*
 * swiftmpi/swiftmpi.h — what an UNCHANGED reference app sees when it
 * includes "../../swiftmpi.h" (src/swiftmpi.h): the parameter-server API of
 * swiftmpi_compat.h (over libswps.so) plus the reference utilities its mains
 * and app classes call.  Compile a reference app against this tree instead
 * of its own:
 *
 *   g++ -std=c++11 -I- -I<repo>/include -I<repo>/include/swiftmpi/apps/word2vec \
 *       <ref>/src/apps/logistic/lr.cpp -L<repo>/swiftmpi_amd/lib -lswps -pthread
 *
 * (-I- stops the compiler from taking the reference's own headers next to
 * the source file; the second -I resolves the apps' "../../swiftmpi.h" and
 * "word2vec_global.h" / "word2vec.h" here.)
 *
 * Reference interfaces restated (paths relative to logicxin/SwiftMPI src/):
 *   GlobalMPI / global_mpi()       utils/mpi.h:7-55 (rank / size from the launcher's environment)
 *   fms::CMDLine                   utils/CMDLine.h:17-183
 *   format_string                  utils/string.h:69-89
 *   split / BKDRHash               utils/string.h:34-48, 130-137
 *   LineFileReader                 utils/string.h:91-121
 *   Vec                            utils/vec1.h:6-258
 *   AsynExec / async_exec          utils/AsynExec.h:17-123
 *   SpinLock                       utils/SpinLock.h
 *   LOG / DLOG / CHECK_* / RAW_LOG_*   glog, as utils/common.h pulls it in
 * Host-side plumbing only: no compute of the hot path lives here.
 */
#ifndef SWIFTMPI_SWIFTMPI_H_
#define SWIFTMPI_SWIFTMPI_H_

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <functional>
#include <iostream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "swiftmpi_compat.h"

namespace swift_snails {

/* ---- glog's LOG / CHECK, as the apps use them ------------------------------ */
namespace detail {
class LogLine {
 public:
  LogLine(const char *sev, bool fatal = false) : _sev(sev), _fatal(fatal) {}
  ~LogLine() {
    std::cerr << _sev << " " << _os.str() << std::endl;
    if (_fatal) std::abort();  // glog's CHECK failure aborts
  }
  template <class T> LogLine &operator<<(const T &x) {
    _os << x;
    return *this;
  }
  LogLine &operator<<(std::ostream &(*f)(std::ostream &)) {
    _os << f;
    return *this;
  }

 private:
  std::ostringstream _os;
  const char *_sev;
  bool _fatal;
};
inline void raw_log(const char *sev, const char *fmt, ...) {
  std::va_list ap;
  va_start(ap, fmt);
  std::fprintf(stderr, "%s ", sev);
  std::vfprintf(stderr, fmt, ap);
  std::fputc('\n', stderr);
  va_end(ap);
}
}  // namespace detail

#ifndef LOG
#define LOG(sev) ::swift_snails::detail::LogLine(#sev)
#define DLOG(sev) ::swift_snails::detail::LogLine(#sev)
#define CHECK(c) \
  if (c) {       \
  } else         \
    ::swift_snails::detail::LogLine("FATAL check failed: " #c, true)
#define CHECK_EQ(a, b) CHECK((a) == (b))
#define CHECK_NE(a, b) CHECK((a) != (b))
#define CHECK_GT(a, b) CHECK((a) > (b))
#define CHECK_GE(a, b) CHECK((a) >= (b))
#define CHECK_LT(a, b) CHECK((a) < (b))
#define CHECK_LE(a, b) CHECK((a) <= (b))
#endif
#define RAW_LOG(sev, ...) ::swift_snails::detail::raw_log(#sev, __VA_ARGS__)
#define RAW_DLOG(sev, ...) ::swift_snails::detail::raw_log(#sev, __VA_ARGS__)
#define RAW_LOG_INFO(...) ::swift_snails::detail::raw_log("INFO", __VA_ARGS__)
#define RAW_LOG_WARNING(...) ::swift_snails::detail::raw_log("WARNING", __VA_ARGS__)
#define RAW_LOG_ERROR(...) ::swift_snails::detail::raw_log("ERROR", __VA_ARGS__)

/* ---- utils/mpi.h: one process per GPU, rank / size from the launcher -------- */
class GlobalMPI {
 public:
  /* lr.cpp's main never loads its -config (lr.cpp:413-509 has no load_conf: the reference's
   * Cluster() then CHECK-fails on the empty config, cluster.h:11-13); the -config of the command
   * line is loaded here, before the app's own load_conf / parse (which finds the same keys again:
   * the first definition wins) */
  static void initialize(int argc, char **argv) {
    for (int i = 1; i + 1 < argc; i++)
      if (std::string(argv[i]) == "-config" || std::string(argv[i]) == "--config") {
        global_config().load_conf(argv[i + 1]);
        global_config().parse();
        break;
      }
  }
  int rank() const { return env_int("RANK", "OMPI_COMM_WORLD_RANK", 0); }
  int size() const { return env_int("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", 1); }
  /* a collective over the key-sharded shard (swps_barrier); one rank: its device work retired */
  void barrier() {
    if (global_swps_table()) swps_check(swps_barrier(global_swps_table()));
  }
};
inline GlobalMPI &global_mpi() {
  static GlobalMPI m;
  return m;
}

/* ---- utils/string.h ----------------------------------------------------------- */
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wformat-security"  // the apps pass runtime formats (lr.cpp:493)
#pragma GCC diagnostic ignored "-Wformat-nonliteral"
template <typename... ARGS> void format_string(std::string &s, const char *format, ARGS... args) {
  const int len = std::snprintf(NULL, 0, format, args...);
  CHECK(len >= 0);
  const size_t old = s.size();
  s.resize(old + len + 1);
  std::snprintf(&s[old], (size_t)len + 1, format, args...);
  s.resize(old + len);
}
template <typename... ARGS> std::string format_string(const char *format, ARGS... args) {
  std::string s;
  format_string(s, format, args...);
  return s;
}
#pragma GCC diagnostic pop

class LineFileReader {
 public:
  LineFileReader() {}
  explicit LineFileReader(FILE *f) : _file(f) {}
  ~LineFileReader() { std::free(_buffer); }
  char *getline() { return getline(_file); }
  char *getline(FILE *f) { return getdelim(f, '\n'); }
  char *getdelim(FILE *f, char delim) {
    ssize_t n = ::getdelim(&_buffer, &_cap, delim, f);
    if (n < 0) {
      _length = 0;
      return NULL;
    }
    if (n >= 1 && _buffer[n - 1] == delim) _buffer[--n] = 0;
    _length = (size_t)n;
    return _buffer;
  }
  char *get() { return _buffer; }
  size_t length() const { return _length; }

 private:
  LineFileReader(const LineFileReader &);
  LineFileReader &operator=(const LineFileReader &);
  char *_buffer = NULL;
  size_t _cap = 0, _length = 0;
  FILE *_file = nullptr;
};

/* split on any of `delim`'s characters, empty fields dropped (utils/string.h:34-48) */
inline std::vector<std::string> split(const std::string &s, const std::string &delim) {
  std::vector<std::string> cols;
  size_t at = s.find_first_not_of(delim);
  while (at != std::string::npos) {
    const size_t end = s.find_first_of(delim, at);
    cols.push_back(s.substr(at, end == std::string::npos ? std::string::npos : end - at));
    at = end == std::string::npos ? end : s.find_first_not_of(delim, end);
  }
  return cols;
}
/* h = h * seed + (char)c over the bytes, char signed as on x86 (utils/string.h:130-137) */
template <typename T = unsigned int> T BKDRHash(const char *str, T seed = 13131) {
  T h = 0;
  for (; *str; str++) h = h * seed + (T)(*str);
  return h;
}

/* ---- utils/vec1.h Vec: the apps' host fp64 vector ----------------------------
 * What an unchanged app computes with on the host (sent2vec.cpp's learn_instance); the
 * library's kernels never use it.  random() is Vec::randInit (vec1.h:229-232): (rand() /
 * (float)RAND_MAX - 0.5) / size from the process's rand() stream (process_rand, swiftmpi_compat.h),
 * element by element. */
class Vec {
 public:
  typedef double value_type;
  Vec() {}
  explicit Vec(size_t n) : _d(n, 0.0) {}
  void init(size_t n, bool random_init = false) {
    _d.assign(n, 0.0);
    if (random_init) random();
  }
  void clear() { std::fill(_d.begin(), _d.end(), 0.0); }
  void random() {
    for (size_t i = 0; i < _d.size(); i++) _d[i] = (process_rand()() / (float)RAND_MAX - 0.5) / _d.size();
  }
  size_t size() const { return _d.size(); }
  value_type *data() { return _d.data(); }
  const value_type *data() const { return _d.data(); }
  value_type &operator[](size_t i) { return _d[i]; }
  const value_type &operator[](size_t i) const { return _d[i]; }
  value_type dot(const Vec &o) const {  // sequential fp64 sum (vec1.h:103-110)
    CHECK_EQ(size(), o.size());
    value_type r = 0.0;
    for (size_t i = 0; i < size(); i++) r += _d[i] * o._d[i];
    return r;
  }
  std::string to_str() const {
    std::ostringstream os;
    os << *this;
    return os.str();
  }
  friend std::ostream &operator<<(std::ostream &os, const Vec &v) {  // "Vec:\t" then "x " per element
    os << "Vec:\t";
    for (size_t i = 0; i < v.size(); i++) os << v._d[i] << " ";
    return os;
  }
  template <class F> friend Vec zip(const Vec &a, const Vec &b, F f) {
    CHECK_EQ(a.size(), b.size());
    Vec r(a.size());
    for (size_t i = 0; i < a.size(); i++) r._d[i] = f(a._d[i], b._d[i]);
    return r;
  }
  template <class F> friend Vec map1(const Vec &a, F f) {
    Vec r(a.size());
    for (size_t i = 0; i < a.size(); i++) r._d[i] = f(a._d[i]);
    return r;
  }
  friend Vec operator*(const Vec &a, value_type b) { return map1(a, [b](value_type x) { return x * b; }); }
  friend Vec operator*(value_type b, const Vec &a) { return a * b; }
  friend Vec operator*(const Vec &a, const Vec &b) { return zip(a, b, [](value_type x, value_type y) { return x * y; }); }
  friend Vec operator/(const Vec &a, value_type b) { return map1(a, [b](value_type x) { return x / b; }); }
  friend Vec operator/(value_type b, const Vec &a) { return map1(a, [b](value_type x) { return b / x; }); }
  friend Vec operator/(const Vec &a, const Vec &b) { return zip(a, b, [](value_type x, value_type y) { return x / y; }); }
  friend Vec operator+(const Vec &a, value_type b) { return map1(a, [b](value_type x) { return x + b; }); }
  friend Vec operator+(value_type b, const Vec &a) { return a + b; }
  friend Vec operator+(const Vec &a, const Vec &b) { return zip(a, b, [](value_type x, value_type y) { return x + y; }); }
  friend Vec operator-(const Vec &a, value_type b) { return map1(a, [b](value_type x) { return x - b; }); }
  friend Vec operator-(value_type b, const Vec &a) { return map1(a, [b](value_type x) { return b - x; }); }
  friend Vec operator-(const Vec &a, const Vec &b) { return zip(a, b, [](value_type x, value_type y) { return x - y; }); }
  friend Vec &operator+=(Vec &a, const Vec &b) {
    CHECK_EQ(a.size(), b.size());
    for (size_t i = 0; i < a.size(); i++) a._d[i] += b._d[i];
    return a;
  }
  friend Vec &operator+=(Vec &a, value_type b) {
    for (auto &x : a._d) x += b;
    return a;
  }
  friend Vec &operator-=(Vec &a, const Vec &b) {
    CHECK_EQ(a.size(), b.size());
    for (size_t i = 0; i < a.size(); i++) a._d[i] -= b._d[i];
    return a;
  }
  friend Vec &operator-=(Vec &a, value_type b) {
    for (auto &x : a._d) x -= b;
    return a;
  }
  friend Vec sqrt(const Vec &a) { return map1(a, [](value_type x) { return std::sqrt(x); }); }

 private:
  std::vector<value_type> _d;
};

/* ---- utils/SpinLock.h ------------------------------------------------------- */
class SpinLock {
 public:
  void lock() {
    while (_f.test_and_set(std::memory_order_acquire)) {
    }
  }
  void unlock() { _f.clear(std::memory_order_release); }

 private:
  std::atomic_flag _f = ATOMIC_FLAG_INIT;
};

/* ---- utils/AsynExec.h: the apps' host thread pool --------------------------
 * async_exec(n, task, channel) runs `task` on n threads and returns when all
 * are done (AsynExec.h:102-123); nthreads = 1 — the reference's only
 * deterministic setting — runs it on the caller's thread. */
class AsynExec {
 public:
  typedef std::function<void()> task_t;
  struct channel_t {};
  AsynExec() {}
  explicit AsynExec(int thread_num) : _n(thread_num) {}
  std::shared_ptr<channel_t> open() { return std::make_shared<channel_t>(); }
  void set_thread_num(int x) { _n = x; }
  int thread_num() const { return _n; }

 private:
  int _n = 0;
};
inline void async_exec(int thread_num, AsynExec::task_t &task, std::shared_ptr<AsynExec::channel_t>) {
  if (thread_num <= 1) {
    task();
    return;
  }
  std::vector<std::thread> ts;
  for (int i = 0; i < thread_num; i++) ts.emplace_back([&task] { task(); });
  for (auto &t : ts) t.join();
}

}  // namespace swift_snails

/* ---- utils/CMDLine.h ------------------------------------------------------- */
namespace fms {
class CMDLine {
 public:
  std::string delimiter = ";,";
  CMDLine(int argc, char **argv) {
    for (int i = 1; i < argc; i++) {
      std::string s(argv[i]);
      if (!name(s)) throw "cannot parse " + s;
      if (value.count(s)) throw "the parameter " + s + " is already specified";
      std::string next = i + 1 < argc ? std::string(argv[i + 1]) : std::string("-");
      if (i + 1 < argc && !name(next)) {
        value[s] = argv[i + 1];
        i++;
      } else {
        value[s] = "";
      }
    }
  }
  std::string registerParameter(const std::string &p, const std::string &h) {
    help[p] = h;
    return p;
  }
  bool hasParameter(const std::string &p) const { return value.count(p) != 0; }
  void setValue(const std::string &p, const std::string &v) { value[p] = v; }
  const std::string &getValue(const std::string &p) { return value[p]; }
  std::string getValue(const std::string &p, const std::string &d) { return hasParameter(p) ? value[p] : d; }
  double getValue(const std::string &p, const double &d) { return hasParameter(p) ? std::atof(value[p].c_str()) : d; }
  int getValue(const std::string &p, const int &d) { return hasParameter(p) ? std::atoi(value[p].c_str()) : d; }
  void print_help() const {
    for (const auto &h : help) {
      std::cout << "-" << h.first;
      for (size_t i = h.first.size() + 1; i < 16; i++) std::cout << " ";
      std::cout << h.second << std::endl;
    }
  }
  void checkParameters() const {
    for (const auto &v : value)
      if (!help.count(v.first)) throw "the parameter " + v.first + " does not exist";
  }

 private:
  static bool name(std::string &s) {
    if (s.empty() || s[0] != '-') return false;
    s = s.substr(s.size() > 1 && s[1] == '-' ? 2 : 1);
    return true;
  }
  std::map<std::string, std::string> help, value;
};
}  // namespace fms

#endif /* SWIFTMPI_SWIFTMPI_H_ */
