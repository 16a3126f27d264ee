// Host-side utilities of libswps: error state, BKDR key hashing, glibc rand()
// emulation, the hash-frag node map and the reference config file format.
#include <fcntl.h>
#include <unistd.h>

#include <cstdio>
#include <fstream>

#include "swps_internal.h"

namespace swps {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }
int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

// utils/string.h:130-137 BKDRHash<size_t>(s, 13131); `char` is signed on
// x86-64 so non-ASCII bytes add sign-extended values.
uint64_t bkdr(const char *s) {
  uint64_t h = 0;
  while (*s) h = h * 13131ULL + (uint64_t)(int64_t)(signed char)(*s++);
  return h;
}

// glibc srandom_r/random_r for TYPE_3 (degree 31, separation 3): the state
// is seeded by the Park–Miller LCG, 310 outputs are discarded, and each output
// is (r[i-31] + r[i-3]) >> 1.  Reproduces rand() after srand(seed), which the
// reference's Vec::randInit draws from (utils/vec1.h:229-232).
GlibcRand::GlibcRand(uint32_t seed) {
  if (seed == 0) seed = 1;
  int32_t s[34];
  s[0] = (int32_t)seed;
  for (int i = 1; i < 31; i++) {
    int64_t hi = s[i - 1] / 127773, lo = s[i - 1] % 127773;
    int64_t w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    s[i] = (int32_t)w;
  }
  for (int i = 31; i < 34; i++) s[i] = s[i - 31];
  for (int i = 0; i < 34; i++) r[i] = s[i];
  idx = 0;  // r holds o[i..i+33] as a ring starting at idx
  for (int i = 34; i < 344; i++) (void)next();
  produced = 0;
}

int32_t GlibcRand::next() {
  // ring of the last 34 words, r[idx] the oldest (i-34): new = r[i-31] + r[i-3]
  int32_t v = (int32_t)((uint32_t)r[(idx + 3) % 34] + (uint32_t)r[(idx + 31) % 34]);
  r[idx] = v;
  idx = (idx + 1) % 34;
  produced++;
  return (int32_t)((uint32_t)v >> 1);
}

namespace {
// a (mod x^31 - x^28 - 1) polynomial over Z / 2^32: c[j] is the coefficient of x^j
void poly31_mulmod(const uint32_t *a, const uint32_t *b, uint32_t *out) {
  uint32_t t[61] = {0};
  for (int i = 0; i < 31; i++)
    for (int j = 0; j < 31; j++) t[i + j] += a[i] * b[j];
  for (int d = 60; d >= 31; d--) {  // x^d = x^(d-3) + x^(d-31)
    t[d - 3] += t[d];
    t[d - 31] += t[d];
  }
  for (int i = 0; i < 31; i++) out[i] = t[i];
}
}  // namespace

void GlibcRand::discard(uint64_t k) {
  if (k < 4096) {
    for (uint64_t i = 0; i < k; i++) (void)next();
    return;
  }
  // the ring holds o[i-34 .. i-1] (r[idx] the oldest) and the next output is o[i]; with
  // b_j = o[i-31+j], o[i-31+e] = sum_j a_j b_j where sum_j a_j x^j = x^e mod P (o[n] = o[n-3] +
  // o[n-31]: x^31 = x^28 + 1).  After k outputs the ring holds o[i+k-34+t], t = 0..33: e = k-3+t
  uint32_t b[31];
  for (int j = 0; j < 31; j++) b[j] = (uint32_t)r[(idx + 3 + j) % 34];
  uint32_t a[31] = {0}, x[31] = {0};
  a[0] = 1;
  x[1] = 1;
  for (uint64_t e = k - 3; e; e >>= 1) {
    if (e & 1) poly31_mulmod(a, x, a);
    poly31_mulmod(x, x, x);
  }
  for (int t = 0; t < 34; t++) {
    uint32_t v = 0;
    for (int j = 0; j < 31; j++) v += a[j] * b[j];
    r[t] = (int32_t)v;
    const uint32_t top = a[30];  // a <- x * a mod P
    for (int j = 30; j > 0; j--) a[j] = a[j - 1];
    a[0] = top;
    a[28] += top;
  }
  idx = 0;
  produced += k;
}

int Config::parse(const std::string &path) {
  std::ifstream f(path);
  if (!f) return fail(SWPS_E_IO, "conf can not open: " + path);
  auto trim = [](std::string s) {
    size_t a = s.find_first_not_of(" \t\n\r");
    if (a == std::string::npos) return std::string();
    size_t b = s.find_last_not_of(" \t\n\r");
    return s.substr(a, b - a + 1);
  };
  std::string line, cur;
  while (std::getline(f, line)) {
    line = trim(line);
    if (line.empty() || line[0] == '#') continue;
    if (line.compare(0, 6, "import") == 0) {
      std::string p = trim(line.substr(line.find(' ') + 1));
      if (p == path) return fail(SWPS_E_CFG, "recursive import");
      SWPS_TRY(parse(p));
      continue;
    }
    if (line.front() == '[' && line.back() == ']') {
      cur = trim(line.substr(1, line.size() - 2));
      if (cur.empty()) return fail(SWPS_E_CFG, "empty section");
      continue;
    }
    size_t c = line.find(':');
    if (c == std::string::npos) return fail(SWPS_E_CFG, "bad config line: " + line);
    std::string k = trim(line.substr(0, c)), v = trim(line.substr(c + 1));
    bool placed = false;
    for (auto &s : sections)
      if (s.first == cur) {
        bool dup = false;
        for (auto &kv : s.second) dup |= kv.first == k;
        if (!dup) s.second.emplace_back(k, v);  // std::map::insert keeps the first
        placed = true;
      }
    if (!placed) sections.push_back({cur, {{k, v}}});
  }
  return SWPS_OK;
}

bool Config::get(const std::string &sec, const std::string &key, std::string &out) const {
  for (auto &s : sections)
    if (s.first == sec)
      for (auto &kv : s.second)
        if (kv.first == key) {
          out = kv.second;
          return true;
        }
  return false;
}

// Running checksum of snapshot payloads: 8-byte words folded with a
// multiply-xorshift step (each put/get chunk independently, chained), tail
// bytes one at a time.  Detects bit flips and truncation; not cryptographic.
uint64_t checksum64(uint64_t h, const void *p, size_t n) {
  const unsigned char *b = (const unsigned char *)p;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, b + i, 8);
    h = (h ^ w) * 0x9E3779B97F4A7C15ULL;
    h ^= h >> 29;
  }
  for (; i < n; i++) {
    h = (h ^ b[i]) * 0x100000001B3ULL;
    h ^= h >> 29;
  }
  return (h ^ (uint64_t)n) * 0xff51afd7ed558ccdULL;
}

// Writes go to <path>.tmp; finish_write flushes and fsyncs it, renames it
// over <path> and fsyncs the directory, so a crash at any point leaves either
// the previous snapshot or the new one, never a torn file (an unfinished
// writer removes its temporary).
int SnapFile::open(const std::string &p, bool write) {
  path = p;
  writing = write;
  tmp = write ? p + ".tmp" : p;
  f = fopen(tmp.c_str(), write ? "wb" : "rb");
  if (!f) return fail(SWPS_E_IO, std::string(write ? "cannot write " : "cannot open ") + tmp);
  return SWPS_OK;
}

SnapFile::~SnapFile() {
  if (f) fclose(f);
  if (writing && !committed) (void)std::remove(tmp.c_str());
}

int SnapFile::put(const void *p, size_t n) {
  if (n && fwrite(p, 1, n, f) != n) return fail(SWPS_E_IO, "short write to " + path);
  sum = checksum64(sum, p, n);
  return SWPS_OK;
}

int SnapFile::get(void *p, size_t n) {
  if (n && fread(p, 1, n, f) != n) return fail(SWPS_E_IO, "truncated snapshot " + path);
  sum = checksum64(sum, p, n);
  return SWPS_OK;
}

int SnapFile::finish_write() {
  const uint64_t s = sum;
  if (fwrite(&s, 1, 8, f) != 8) return fail(SWPS_E_IO, "short write to " + tmp);
  if (fflush(f) != 0 || fsync(fileno(f)) != 0) return fail(SWPS_E_IO, "cannot flush " + tmp);
  const int bad = fclose(f);
  f = nullptr;
  if (bad) return fail(SWPS_E_IO, "cannot close " + tmp);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) return fail(SWPS_E_IO, "cannot rename " + tmp + " to " + path);
  committed = true;
  const size_t slash = path.find_last_of('/');
  const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
  const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (dfd >= 0) {  // make the rename itself durable
    (void)fsync(dfd);
    ::close(dfd);
  }
  return SWPS_OK;
}

int SnapFile::finish_read() {
  uint64_t s = 0;
  if (fread(&s, 1, 8, f) != 8) return fail(SWPS_E_IO, "truncated snapshot " + path);
  if (s != sum) return fail(SWPS_E_IO, "snapshot checksum mismatch in " + path + " (corrupt file)");
  char extra;
  if (fread(&extra, 1, 1, f) != 0) return fail(SWPS_E_IO, "trailing bytes after the snapshot checksum in " + path);
  return SWPS_OK;
}

}  // namespace swps

extern "C" {

const char *swps_last_error(void) { return swps::g_last_error.c_str(); }
int swps_version(void) { return 1; }

uint64_t swps_fmix64(uint64_t x) { return swps::fmix64(x); }
uint64_t swps_bkdr(const char *s) { return swps::bkdr(s); }

// cluster/hashfrag.h:33-49: frag i -> node clamp(i / int(frag_num/num_nodes) + 1, 1, num_nodes)
int swps_hashfrag_table(int32_t frag_num, int32_t num_nodes, uint32_t *out) {
  if (num_nodes <= 0 || frag_num <= 0) return swps::fail(SWPS_E_CFG, "frag_num and num_nodes must be positive");
  int each = frag_num / num_nodes;
  if (each == 0) return swps::fail(SWPS_E_CFG, "frag_num < num_nodes (reference divides by zero)");
  for (int i = 0; i < frag_num; i++) {
    int id = (int)(uint32_t)(i / each) + 1;
    if (id < 1) id = 1;
    if (id > num_nodes) id = num_nodes;
    out[i] = (uint32_t)id;
  }
  return SWPS_OK;
}

// cluster/hashfrag.h:51-56
int swps_to_node_id(const uint64_t *keys, uint64_t n, int32_t frag_num, const uint32_t *table, int32_t *out) {
  if (frag_num <= 0) return swps::fail(SWPS_E_CFG, "frag_num must be positive");
  for (uint64_t i = 0; i < n; i++) out[i] = (int32_t)table[swps::fmix64(keys[i]) % (uint64_t)frag_num];
  return SWPS_OK;
}

}  // extern "C"
