// glibc rand() (random_r TYPE_3: o[i] = o[i-3] + o[i-31] mod 2^32, output o >> 1) by jump-ahead on
// the device: the recurrence is linear in its state, so o[3 + e] = sum_j a_j o[3 + j] with
// sum_j a_j x^j = x^e mod (x^31 - x^28 - 1) — a thread squares-and-multiplies to the start of its
// run of outputs, then steps the recurrence (GlibcRand in swps_host.cpp is the host form).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace swps {

struct Poly31 {
  uint32_t c[31];
};
__device__ inline void poly_mulmod(const Poly31 &a, const Poly31 &b, Poly31 &out) {
  uint32_t t[61];
  for (int i = 0; i < 61; i++) t[i] = 0;
  for (int i = 0; i < 31; i++)
    for (int j = 0; j < 31; j++) t[i + j] += a.c[i] * b.c[j];
  for (int d = 60; d >= 31; d--) {  // x^d = x^(d-3) + x^(d-31)
    t[d - 3] += t[d];
    t[d - 31] += t[d];
  }
  for (int i = 0; i < 31; i++) out.c[i] = t[i];
}

constexpr uint64_t kRandRun = 8192;  // outputs per thread

// the 31 values o[3..33] after srand(seed) (glibc's seeding, GlibcRand)
inline std::vector<uint32_t> glibc_base(uint32_t seed) {
  std::vector<uint32_t> base(31);
  int32_t s0[34];
  s0[0] = (int32_t)(seed ? seed : 1);
  for (int i = 1; i < 31; i++) {
    const int64_t hi = s0[i - 1] / 127773, lo = s0[i - 1] % 127773;
    int64_t v = 16807 * lo - 2836 * hi;
    if (v < 0) v += 2147483647;
    s0[i] = (int32_t)v;
  }
  for (int i = 31; i < 34; i++) s0[i] = s0[i - 31];
  for (int j = 0; j < 31; j++) base[j] = (uint32_t)s0[3 + j];
  return base;
}

// a thread's ring of the 31 values o[m0 .. m0 + 30] (m0 >= 3)
__device__ inline void glibc_ring_at(const uint32_t *__restrict__ base, uint64_t m0, uint32_t *ring) {
  Poly31 r, x;  // r = x^(m0-3) mod P
  for (int i = 0; i < 31; i++) {
    r.c[i] = i == 0 ? 1u : 0u;
    x.c[i] = i == 1 ? 1u : 0u;
  }
  for (uint64_t e = m0 - 3; e; e >>= 1) {
    if (e & 1) poly_mulmod(r, x, r);
    poly_mulmod(x, x, x);
  }
  for (int d = 0; d < 31; d++) {
    uint32_t v = 0;
    for (int j = 0; j < 31; j++) v += r.c[j] * base[j];
    ring[d] = v;
    const uint32_t top = r.c[30];  // r <- x * r mod P
    for (int j = 30; j > 0; j--) r.c[j] = r.c[j - 1];
    r.c[0] = top;
    r.c[28] += top;
  }
}

}  // namespace swps
