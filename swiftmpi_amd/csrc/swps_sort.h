// Stable key/value radix sort for the per-minibatch inverted indexes.
//
// rocPRIM picks a block merge sort below 1M items: at the B = 100 minibatch
// (≈0.6M gradient records, 15-bit keys) that is ~20 kernels per sort — 37 %
// of the step on the trace (profiles/r02_b100_*).  Onesweep sorts the same
// keys in one histogram kernel plus one kernel per 8-bit digit, so the merge
// path is switched off (MergeSortLimit = 0; inputs that fit one block still
// get the single-block sort).  Same stable order, so same results.
#pragma once
#include <cstdlib>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

namespace swps {

using OnesweepCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                               rocprim::default_config, 0>;

// Wider digits for 17-20-bit keys: the bench minibatch's local key indices
// (U ~ 2^18) sort in 2 onesweep passes of 9 bits instead of 3 of 8 (same
// stable order, so same results).  Block shape of rocPRIM's gfx950 default
// (same-box A/B at the bench batch, round 4: 512 x 16, 1024 x 8 and 256 x 16 tiles
// within 0.5 % of it).
template <unsigned RB>
using OnesweepWide = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>, RB,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;

// Small inputs (< kSmallSort items: the B = 100 minibatch's ~0.6M records, a sharded
// step's ~0.2M served keys): the default tile (1024 x 16 items) leaves a handful of
// workgroups per onesweep pass; 256 x 8-item tiles give the passes 8x the workgroups.
template <unsigned RB>
using OnesweepSmall = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<256, 8>, rocprim::kernel_config<256, 8>, RB,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
constexpr uint64_t kSmallSort = 1u << 20;
// Off by default: same-box A/B at B = 100 lines 0.322 ms/step default tiles vs 0.324 small
// (the small-tile passes overlap the learn stream and slow its kernels); SWPS_SORT_SMALL=1 on.
inline int sort_small_mode() {
  static const int on = [] {
    const char *e = getenv("SWPS_SORT_SMALL");
    return e ? atoi(e) : 0;
  }();
  return on;
}

// tmp == nullptr: *bytes = the temporary storage needed (same `bits` and `n` for both calls)
inline bool sort_wide() {  // SWPS_SORT_WIDE=0: the default 8-bit digits only (A/B, tests)
  static const bool on = [] {
    const char *e = getenv("SWPS_SORT_WIDE");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

template <typename K, typename V>
inline hipError_t sort_pairs(void *tmp, size_t &bytes, const K *kin, K *kout, const V *vin, V *vout, uint64_t n,
                             int bits, hipStream_t s) {
  if (!sort_wide())
    return rocprim::radix_sort_pairs<OnesweepCfg>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits,
                                                  s);
  if (n < kSmallSort && sort_small_mode()) {
    if (bits > 16 && bits <= 20)  // two passes of 9 or 10 bits
      return rocprim::radix_sort_pairs<OnesweepSmall<10>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                          (unsigned)bits, s);
    return rocprim::radix_sort_pairs<OnesweepSmall<8>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                       (unsigned)bits, s);
  }
  if (sizeof(K) == 4 && sizeof(V) == 4 && bits > 16 && bits <= 18)
    return rocprim::radix_sort_pairs<OnesweepWide<9>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits,
                                                      s);
  if (sizeof(K) == 4 && sizeof(V) == 4 && bits > 18 && bits <= 20)
    return rocprim::radix_sort_pairs<OnesweepWide<10>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                       (unsigned)bits, s);
  return rocprim::radix_sort_pairs<OnesweepCfg>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, s);
}

// The same with the values 0, 1, 2, ... (a record's index): read from a counting iterator instead of
// an array the records kernel wrote (SWPS_SORT_IOTA=0: the array, A/B)
inline bool sort_iota() {
  static const bool on = [] {
    const char *e = getenv("SWPS_SORT_IOTA");
    return !(e && atoi(e) == 0);
  }();
  return on;
}
template <typename K>
inline hipError_t sort_pairs_iota(void *tmp, size_t &bytes, const K *kin, K *kout, uint32_t *vout, uint64_t n,
                                  int bits, hipStream_t s) {
  const rocprim::counting_iterator<uint32_t> vin(0u);
  if (!sort_wide())
    return rocprim::radix_sort_pairs<OnesweepCfg>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, s);
  if (n < kSmallSort && sort_small_mode()) {
    if (bits > 16 && bits <= 20)
      return rocprim::radix_sort_pairs<OnesweepSmall<10>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                          (unsigned)bits, s);
    return rocprim::radix_sort_pairs<OnesweepSmall<8>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                       (unsigned)bits, s);
  }
  if (sizeof(K) == 4 && bits > 16 && bits <= 18)
    return rocprim::radix_sort_pairs<OnesweepWide<9>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits,
                                                      s);
  if (sizeof(K) == 4 && bits > 18 && bits <= 20)
    return rocprim::radix_sort_pairs<OnesweepWide<10>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                       (unsigned)bits, s);
  return rocprim::radix_sort_pairs<OnesweepCfg>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits, s);
}

// Explicit tile shapes for mid-size sorts (the LR per-step plan: ~2.5M records per minibatch):
// rocPRIM's default 1024 x 16-item tiles leave ~150 workgroups per onesweep pass for 256 CUs.
// mode 1: 256 x 8 items, 2: 512 x 8, 3: 256 x 16, else rocPRIM's default (8-bit digits throughout)
template <unsigned BS, unsigned IPT>
using OnesweepTile = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<BS, IPT>, rocprim::kernel_config<BS, IPT>, 8,
                                        rocprim::block_radix_rank_algorithm::match>,
    0>;
template <typename K, typename VI, typename V>
inline hipError_t sort_pairs_tiled(int mode, void *tmp, size_t &bytes, const K *kin, K *kout, VI vin, V *vout,
                                   uint64_t n, int bits, hipStream_t s) {
  switch (mode) {
    case 1:
      return rocprim::radix_sort_pairs<OnesweepTile<256, 8>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                             (unsigned)bits, s);
    case 2:
      return rocprim::radix_sort_pairs<OnesweepTile<512, 8>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                             (unsigned)bits, s);
    case 3:
      return rocprim::radix_sort_pairs<OnesweepTile<256, 16>>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                                              (unsigned)bits, s);
    default:
      return rocprim::radix_sort_pairs<OnesweepCfg>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u, (unsigned)bits,
                                                    s);
  }
}

// keys-only form (same onesweep configuration)
template <typename K>
inline hipError_t sort_keys(void *tmp, size_t &bytes, const K *kin, K *kout, uint64_t n, int bits, hipStream_t s) {
  return rocprim::radix_sort_keys<OnesweepCfg>(tmp, bytes, kin, kout, (size_t)n, 0u, (unsigned)bits, s);
}

}  // namespace swps
