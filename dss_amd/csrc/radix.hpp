// Hand-written LSD radix sort for the index build and the per-batch key
// grouping (north_star "LDS-tiled radix sort of 64-bit
// cell IDs with wavefront ballot/prefix-scan compaction").  Stable, sorts the
// low `bits` bits of unsigned keys ascending; ki/vi are left untouched and the
// result lands in ko/vo (hipCUB DeviceRadixSort argument meaning, so the call
// sites read the same).  n < 2^32 - 4096.
#pragma once
#include "common.hpp"

namespace dss {

template <typename K, typename V>
void radix_sort_pairs(const K *ki, K *ko, const V *vi, V *vo, int64_t n, int bits, DevBuf<unsigned char> &tmp,
                      hipStream_t s);

// The same over the first *dn keys (a device-side count, <= n_max): no host
// sync; `bits` is taken as given (no varying-bit narrowing).
template <typename K, typename V>
void radix_sort_pairs_dn(const K *ki, K *ko, const V *vi, V *vo, int64_t n_max, const int64_t *dn, int bits,
                         DevBuf<unsigned char> &tmp, hipStream_t s);

// (u64 key, u32 value) pairs, as radix_sort_pairs, moved as packed 8-B words
// when the keys' constant low bits leave room for the values (level-13 cell
// ids with entity ids): 8 B per element per middle pass instead of 12.
void radix_sort_pairs_packed(const uint64_t *ki, uint64_t *ko, const uint32_t *vi, uint32_t *vo, int64_t n, int bits,
                             DevBuf<unsigned char> &tmp, hipStream_t s);

template <typename K>
void radix_sort_keys(const K *ki, K *ko, int64_t n, int bits, DevBuf<unsigned char> &tmp, hipStream_t s);

}  // namespace dss
