// tuning/pdht_hooks.h -- the TUNING build's answer to product/pdht_hooks.h
// (libpdht_hip_tuning.so only: the Makefile puts this directory, not
// product/, on its include path).  A process-wide variant number
// (pdht_hip_set_variant, tuning/pdht_tuning.hip) selects an alternative
// kernel or shape where one exists, and the workgroups per CU of the
// persistent grids can be overridden; pdht_hip_tuning.h lists the variants.
#pragma once
#include <cstddef>
#include <cstdint>

namespace pdht {

constexpr int kNoVariant = -1;
int tuning_variant();
int tuning_per_cu();

static inline int hook_per_cu(int per_cu) {
  const int o = tuning_per_cu();
  return o ? o : per_cu;
}
// 61: the chunked copy pipeline instead of zero-copy on pinned buffers
static inline bool hook_zero_copy(bool dflt) { return tuning_variant() == 61 ? false : dflt; }
// the bucketing workspace always reserves the two-pass region (variants force
// two passes at any nranks)
static inline bool hook_bucket_reserve(bool, size_t keysize) {
  return keysize == 8 || keysize == 16 || keysize == 32;
}
// 294 / 295: tile-local pass-1 tiles of 8192 keys (8/16-B keys)
static inline unsigned hook_tl_tile_shift(unsigned dflt, size_t keysize) {
  const int v = tuning_variant();
  if (v == 302 && keysize == 16) return 12;  // 16-B keys' pass 1 in 4096-key tiles (8 x 8, r06 first form)
  return (v == 294 || v == 295 || v == 297) && keysize <= 16 ? 13 : dflt;
}
// 164 / 295: two-pass arrays of 8/16-B keys on the balanced digit split
static inline bool hook_fine_plus(bool dflt) {
  return tuning_variant() == 164 || tuning_variant() == 295 ? false : dflt;
}

}  // namespace pdht
