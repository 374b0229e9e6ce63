// product/pdht_hooks.h -- the A/B hook points of the hash paths, PRODUCT
// build: every hook answers "not taken" (kNoVariant) or returns the
// product's own choice unchanged, and the compiler removes the call.
//
// The sources include "pdht_hooks*.h" by name; the Makefile puts this
// directory on the include path of the product libraries and
// pdht_amd/csrc/tuning/ on that of libpdht_hip_tuning.so, whose headers of
// the same names route each hook to the alternative kernels and shapes the
// A/B harness selects (tools/abbench.py; DESIGN.md §4 has the measurements).
// The product sources therefore carry no #ifdef and no tuning code.
#pragma once
#include <cstddef>
#include <cstdint>

namespace pdht {

constexpr int kNoVariant = -1;

// runtime.h: workgroups per CU of a persistent grid; zero-copy on pinned
// host buffers (pdht_host.hip)
static inline int hook_per_cu(int per_cu) { return per_cu; }
static inline bool hook_zero_copy(bool dflt) { return dflt; }
// pdht_bucket.hip: reserve the two-pass region in the workspace
static inline bool hook_bucket_reserve(bool dflt, size_t) { return dflt; }
// pdht_bucket.hip: log2 keys per pass-1 tile of the tile-local two passes;
// the fine digit one bit wider for 8/16-B array outputs
static inline unsigned hook_tl_tile_shift(unsigned dflt, size_t) { return dflt; }
static inline bool hook_fine_plus(bool dflt) { return dflt; }

}  // namespace pdht
