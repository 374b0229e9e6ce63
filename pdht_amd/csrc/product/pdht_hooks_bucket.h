// product/pdht_hooks_bucket.h -- pdht_bucket.hip's hook points, product
// build: every choice stays the product's (product/pdht_hooks.h explains the
// mechanism).
#pragma once

namespace pdht {

template <class K>
static inline K hook_bucket_kind(K dflt, bool, u32) { return dflt; }
template <class S>
static inline S hook_staged_shape(S dflt) { return dflt; }
static inline void hook_tl_order(u32, u64, u32 *, u32 *) {}
// the r02-r05 two passes (the A/B build's baseline): not compiled here
template <class... A>
static inline int hook_two_pass_r05(A &&...) { return kNoVariant; }
static inline size_t hook_two_pass_region(size_t dflt, size_t, size_t, u32) { return dflt; }
template <int L, class Out, class... A>
static inline int hook_tl_shape(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_staged_launch(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_records(A &&...) { return kNoVariant; }

}  // namespace pdht
