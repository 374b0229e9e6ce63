// product/pdht_hooks_launch.h -- launch.h's hook points, product build: none
// taken (product/pdht_hooks.h explains the mechanism).
#pragma once

namespace pdht {

template <class... A>
static inline int hook_small(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_xpose64(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_crc_long(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_long_walk(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_var(A &&...) { return kNoVariant; }
static inline u64 hook_chunk_bytes(u64 dflt) { return dflt; }

}  // namespace pdht
