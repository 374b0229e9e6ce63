// product/pdht_hooks_entry.h -- hook points of the C-ABI entry points
// (pdht_var.hip, pdht_fixed128.hip), product build: none taken.
#pragma once

namespace pdht {

template <class... A>
static inline int hook_var_city64(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_key_stream_var(A &&...) { return kNoVariant; }
template <class... A>
static inline int hook_crc128_long(A &&...) { return kNoVariant; }

}  // namespace pdht
