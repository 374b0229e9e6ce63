// tuning/pdht_tuning.hip -- the process-wide A/B state of
// libpdht_hip_tuning.so and its two extra entry points
// (pdht_hip_tuning.h).  Compiled into the tuning library only; the product
// libraries have no mutable global knobs.
#include <hip/hip_runtime.h>

#include <atomic>

#include "../pdht_hip_tuning.h"
#include "pdht_hooks.h"

namespace pdht {
static std::atomic<int> g_variant{0};
static std::atomic<int> g_per_cu{0};
int tuning_variant() { return g_variant.load(std::memory_order_relaxed); }
int tuning_per_cu() { return g_per_cu.load(std::memory_order_relaxed); }
}  // namespace pdht

#define PDHT_API extern "C" __attribute__((visibility("default")))
PDHT_API int pdht_hip_set_variant(int v) { return pdht::g_variant.exchange(v); }
PDHT_API int pdht_hip_set_blocks_per_cu(int per_cu) { return pdht::g_per_cu.exchange(per_cu); }
