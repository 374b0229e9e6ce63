// city_host.hip -- the scalar city.h / citycrc.h API (include/pdht_city.h).
//
// Host instantiations of the same city_core.h templates the kernels use, so
// a single-key CityHash64 on the CPU and a batch on the GPU are produced by
// one body of code.  Replaces the compiled reference city.c for callers such
// as libpdht/hash.c:26 and the user hash functions of test/ and bench/.
#include "../../include/pdht_city.h"
#include "city_core.h"

#define PDHT_API extern "C" __attribute__((visibility("default")))

using pdht::HostReader;

static inline uint128 to_c(pdht::u128 r) {
  uint128 o;
  o.first = r.lo;
  o.second = r.hi;
  return o;
}

PDHT_API uint64 CityHash64(const char *buf, size_t len) {
  return pdht::city64(HostReader{reinterpret_cast<const uint8_t *>(buf)}, len);
}
PDHT_API uint64 CityHash64WithSeed(const char *buf, size_t len, uint64 seed) {
  return pdht::city64_seeds(HostReader{reinterpret_cast<const uint8_t *>(buf)}, len, pdht::kK2, seed);
}
PDHT_API uint64 CityHash64WithSeeds(const char *buf, size_t len, uint64 seed0, uint64 seed1) {
  return pdht::city64_seeds(HostReader{reinterpret_cast<const uint8_t *>(buf)}, len, seed0, seed1);
}
PDHT_API uint128 CityHash128(const char *s, size_t len) {
  return to_c(pdht::city128(HostReader{reinterpret_cast<const uint8_t *>(s)}, len));
}
PDHT_API uint128 CityHash128WithSeed(const char *s, size_t len, uint128 seed) {
  return to_c(pdht::city128_seed(HostReader{reinterpret_cast<const uint8_t *>(s)}, len,
                                 pdht::u128{seed.first, seed.second}));
}
PDHT_API uint128 CityHashCrc128(const char *s, size_t len) {
  return to_c(pdht::crc128(HostReader{reinterpret_cast<const uint8_t *>(s)}, len));
}
PDHT_API uint128 CityHashCrc128WithSeed(const char *s, size_t len, uint128 seed) {
  return to_c(pdht::crc128_seed(HostReader{reinterpret_cast<const uint8_t *>(s)}, len,
                                pdht::u128{seed.first, seed.second}));
}
PDHT_API void CityHashCrc256(const char *s, size_t len, uint64 *result) {
  pdht::crc256(HostReader{reinterpret_cast<const uint8_t *>(s)}, len, result);
}
// city.c:173-187 and :190-198 (non-static in the reference, not in city.h)
PDHT_API uint128 WeakHashLen32WithSeeds6(uint64 w, uint64 x, uint64 y, uint64 z, uint64 a, uint64 b) {
  return to_c(pdht::weak32(w, x, y, z, a, b));
}
PDHT_API uint128 WeakHashLen32WithSeeds(const char *s, uint64 a, uint64 b) {
  const pdht::HostReader r{reinterpret_cast<const uint8_t *>(s)};
  return to_c(pdht::weak32(pdht::fetch64(r, 0), pdht::fetch64(r, 8), pdht::fetch64(r, 16),
                           pdht::fetch64(r, 24), a, b));
}
