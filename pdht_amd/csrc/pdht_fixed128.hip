// pdht_fixed128.hip -- device-resident CityHash128 / CityHashCrc128 batches of
// fixed-length keys (include/pdht_hip.h).
#include "launch.h"
#include "pdht_hooks_entry.h"  // A/B hook points (product/: none taken)

using namespace pdht;

PDHT_API int pdht_city128_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                    uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity128{}, Sink128{nullptr, out}, ST(s));
}

PDHT_API int pdht_city128_seed_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                         uint64_t lo, uint64_t hi, uint64_t *out,
                                         pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity128Seed{lo, hi}, Sink128{nullptr, out}, ST(s));
}

PDHT_API int pdht_citycrc128_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                       uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  if (keylen > 900) {  // CityHashCrc256 rounds: CRC-32C byte tables in LDS
    if (int rc = hook_crc128_long(keys, stride, keylen, n, out, s); rc != kNoVariant) return rc;
    return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128>{}, Sink128{nullptr, out}, ST(s));
  }
  return launch_fixed(keys, stride, keylen, n, AlgoCrc128{}, Sink128{nullptr, out}, ST(s));
}

PDHT_API int pdht_citycrc128_seed_batch_dev(const void *keys, size_t stride, size_t keylen,
                                            size_t n, uint64_t lo, uint64_t hi, uint64_t *out,
                                            pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  if (keylen > 900)
    return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128Seed>{{lo, hi}}, Sink128{nullptr, out},
                        ST(s));
  return launch_fixed(keys, stride, keylen, n, AlgoCrc128Seed{lo, hi}, Sink128{nullptr, out}, ST(s));
}
