// pdht_var.hip -- device-resident batches of variable-length (offset-indexed)
// keys and their data-movement calibration (include/pdht_hip.h).
#include "launch.h"
#include "pdht_hooks_entry.h"  // A/B hook points (product/: none taken)

using namespace pdht;

PDHT_API int pdht_city64_batch_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                       size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  if (int rc = hook_var_city64(bytes, offsets, n, out, s); rc != kNoVariant) return rc;
  return launch_var(bytes, nbytes, offsets, 0, n, AlgoCity64{}, Sink64{nullptr, out}, ST(s));
}

PDHT_API int pdht_city128_batch_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                        size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_var(bytes, nbytes, offsets, 0, n, AlgoCity128{}, Sink128{nullptr, out}, ST(s));
}

PDHT_API int pdht_citycrc128_batch_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                           size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  // any key may exceed 900 B (CityHashCrc256 rounds): CRC-32C tables in LDS
  return launch_var(bytes, nbytes, offsets, 0, n, CrcLds<AlgoCrc128>{}, Sink128{nullptr, out}, ST(s));
}

// Variable-length counterpart: the default offset-indexed kernel's data
// movement (window DMA, offsets, LDS reads of every key byte, digest stores)
// with an XOR fold for the hash.
PDHT_API int pdht_hip_key_stream_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                         size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  if (int rc = hook_key_stream_var(bytes, nbytes, offsets, n, out, s); rc != kNoVariant) return rc;
  return launch_var(bytes, nbytes, offsets, 0, n, AlgoFoldVar{}, Sink64{nullptr, out}, ST(s));
}
