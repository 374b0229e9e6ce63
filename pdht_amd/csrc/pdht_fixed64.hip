// pdht_fixed64.hip -- device-resident CityHash64 batches of fixed-length keys and
// the fused pdht_hash placement (include/pdht_hip.h).
#include "launch.h"

using namespace pdht;

PDHT_API int pdht_city64_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                   uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity64{}, Sink64{nullptr, out}, ST(s));
}

PDHT_API int pdht_city64_seeds_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                         uint64_t seed0, uint64_t seed1, uint64_t *out,
                                         pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity64Seeds{seed0, seed1}, Sink64{nullptr, out},
                      ST(s));
}

PDHT_API int pdht_place_batch_dev(const void *keys, size_t keysize, size_t n, uint32_t nptes,
                                  uint32_t nranks, uint64_t *mbits, uint32_t *ptindex, void *rank,
                                  size_t rank_stride, uint64_t *hist, pdht_hip_stream_t s) {
  if (int rc = check_place(n, mbits, nptes, nranks, rank, rank_stride)) return rc;
  return launch_fixed(keys, keysize, keysize, n, AlgoCity64{},
                      make_place_sink(mbits, ptindex, rank, rank_stride, hist, nptes, nranks), ST(s));
}
