/*
 * pdht_hash.c -- drop-in replacement of libpdht/hash.c (C99).
 *
 * Scalar path: identical to the reference (hash.c:25-30), one CityHash64 on
 * the CPU per key (pdht_city.h, same code the GPU kernels run).
 * Batch path: pdht_hash_batch hands the whole batch to the GPU engine
 * (pdht_hip.h, fused digest + ptindex + rank) when the table uses the
 * default hash, and calls the installed plugin per key otherwise -- exactly
 * what n calls of dht->hashfn (putget.c:53) would have produced.
 *
 * Compiled standalone here (stand-in pdht_t, see pdht_hash.h) and, with
 * -DPDHT_HIP_WITH_REAL_PDHT, against the reference pdht.h.
 */
#include "pdht_hash.h"

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "pdht_city.h"
#include "pdht_hip.h"

/* The batch entry points write rank r of key i as a u32 at
 * (char *)rank + i * sizeof(ptl_process_t): that needs the Portals 4 layout
 * (8-byte union, .rank at offset 0), whichever header supplied the type.
 * (C99: a negative array size fails the build.) */
typedef char pdht_hip_ptl_process_is_8_bytes[sizeof(ptl_process_t) == 8 ? 1 : -1];
typedef char pdht_hip_ptl_rank_at_offset_0[offsetof(ptl_process_t, rank) == 0 ? 1 : -1];
typedef char pdht_hip_ptl_rank_is_u32[sizeof(((ptl_process_t *)0)->rank) == 4 ? 1 : -1];

#ifndef PDHT_HIP_WITH_REAL_PDHT
#define PDHT_SHIM_API __attribute__((visibility("default")))
/* c->size stand-in; a real pdht build reads c->size instead. */
PDHT_SHIM_API int pdht_hip_shim_nranks = 1;

PDHT_SHIM_API void pdht_hip_table_init(pdht_t *dht, unsigned keysize, unsigned nptes) {
  memset(dht, 0, sizeof *dht);
  dht->keysize = keysize;      /* init.c:80 */
  dht->hashfn = pdht_hash;     /* init.c:90 */
  dht->ptl.nptes = nptes;      /* init.c:94 */
}
#else
#define PDHT_SHIM_API
#endif

/* libpdht/hash.c:25-30 */
PDHT_SHIM_API void pdht_hash(pdht_t *dht, void *key, ptl_match_bits_t *mbits,
                             uint32_t *ptindex, ptl_process_t *rank) {
  *mbits = CityHash64((char *)key, dht->keysize);
#ifndef PDHT_HIP_MPI_FLAVOUR
  *ptindex = *mbits % dht->ptl.nptes;
#else
  (void)ptindex; /* libmpipdht/hash.c:6-9 leaves it untouched */
#endif
  (*rank).rank = *mbits % PDHT_HIP_NRANKS();
}

/* libpdht/hash.c:39-41 */
PDHT_SHIM_API void pdht_sethash(pdht_t *dht, pdht_hashfunc hfun) { dht->hashfn = hfun; }

PDHT_SHIM_API int pdht_hash_batch(pdht_t *dht, const void *keys, size_t n,
                                  ptl_match_bits_t *mbits, uint32_t *ptindex,
                                  ptl_process_t *rank, int device) {
  if (n == 0) return 0;
  if (!dht || !keys || !mbits || !rank) return PDHT_HIP_ERROR;
  if (dht->hashfn != pdht_hash) {
    /* a user plugin (pdht_sethash): run it exactly as putget.c:53 would */
    uint32_t scratch;
    const char *k = (const char *)keys;
    for (size_t i = 0; i < n; ++i)
      dht->hashfn(dht, (void *)(k + i * dht->keysize), &mbits[i],
                  ptindex ? &ptindex[i] : &scratch, &rank[i]);
    return 0;
  }
  return pdht_place_batch_host(keys, dht->keysize, n,
#ifndef PDHT_HIP_MPI_FLAVOUR
                               dht->ptl.nptes, (uint32_t)PDHT_HIP_NRANKS(), mbits, ptindex,
#else
                               1u, (uint32_t)PDHT_HIP_NRANKS(), mbits, NULL,
#endif
                               rank, sizeof(ptl_process_t), device);
}

PDHT_SHIM_API int pdht_hash_batch_dev(pdht_t *dht, const void *keys, size_t n,
                                      ptl_match_bits_t *mbits, uint32_t *ptindex,
                                      ptl_process_t *rank, uint64_t *rank_hist,
                                      void *stream) {
  if (!dht) return PDHT_HIP_ERROR;
  if (dht->hashfn != pdht_hash) return PDHT_HIP_ERROR; /* plugins run on the CPU only */
#ifdef PDHT_HIP_MPI_FLAVOUR
  (void)ptindex; /* libmpipdht/hash.c:6-9 computes no ptindex */
#endif
  return pdht_place_batch_dev(keys, dht->keysize, n,
#ifndef PDHT_HIP_MPI_FLAVOUR
                              dht->ptl.nptes, (uint32_t)PDHT_HIP_NRANKS(), mbits, ptindex,
#else
                              1u, (uint32_t)PDHT_HIP_NRANKS(), mbits, NULL,
#endif
                              rank, sizeof(ptl_process_t), rank_hist,
                              (pdht_hip_stream_t)stream);
}
