/*
 * pdht_hash.h -- pdht's hash-function plugin boundary, GPU-batch capable.
 *
 * Replaces /root/reference/libpdht/hash.c (and libmpipdht/hash.c):
 *   pdht_hash     -- libpdht/hash.c:25-30   (default dht->hashfn, init.c:90)
 *   pdht_sethash  -- libpdht/hash.c:39-41   (pdht.h:353)
 *   pdht_hashfunc -- libpdht/pdht.h:196     (plugin signature)
 * and adds
 *   pdht_hash_batch / pdht_hash_batch_dev -- the same placement for n keys,
 *   computed by the GPU engine (pdht_hip.h) when dht->hashfn is pdht_hash, or
 *   by calling the installed plugin once per key (reference semantics for
 *   user hash functions such as test/scaling.c:39-43) otherwise.
 *
 * Two ways to compile it:
 *   * inside a real pdht build: define PDHT_HIP_WITH_REAL_PDHT and put the
 *     reference include dir first; pdht_t / ptl_* / the global context `c`
 *     then come from pdht.h (+ portals4.h) and our src/pdht_hash.c replaces
 *     libpdht/hash.c unchanged;
 *   * standalone (this repo, no Portals): the minimal layout-compatible
 *     stand-ins below are used.  Only the fields the hash path reads exist:
 *     keysize (pdht.h:231), hashfn (:237), ptl.nptes (:203) and the rank
 *     count c->size (pdht.h:144), which the stand-in keeps in
 *     pdht_hip_shim_nranks.
 * Define PDHT_HIP_MPI_FLAVOUR for libmpipdht semantics (ptindex untouched,
 * libmpipdht/hash.c:6-9).
 */
#ifndef PDHT_HIP_HASH_H_
#define PDHT_HIP_HASH_H_

#include <stddef.h>
#include <stdint.h>

#ifdef PDHT_HIP_WITH_REAL_PDHT
#ifdef PDHT_HIP_MPI_FLAVOUR
#include <pdht.h> /* libmpipdht/pdht.h: pdht_t, pdht_hash (:236) */
extern pdht_context_t *c; /* as libmpipdht/hash.c:4 */
#else
#include <pdht_impl.h> /* libpdht: pdht.h + pdht_hash (pdht_impl.h:128) + c */
#endif
#define PDHT_HIP_NRANKS() (c->size)
#else

#ifdef __cplusplus
extern "C" {
#endif

/* portals4.h stand-ins: ptl_match_bits_t is a uint64_t; ptl_process_t is the
 * 8-byte union { struct { ptl_nid_t nid; ptl_pid_t pid; } phys;
 * ptl_rank_t rank; } with 32-bit members. */
typedef uint64_t ptl_match_bits_t;
typedef uint32_t ptl_rank_t;
typedef union {
  struct {
    uint32_t nid;
    uint32_t pid;
  } phys;
  ptl_rank_t rank;
} ptl_process_t;

struct pdht_s;
/* libpdht/pdht.h:196 */
typedef void (*pdht_hashfunc)(struct pdht_s *dht, void *key,
                              ptl_match_bits_t *bits, uint32_t *ptindex,
                              ptl_process_t *rank);

/* Minimal pdht_t: the fields of libpdht/pdht.h:229-255 read by the hash. */
struct pdht_hip_ptl_s {
  unsigned nptes; /* pdht.h:203 */
};
struct pdht_s {
  unsigned keysize;             /* pdht.h:231 */
  pdht_hashfunc hashfn;         /* pdht.h:237 */
  struct pdht_hip_ptl_s ptl;    /* pdht.h:250 */
};
typedef struct pdht_s pdht_t;

/* c->size of the reference (pdht.h:144, :152): number of ranks. */
extern int pdht_hip_shim_nranks;
#define PDHT_HIP_NRANKS() (pdht_hip_shim_nranks)

/* Convenience constructor for the stand-in table (init.c:80, :90, :94). */
void pdht_hip_table_init(pdht_t *dht, unsigned keysize, unsigned nptes);

#ifdef __cplusplus
}
#endif
#endif /* PDHT_HIP_WITH_REAL_PDHT */

#ifdef __cplusplus
extern "C" {
#endif

/* libpdht/hash.c:25-30 -- one key, CPU (bit-identical to the reference). */
void pdht_hash(pdht_t *dht, void *key, ptl_match_bits_t *mbits,
               uint32_t *ptindex, ptl_process_t *rank);
/* libpdht/hash.c:39-41 */
void pdht_sethash(pdht_t *dht, pdht_hashfunc hfun);

/* n packed keys (dht->keysize bytes each) in HOST memory -> n placements.
 * Returns 0 (PdhtStatusOK) or 1 (PdhtStatusError, see pdht_hip_last_error).
 * ptindex may be NULL.  `device` selects the GPU. */
int pdht_hash_batch(pdht_t *dht, const void *keys, size_t n,
                    ptl_match_bits_t *mbits, uint32_t *ptindex,
                    ptl_process_t *rank, int device);
/* Same with DEVICE pointers (GPU engine only: a user plugin cannot run on
 * device memory, so this fails unless dht->hashfn == pdht_hash). */
int pdht_hash_batch_dev(pdht_t *dht, const void *keys, size_t n,
                        ptl_match_bits_t *mbits, uint32_t *ptindex,
                        ptl_process_t *rank, uint64_t *rank_hist,
                        void *stream);

#ifdef __cplusplus
}
#endif
#endif /* PDHT_HIP_HASH_H_ */
