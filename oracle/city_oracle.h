/*
 * city_oracle.h -- CPU restatement of pdht's CityHash path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle: tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may call it as the *checker*.
 * Nothing in pdht_amd/ (the product) links, loads or calls it.
 *
 * It restates, function by function, the algorithm of the reference files
 *   /root/reference/libpdht/city.c     (CityHash v1.0.x, Nusov C port)
 *   /root/reference/libpdht/citycrc.h  (CRC variants, SSE4.2 only)
 *   /root/reference/libpdht/hash.c     (pdht_hash placement)
 * and is pinned by the JSON fixtures in tests/golden/, which were produced by compiling the
 * reference city.c itself (oracle/Makefile -> oracle/_ref/).
 */
#ifndef PDHT_CITY_ORACLE_H
#define PDHT_CITY_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- scalar hashes (city.h:68-84, citycrc.h:39-46) ---------------------- */
uint64_t oracle_city64(const uint8_t *s, size_t len);
uint64_t oracle_city64_seed(const uint8_t *s, size_t len, uint64_t seed);
uint64_t oracle_city64_seeds(const uint8_t *s, size_t len, uint64_t seed0,
                             uint64_t seed1);
/* out[0] = uint128.first (low), out[1] = uint128.second (high) */
void oracle_city128(const uint8_t *s, size_t len, uint64_t out[2]);
void oracle_city128_seed(const uint8_t *s, size_t len, uint64_t seed_lo,
                         uint64_t seed_hi, uint64_t out[2]);
void oracle_citycrc128(const uint8_t *s, size_t len, uint64_t out[2]);
void oracle_citycrc128_seed(const uint8_t *s, size_t len, uint64_t seed_lo,
                            uint64_t seed_hi, uint64_t out[2]);
void oracle_citycrc256(const uint8_t *s, size_t len, uint64_t out[4]);
/* _mm_crc32_u64 semantics (CRC-32C, no pre/post inversion). */
uint64_t oracle_crc32c_u64(uint64_t crc, uint64_t v);

/* ---- pdht_hash restatement (libpdht/hash.c:25-30) ------------------------ */
void oracle_pdht_hash(const void *key, unsigned keysize, unsigned nptes,
                      int nranks, uint64_t *mbits, uint32_t *ptindex,
                      uint32_t *rank);

/* ---- batch helpers (loops over the scalar functions) --------------------- */
void oracle_city64_fixed(const uint8_t *keys, size_t stride, size_t len,
                         size_t n, uint64_t *out);
void oracle_city64_var(const uint8_t *bytes, const uint64_t *offsets, size_t n,
                       uint64_t *out);
void oracle_city128_fixed(const uint8_t *keys, size_t stride, size_t len,
                          size_t n, uint64_t *out /* 2n */);
void oracle_citycrc128_fixed(const uint8_t *keys, size_t stride, size_t len,
                             size_t n, uint64_t *out /* 2n */);
void oracle_city128_var(const uint8_t *bytes, const uint64_t *offsets, size_t n,
                        uint64_t *out /* 2n */);
void oracle_citycrc128_var(const uint8_t *bytes, const uint64_t *offsets,
                           size_t n, uint64_t *out /* 2n */);
void oracle_pdht_hash_fixed(const uint8_t *keys, unsigned keysize, size_t n,
                            unsigned nptes, int nranks, uint64_t *mbits,
                            uint32_t *ptindex, uint32_t *rank);

/* Position-weighted fold checksum  sum_i d_i * (2i+1)  mod 2^64. */
uint64_t oracle_fold64(const uint64_t *d, size_t n, uint64_t first_index);

/* ---- synthetic workload ---------------------------------- */
/* out[w] = splitmix64 output number (start + w) of the stream seeded `seed`. */
void oracle_splitmix64_fill(uint64_t seed, uint64_t start, size_t nwords,
                            uint64_t *out);

/* ---- CPU timing harness (bench.py cpu_baseline) -------------------------- */
typedef uint64_t (*oracle_city64_fn)(const char *s, size_t len);
/* Hash n fixed-length keys `reps` times over `threads` pthreads (contiguous
 * slices), through `fn` (the reference CityHash64 or oracle_city64_c).
 * Returns wall seconds (CLOCK_MONOTONIC_RAW) of the whole run; writes the
 * digests of the last rep to out. */
double oracle_time_city64(oracle_city64_fn fn, const uint8_t *keys, size_t len,
                          size_t n, int threads, int reps, uint64_t *out);
uint64_t oracle_city64_c(const char *s, size_t len);

/* Apply an external CityHash64 / CityHash128-shaped function (e.g. the
 * reference's, loaded from oracle/_ref) over a batch with `threads` pthreads.
 * offsets == NULL: fixed-length keys at `stride`, `len` bytes each;
 * otherwise key i = bytes[offsets[i], offsets[i+1]). */
typedef struct {
  uint64_t first, second;
} oracle_u128;
typedef oracle_u128 (*oracle_city128_fn)(const char *s, size_t len);
void oracle_apply64(oracle_city64_fn fn, const uint8_t *bytes,
                    const uint64_t *offsets, size_t stride, size_t len,
                    size_t n, uint64_t *out, int threads);
void oracle_apply128(oracle_city128_fn fn, const uint8_t *bytes,
                     const uint64_t *offsets, size_t stride, size_t len,
                     size_t n, uint64_t *out /* 2n */, int threads);

/* The product's pdht_hashfunc driven over a batch (tests: cfg1). */
typedef void (*oracle_hashfunc)(void *dht, void *key, uint64_t *mbits, uint32_t *ptindex,
                                void *rank);
void oracle_apply_hashfn(oracle_hashfunc fn, void *dht, const uint8_t *keys, size_t keysize,
                         size_t n, uint64_t *mbits, uint32_t *ptindex, uint64_t *rank8);
/* CPU baseline harness (bench.py): mode 0 = 64-bit digest, 1 = 128-bit,
 * 2 = pdht_hash semantics (digest + both reductions). */
double oracle_time_batch(int mode, void *fn, const uint8_t *bytes, const uint64_t *offsets,
                         size_t stride, size_t len, size_t n, int threads, int reps,
                         uint64_t nptes, uint64_t nranks, uint64_t *out, uint32_t *pt,
                         uint32_t *rk);
/* CPU baseline of destination bucketing (bench.py bucket / records): hash,
 * count per rank, stable scatter -- the same outputs as the GPU bucketing. */
double oracle_time_bucket(oracle_city64_fn fn, const uint8_t *keys, size_t L, size_t n, int threads,
                          int reps, uint64_t nptes, uint32_t nranks, int records, uint32_t src,
                          uint32_t ht, uint64_t *mb, uint32_t *rk, uint32_t *hist, uint8_t *keys_out,
                          uint64_t *mbits_out, uint32_t *pt_out, uint32_t *idx_out, uint8_t *rec_out,
                          uint64_t *offsets);

#ifdef __cplusplus
}
#endif
#endif
