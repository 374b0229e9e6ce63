/*
 * pdht_hip.h -- C-ABI of the MI355X batch key-hashing engine.
 *
 * The reference hashes one key per call on the initiator CPU
 * (dht->hashfn -> pdht_hash -> CityHash64, libpdht/putget.c:53,
 * libpdht/hash.c:25-30).  This header adds the batch entry points a caller
 * (a bulk loader such as bench/Meraculous/buildUFXhashBinary.h:83-112, or
 * pdht_hash_batch in pdht_hash.h) binds to hash many keys at once on a GPU.
 * Plain pointers and sizes only: no HIP or torch types appear, a stream is an
 * opaque pointer (a hipStream_t may be passed; NULL = the default stream).
 *
 * Every function returns 0 (== PdhtStatusOK, libpdht/pdht.h:178-184) on
 * success and PDHT_HIP_ERROR (== PdhtStatusError) otherwise; the reason is
 * kept per thread in pdht_hip_last_error().  Nothing here falls back to the
 * CPU: with no usable GPU the batch calls fail.
 *
 * Digest layouts: 64-bit digests are one uint64 per key; 128-bit digests are
 * two uint64 per key, {first (low), second (high)} exactly as the
 * reference's uint128 (city.h:58-65).
 *
 * Key layouts:
 *   fixed  -- key i occupies bytes [i*stride, i*stride + keylen) of `keys`
 *             (stride >= keylen; stride == keylen for packed keys);
 *   var    -- key i occupies bytes [offsets[i], offsets[i+1]) of `bytes`;
 *             offsets has n+1 non-decreasing entries.
 */
#ifndef PDHT_HIP_H_
#define PDHT_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDHT_HIP_OK 0
#define PDHT_HIP_ERROR 1 /* == PdhtStatusError */
/* ABI revision of this header; pdht_hip_version() names the same number
 * ("abi 4").  Revision 2 changed index_out to uint32_t, gave
 * pdht_bucket_workspace_bytes its keysize and the *_var_dev entry points
 * their nbytes; revision 4 sizes the workspace of pdht_bucket_records_dev by
 * pdht_bucket_records_workspace_bytes (array callers no longer reserve the
 * records' two-pass region): a caller built against an older header must be
 * rebuilt. */
#define PDHT_HIP_ABI_VERSION 4

typedef struct ihipStream_t *pdht_hip_stream_t; /* layout of hipStream_t */

/* ---- runtime ------------------------------------------------------------ */
const char *pdht_hip_version(void);
/* Last error message of the calling thread ("" if none). */
const char *pdht_hip_last_error(void);
/* Number of visible GPUs (0 on a host without one; still returns OK). */
int pdht_hip_device_count(int *count);
/* Make `device` current for the calling thread (hipSetDevice) and
 * initialise its per-device state once. */
int pdht_hip_set_device(int device);

/* ---- device-resident batches (all pointers are device pointers) --------- */
/* CityHash64 (city.h:68) over fixed-length keys. */
int pdht_city64_batch_dev(const void *keys, size_t stride, size_t keylen,
                          size_t n, uint64_t *out, pdht_hip_stream_t stream);
/* CityHash64WithSeeds (city.h:76); CityHash64WithSeed(s) == seeds(k2, s). */
int pdht_city64_seeds_batch_dev(const void *keys, size_t stride, size_t keylen,
                                size_t n, uint64_t seed0, uint64_t seed1,
                                uint64_t *out, pdht_hip_stream_t stream);
/* CityHash64 over variable-length keys.  nbytes = key bytes the batch spans
 * (offsets[n] - offsets[0]; 0 if unknown): it sizes the kernel's LDS window
 * for the mean key length and is never used to address memory. */
int pdht_city64_batch_var_dev(const void *bytes, size_t nbytes,
                              const uint64_t *offsets, size_t n, uint64_t *out,
                              pdht_hip_stream_t stream);
/* CityHash128 (city.h:80): out[2i] = first, out[2i+1] = second. */
int pdht_city128_batch_dev(const void *keys, size_t stride, size_t keylen,
                           size_t n, uint64_t *out, pdht_hip_stream_t stream);
/* CityHash128WithSeed (city.h:84). */
int pdht_city128_seed_batch_dev(const void *keys, size_t stride, size_t keylen,
                                size_t n, uint64_t seed_lo, uint64_t seed_hi,
                                uint64_t *out, pdht_hip_stream_t stream);
int pdht_city128_batch_var_dev(const void *bytes, size_t nbytes,
                               const uint64_t *offsets, size_t n, uint64_t *out,
                               pdht_hip_stream_t stream);
/* CityHashCrc128 (citycrc.h:39). */
int pdht_citycrc128_batch_dev(const void *keys, size_t stride, size_t keylen,
                              size_t n, uint64_t *out,
                              pdht_hip_stream_t stream);
/* CityHashCrc128WithSeed (citycrc.h:43). */
int pdht_citycrc128_seed_batch_dev(const void *keys, size_t stride,
                                   size_t keylen, size_t n, uint64_t seed_lo,
                                   uint64_t seed_hi, uint64_t *out,
                                   pdht_hip_stream_t stream);
int pdht_citycrc128_batch_var_dev(const void *bytes, size_t nbytes,
                                  const uint64_t *offsets, size_t n,
                                  uint64_t *out, pdht_hip_stream_t stream);

/* Fused placement = pdht_hash (libpdht/hash.c:25-30) over a batch of packed
 * keysize-byte keys:
 *   mbits[i]   = CityHash64(key_i, keysize)
 *   ptindex[i] = mbits[i] % nptes                 (skipped if ptindex NULL)
 *   rank_i     = mbits[i] % nranks, stored as a uint32 at
 *                (char*)rank + i*rank_stride       (skipped if rank NULL;
 *                rank_stride 8 writes the .rank member of a ptl_process_t
 *                array, 4 a dense uint32 array)
 *   hist[r]   += number of keys placed on rank r  (skipped if hist NULL;
 *                nranks uint64 counters, accumulated, not cleared) -- the
 *                rankputs[] statistic of putget.c:55 / util.c:386-397. */
int pdht_place_batch_dev(const void *keys, size_t keysize, size_t n,
                         uint32_t nptes, uint32_t nranks, uint64_t *mbits,
                         uint32_t *ptindex, void *rank, size_t rank_stride,
                         uint64_t *hist, pdht_hip_stream_t stream);

/* Destination bucketing (the shape of the Meraculous
 * loader, bench/Meraculous/buildUFXhashBinary.h:83-112): a stable counting
 * sort of n packed keysize-byte keys by rank = CityHash64 % nranks.  Bucket
 * r occupies positions [bucket_offsets[r], bucket_offsets[r+1]) of the
 * outputs, keys in their original order; bucket_offsets has nranks+1
 * entries.  Outputs at bucketed positions: mbits_out (required),
 * keys_out (keysize bytes per key), ptindex_out (% nptes), index_out
 * (original key index, uint32: n < 2^32) -- each optional (NULL): a caller
 * holding index_out can gather keys itself and pass keys_out = NULL; with
 * nptes == 1 (pdht's default, pdht_impl.h:41) every ptindex is 0 and
 * ptindex_out is best NULL.  nranks <= 8192, n < 2^32.  `workspace`
 * (device) must hold pdht_bucket_workspace_bytes(n, keysize, nranks): the
 * per-tile counts and, for 8/16/32-B keys at the rank counts that take the
 * two-pass sort (from 1575 / 1575 / 2049 ranks for 8 / 16 / 32-B keys), its
 * intermediate (about n x (keysize + 2) bytes). */
size_t pdht_bucket_workspace_bytes(size_t n, size_t keysize, uint32_t nranks);
int pdht_bucket_batch_dev(const void *keys, size_t keysize, size_t n,
                          uint32_t nptes, uint32_t nranks, void *workspace,
                          size_t workspace_bytes, void *keys_out,
                          uint64_t *mbits_out, uint32_t *ptindex_out,
                          uint32_t *index_out, uint64_t *bucket_offsets,
                          pdht_hip_stream_t stream);

/* The same bucketing, written as one wire record per key instead of separate
 * arrays: the MPI variant's request message (message_t,
 * libmpipdht/pdht.h:120-127, filled by pdht_put at libmpipdht/putget.c:85-97)
 * with the key as payload, so that bucket r is a ready send buffer for rank
 * r.  Record at bucketed position p, stride pdht_bucket_record_bytes(keysize)
 * = 24 + keysize rounded up to 8:
 *   +0  uint32 type      = msg_type (pdhtPut = 1 in the reference's enum)
 *   +4  uint32 rank      = src_rank (the sender, c->rank)
 *   +8  uint32 ht_index  = ht_index (the table's index, c->hts[])
 *   +12 uint32 index     = original position of the key in the batch
 *                          (message_t's alignment padding)
 *   +16 uint64 mbits     = CityHash64(key)
 *   +24 key[keysize], zero-padded to the stride.
 * records (device, 8-byte aligned) holds n records; bucket_offsets as for
 * pdht_bucket_batch_dev, the workspace sized by
 * pdht_bucket_records_workspace_bytes.  ptindex is not stored (it is
 * mbits % nptes; the MPI message carries ht_index instead). */
size_t pdht_bucket_record_bytes(size_t keysize);
/* Workspace of pdht_bucket_records_dev: as pdht_bucket_workspace_bytes, with
 * the records' two-pass thresholds (from 2048 / 1463 / 256 ranks for 8 / 16 /
 * 32-B keys). */
size_t pdht_bucket_records_workspace_bytes(size_t n, size_t keysize, uint32_t nranks);
int pdht_bucket_records_dev(const void *keys, size_t keysize, size_t n,
                            uint32_t nranks, uint32_t msg_type, uint32_t src_rank,
                            uint32_t ht_index, void *workspace,
                            size_t workspace_bytes, void *records,
                            uint64_t *bucket_offsets, pdht_hip_stream_t stream);

/* ---- host-resident batches ---------------------------------------------- */
/* Keys and digests in host memory.  Chunks are copied H2D, hashed and copied
 * back D2H on several streams so copies and kernels overlap; pinned
 * (hipHostMalloc / registered) buffers are DMA'd directly, pageable ones go
 * through pinned staging.  Blocking: returns when `out` is complete. */
int pdht_city64_batch_host(const void *keys, size_t keylen, size_t n,
                           uint64_t *out, int device);
int pdht_city64_batch_var_host(const void *bytes, const uint64_t *offsets,
                               size_t n, uint64_t *out, int device);
int pdht_citycrc128_batch_host(const void *keys, size_t keylen, size_t n,
                               uint64_t *out, int device);
int pdht_place_batch_host(const void *keys, size_t keysize, size_t n,
                          uint32_t nptes, uint32_t nranks, uint64_t *mbits,
                          uint32_t *ptindex, void *rank, size_t rank_stride,
                          int device);

/* ---- synthetic workloads (benchmarks/tests) ----------------------------- */
/* out[w] = splitmix64 output number (first + w) of the stream seeded `seed`:
 * z = seed + (first+w+1)*0x9e3779b97f4a7c15, then the splitmix64 finaliser. */
int pdht_hip_splitmix64_fill_dev(uint64_t seed, uint64_t first, size_t nwords,
                                 uint64_t *out, pdht_hip_stream_t stream);
/* lens[i] = lo + splitmix64(seed)[first+i] % (hi - lo + 1) */
int pdht_hip_mixed_lengths_dev(uint64_t seed, uint64_t first, size_t n,
                               uint32_t lo, uint32_t hi, uint64_t *lens,
                               pdht_hip_stream_t stream);

/* ---- introspection and calibration -------------------------------------- */
/* Tag of the kernel (and launch shape) the last batch call on this thread
 * launched, e.g. "k_fixed_xpose64<nt,d2>@3" (3 workgroups per CU). */
const char *pdht_hip_last_kernel(void);
/* HBM calibration: stream `bytes` (multiple of 16, 16-B aligned) through a
 * read-only kernel with 16-B coalesced loads (nt != 0: non-temporal) and
 * XOR-fold them into *out (one uint64, device).  Gives the achievable read
 * bandwidth the hash kernels are compared with. */
int pdht_hip_read_stream_dev(const void *buf, size_t bytes, int nt, uint64_t *out,
                             pdht_hip_stream_t stream);
/* Key-stream calibration: n packed 64-B keys (16-B aligned) -> out[n], each
 * digest an XOR fold of the key's bytes, moved exactly as the default 64-B
 * CityHash64 kernel moves them (same loads, LDS transpose, stores, grid).
 * The hash kernel's time minus this one is what the hash arithmetic costs. */
int pdht_hip_key_stream_dev(const void *keys, size_t n, uint64_t *out, pdht_hip_stream_t stream);
/* The same for offset-indexed keys: the variable-length kernel's window DMA,
 * offsets reads, LDS reads of every key byte and digest stores, with the hash
 * replaced by an XOR fold (out[i] = fold of key i; see tests). */
int pdht_hip_key_stream_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets, size_t n,
                                uint64_t *out, pdht_hip_stream_t stream);
#ifdef __cplusplus
}
#endif
#endif /* PDHT_HIP_H_ */
