/*
 * pdht_hip_tuning.h -- extra entry points of the TUNING build only
 * (pdht_amd/lib/libpdht_hip_tuning.so: the same sources as the product,
 * compiled with the A/B hook headers of pdht_amd/csrc/tuning/ instead of
 * pdht_amd/csrc/product/, plus tuning/pdht_tuning.hip).  Used by tools/ and the A/B tests; not
 * part of the drop-in boundary (include/), and not exported by the product
 * library libpdht_hip.so.
 */
#ifndef PDHT_HIP_TUNING_H_
#define PDHT_HIP_TUNING_H_

#ifdef __cplusplus
extern "C" {
#endif

/* Select an alternative kernel where one exists (0 = the product's choice).
 * The alternatives live in pdht_amd/csrc/tuning/ (kernels_tuning.h and the
 * pdht_hooks*.h headers the sources' hook points resolve to in this build);
 * the product sources and headers hold only what ships.  Every variant the sources know (DESIGN.md
 * §4 has the measurements):
 *   64-B keys      7  one tile of prefetch per wave, 4 WG/CU (r01: 2-5 % slower)
 *                 26  plain instead of non-temporal digest stores (2-6 % slower)
 *                188  digests stored 16 B per lane (even lanes, DPP pairs: Sink64x2T)
 *                206  s_setprio 1 around each wave's prefetch issue
 *              80/81  1024-thread transpose at 1 / 2 WG/CU (cfg1 shape)
 *                 82  the 256-thread transpose whatever the histogram
 *            250/251  tile order scattered (bijection) / per-wave contiguous runs
 *   long keys     96  r02 spans before the 128-B line spans (240-B / 64-B)
 *                153  timing only: CRC lookups replaced by a fold (wrong digests)
 *                150  CRC-32C on r02's 6-bit-slice tables (product: byte tables)
 *                303  CRC-32C on 11-bit-slice tables (6 lookups per word, 42 KiB)
 *            279-281  CRC long keys of 1024 / 2048 / 4096 B through an LDS-DMA ring of
 *                     R = 4 / 2 / 3 coalesced line-rounds per wave (k_long_ring)
 *            190/191  CityHashCrc256Long's block loop as a 128-B line stream
 *                     (kLongStream), 8 / 4 WG/CU
 *   var keys      12  10224-B window at 4 WG/CU;  13 16 KiB window at 2 WG/CU
 *                252  workgroup-combined digest stores (4 consecutive tiles, 2 KiB runs)
 *            170-173  CityHash64: k_window_pipe (offsets a tile ahead, digests a tile
 *                     late, vmcnt(2)): G = 1 / 4 / 16 consecutive tiles per wave at
 *                     4 WG/CU; 173 = G 1 at 3 WG/CU; 174 = G 1 / 175 = the product
 *                     window kernel with the r03 funnel reader (dword runs +
 *                     v_alignbyte_b32; product since r04: unaligned ds_read_b128)
 *   calibration 40-45 (pdht_hip_key_stream_var_dev) the window kernel's data
 *                     movement alone (digest = key length): 40 as shipped,
 *                     41 default-policy DMA, 42 plain stores, 43 3 WG/CU,
 *                     44/45 windows on 128-B lines
 *           110 / 111 (same entry) the window kernel hashing every key twice
 *                     / once: what the arithmetic costs over 40
 *                189  CityHash64 window kernel with 16-B-per-lane digest stores
 *            203/204  CityHash64 window kernel, s_setprio 3 / 1 while fetching
 *                205  variable-length window kernel without s_setprio (product: 1)
 *            180-187  k_window_pipe G1 cache policies (DMA / digest stores): nt / plain,
 *                     nt / sc0, nt / sc1, nt / sc1|nt, nt / sc0|sc1|nt, plain / nt,
 *                     sc0|nt / nt, sc1 / nt
 *            176-179  (same entry) k_window_pipe: length-only with stores / into a
 *                     32 KiB ring; CityHash64 with stores / into the ring
 *       119-121, 125  (same entry) keys read as fixed rows of the mean length,
 *                     no offsets: nt / no / plain digest stores / plain stores
 *                     into 32 KiB (L2-resident)
 *   cfg3 path 140-144 (pdht_city64_batch_var_dev) digests wrapped into 32 KiB
 *                     / 2 / 8 / 32 / 128 MiB of out (wrong digests: where the
 *                     writes land)
 *   launches  114-118 key bytes per launch: 256 MiB / 1 GiB / 2 GiB / 4 GiB /
 *                     all in one launch (product: 512 MiB)
 *   bucketing     21  generic-length scatter for 8/16/32-B keys
 *                 70  one pass (staged scatter) up to 2048 ranks
 *                 71  two passes from 2 ranks up
 *              83/87  owner-table ranking on 8 x 16 / 4 x 16 tiles, any nranks
 *              85/89  ballot ranking, any nranks (85: static tile order)
 *                202  the r02-r03 two-pass sub-tile shape (4 x 8 @ 4 for both passes,
 *                     pass 2 storing in two phases); r04's other shapes (192-201), r05's
 *                     LDS-DMA pipelined passes, packed pass-1 tables and prefetching
 *                     count kernel (230-242), higher-occupancy shapes (253-259) and 8-B
 *                     arrays in 4 keys per lane (273-276) were
 *                     measured slower and removed
 *                264  fine counts column-scanned over 32-tile chunks (k_bucket_colscan,
 *                     r02-r05; product: the count kernel scans down its own chunk)
 *            265/266  8-B arrays' pass 2 as r04-r05 shipped it (two store phases, 4x8@4) /
 *                     one store phase in 4x8@4 (product: one phase, 8x8@2)
 *            267-269  16/32-B keys' two passes: 8x4@2 both / pass 2 4x4@4 / pass 1 4x8@4,
 *                     pass 2 8x4@2 (product: 32-B arrays 267, 16/32-B records 268)
 *                270  16/32-B keys' two passes as r04-r05 shipped them (spilling)
 *            271/272  8-B records' pass 2 in 4x4@4 / 4x8@4 (r04-r05; product 8x4@2)
 *                290  the r02-r05 two-pass form (counting kernel + fine-count scans
 *                     ahead of pass 1, pass 1 writing global fine-bucket runs) instead
 *                     of the tile-local one (r06); 202 and 264-272 imply it
 *            291-293  tile-local two passes: pass 2 in 4x8@4 / 8x4@2; pass 1 in
 *                     16 waves @ 1 on the product's tiles (1024 threads) (8/16-B keys)
 *            294/295  tile-local pass 1 on 8192-key tiles (16x8@1), pass-2 gathers of
 *                     runs twice as long (8/16-B keys); 295 on the balanced digit split
 *                304  16-B keys' tile-local pass 2 in r06's first shapes (arrays 8x8@2,
 *                     records 4x4@4)
 *                305  32-B records' tile-local pass 2 in 8x4@2
 *                323  8-B arrays' tile-local pass 2 storing in two phases (not ONE)
 *                322  tile-local pass 1 loading its keys with plain (temporal) loads
 *                321  the staged scatter loading its keys non-temporally (before r06)
 *                320  tile-local pass 2's gather in the other load policy (non-temporal;
 *                     32-B records temporal)
 *            316-319  tile-local pass-2 segments in blocks of og fine buckets x os
 *                     segments: 8x8, 16x4, 32x2, 4x16
 *                298  timing probe: tile-local pass 2 reading contiguous rows instead of
 *                     gathering its f-runs (wrong outputs; 8/16-B keys)
 *                302  tile-local, 16-B keys: pass 1 in 8x8 (4096-key tiles; spills 23 VGPRs,
 *                     0.4-1.9 % slower than the product's 8x4)
 *            296/297  tile-local pass-2 segments in chunk-range-major order (the
 *                     workgroups of an XCD gather neighbouring f-runs of the same tiles);
 *                     297 with 294's 8192-key tiles
 *                164  two-pass arrays of 8/16-B keys on the balanced digit split
 *                     F = 2^ceil(nbits/2) (product: one fine bit more)
 *   records      112  r02 store order (header halves a staging round early)
 *   host          61  chunked copy pipeline instead of zero-copy on pinned buffers
 *   small keys   219  8-B placement with a histogram, 4 keys per lane (the shape
 *                     before late r04; product: 8); 220 16 keys per lane
 *            221-223  8-B hashing: plain loads (the shape before late r04; product:
 *                     non-temporal) / 8 keys per lane / 8 keys per lane, 1024 threads @1
 *                224  32-B keys with plain loads and stores (product: non-temporal)
 *           225, 226  16-B keys, 4 keys per lane in flight: placement with a histogram
 *                     (1024 threads @2) / hashing (@8) (product: 2)
 * Process-wide; returns the previous value. */
int pdht_hip_set_variant(int variant);
/* Override the workgroups per CU of the persistent grids (0 = default).
 * Returns the previous value. */
int pdht_hip_set_blocks_per_cu(int per_cu);

#ifdef __cplusplus
}
#endif
#endif /* PDHT_HIP_TUNING_H_ */
