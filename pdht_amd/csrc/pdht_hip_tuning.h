/*
 * pdht_hip_tuning.h -- extra entry points of the TUNING build only
 * (pdht_amd/lib/libpdht_hip_tuning.so, compiled with -DPDHT_HIP_TUNING from
 * the same sources as the product).  Used by tools/ and the A/B tests; not
 * part of the drop-in boundary (include/), and not exported by the product
 * library libpdht_hip.so.
 */
#ifndef PDHT_HIP_TUNING_H_
#define PDHT_HIP_TUNING_H_

#ifdef __cplusplus
extern "C" {
#endif

/* Select an alternative kernel where one exists (0 = the product's choice):
 *   64-B keys  7 one tile of prefetch per wave, 4 WG/CU; 26 plain digest stores
 *   var keys  12 10224-B window at 4 WG/CU;   13 16 KiB window at 2 WG/CU
 *   bucketing 21 generic-length scatter;      22 register scatter
 *   host      61 chunked copy pipeline instead of zero-copy on pinned buffers
 * Process-wide; returns the previous value. */
int pdht_hip_set_variant(int variant);
/* Override the workgroups per CU of the persistent grids (0 = default).
 * Returns the previous value. */
int pdht_hip_set_blocks_per_cu(int per_cu);

#ifdef __cplusplus
}
#endif
#endif /* PDHT_HIP_TUNING_H_ */
