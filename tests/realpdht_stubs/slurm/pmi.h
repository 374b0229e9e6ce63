/* TEST-ONLY compile stub of <slurm/pmi.h> (absent from this image); the
 * reference's pdht.h includes it but its declarations use nothing from it. */
#ifndef PDHT_TEST_STUB_SLURM_PMI_H
#define PDHT_TEST_STUB_SLURM_PMI_H
#endif
