/* TEST-ONLY compile stub of <portals4.h> (absent from this image): just the
 * types the reference's pdht.h / pdht_impl.h declare their structs with, so
 * that tests/test_product_cpu.py can compile pdht_amd/host/pdht_hash.c's
 * -DPDHT_HIP_WITH_REAL_PDHT branch against the real pdht headers.  Nothing
 * is linked or run.  ptl_process_t follows the Portals 4 spec layout (a union
 * of {nid, pid} and rank, 32-bit members): the stride the batch writes. */
#ifndef PDHT_TEST_STUB_PORTALS4_H
#define PDHT_TEST_STUB_PORTALS4_H
#include <stdint.h>
typedef uint64_t ptl_size_t;
typedef uint64_t ptl_match_bits_t;
typedef uint32_t ptl_nid_t;
typedef uint32_t ptl_pid_t;
typedef uint32_t ptl_rank_t;
typedef uint32_t ptl_pt_index_t;
typedef union {
  struct {
    ptl_nid_t nid;
    ptl_pid_t pid;
  } phys;
  ptl_rank_t rank;
} ptl_process_t;
typedef struct { void *h; } ptl_handle_ni_t;
typedef struct { void *h; } ptl_handle_md_t;
typedef struct { void *h; } ptl_handle_me_t;
typedef struct { void *h; } ptl_handle_ct_t;
typedef struct { void *h; } ptl_handle_eq_t;
typedef struct { ptl_size_t success, failure; } ptl_ct_event_t;
typedef struct { int max_entries; } ptl_ni_limits_t;
typedef struct { void *start; ptl_size_t length; ptl_match_bits_t match_bits, ignore_bits; } ptl_me_t;
typedef int ptl_event_kind_t;
typedef struct { ptl_event_kind_t type; } ptl_event_t;
#define PTL_PT_MATCH_UNORDERED 1
#endif
