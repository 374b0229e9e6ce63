// runtime.h -- what the C-ABI translation units share (pdht_hip.hip defines
// it): the per-thread error and kernel-tag strings, per-device state, grid
// sizing, the invariant-divisor setup and the placement checks.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/pdht_hip.h"
#include "kernels.h"

#define PDHT_API extern "C" __attribute__((visibility("default")))
#define ST(s) reinterpret_cast<hipStream_t>(s)

namespace pdht {

// ------------------------------------------------------------- errors ---
// The calling thread's last error (pdht_hip_last_error) and the tag of the
// kernel its last batch call launched (pdht_hip_last_kernel).
extern thread_local char g_err[512];
extern thread_local const char *g_kernel;
int fail(const char *fmt, const char *a = "", long long b = 0);
#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return fail("%s (" #expr ")", hipGetErrorString(e_)); \
  } while (0)

}  // namespace pdht

// A/B hook points (product/pdht_hooks.h: in the product libraries every hook
// is "not taken" -- one measured-best kernel per path, no process-global
// mutable state, no environment knobs; tuning/pdht_hooks.h in
// libpdht_hip_tuning.so, for tools/ and the A/B tests).
#include "pdht_hooks.h"

namespace pdht {

// ------------------------------------------------------- device state ---
constexpr int kMaxDev = 64;
struct DevInfo {
  std::once_flag once;
  int cus = 0;
  hipError_t err = hipSuccess;
};
extern DevInfo g_dev[kMaxDev];
int current_device(int *dev);

// Persistent grid: enough workgroups to keep every CU at `per_cu` blocks,
// never more than the work needs.
unsigned grid_for(u64 work_blocks, int per_cu, int dev);

FastMod make_fastmod(u64 d);

// pdht_hash placement (hash.c:25-30) as a kernel sink, and its argument checks.
SinkPlace make_place_sink(u64 *mbits, u32 *ptindex, void *rank, size_t rank_stride, u64 *hist, u32 nptes,
                          u32 nranks);
int check_place(size_t n, const u64 *mbits, u32 nptes, u32 nranks, const void *rank, size_t rank_stride);

}  // namespace pdht
