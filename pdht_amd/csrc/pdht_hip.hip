// pdht_hip.hip -- C-ABI of the batch key-hashing engine (include/pdht_hip.h):
// the shared runtime (runtime.h), the runtime entry points, the synthetic
// workload generators and the calibration kernels.  The hash entry points
// live in pdht_fixed64.hip / pdht_fixed128.hip (fixed-length keys),
// pdht_var.hip (variable-length keys), pdht_host.hip (host-resident
// batches) and pdht_bucket.hip (destination bucketing).  Kernels: kernels.h,
// bucket.h.  Algorithm: city_core.h.
#include "runtime.h"

namespace pdht {

// ------------------------------------------------------------- errors ---
thread_local char g_err[512] = "";
thread_local const char *g_kernel = "";

int fail(const char *fmt, const char *a, long long b) {
  snprintf(g_err, sizeof g_err, fmt, a, b);
  return PDHT_HIP_ERROR;
}

// ------------------------------------------------------- device state ---
DevInfo g_dev[kMaxDev];

int current_device(int *dev) {
  HIP_TRY(hipGetDevice(dev));
  if (*dev < 0 || *dev >= kMaxDev) return fail("device index %s%lld out of range", "", *dev);
  DevInfo &d = g_dev[*dev];
  std::call_once(d.once, [&] {
    d.err = hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, *dev);
  });
  if (d.err != hipSuccess) return fail("%s (querying CU count)", hipGetErrorString(d.err));
  return 0;
}

unsigned grid_for(u64 work_blocks, int per_cu, int dev) {
  per_cu = hook_per_cu(per_cu);
  const u64 cap = (u64)std::max(1, g_dev[dev].cus) * per_cu;
  return (unsigned)std::max<u64>(1, std::min<u64>(work_blocks, cap));
}

FastMod make_fastmod(u64 d) {
  FastMod f{};
  f.d = d;
  if ((d & (d - 1)) == 0) {  // includes d == 1 (mask 0)
    f.pow2 = 1;
    return f;
  }
  u32 l = 64 - __builtin_clzll(d - 1);  // ceil(log2 d), 2..64
  unsigned __int128 num = ((unsigned __int128)(((unsigned __int128)1 << l) - d)) << 64;
  f.m = (u64)(num / d) + 1;
  f.sh = l - 1;
  f.pow2 = 0;
  return f;
}

// --------------------------------------------------------- launchers ---

SinkPlace make_place_sink(u64 *mbits, u32 *ptindex, void *rank, size_t rank_stride,
                                 u64 *hist, u32 nptes, u32 nranks) {
  SinkPlace s{};
  s.mbits = mbits;
  s.ptindex = ptindex;
  s.rank = static_cast<uint8_t *>(rank);
  s.rank_stride = rank_stride;
  s.hist = hist;
  s.pt = make_fastmod(nptes);
  s.rk = make_fastmod(nranks);
  s.nranks = nranks;
  return s;
}

int check_place(size_t n, const u64 *mbits, u32 nptes, u32 nranks, const void *rank,
                       size_t rank_stride) {
  if (n && !mbits) return fail("mbits must not be NULL%s", "");
  if (nptes == 0) return fail("nptes must be >= 1 (hash.c:27 divides by it)%s", "");
  if (nranks == 0) return fail("nranks must be >= 1 (hash.c:29 divides by it)%s", "");
  if (nranks > 0x7fffffffu) return fail("nranks is c->size, an int: must be < 2^31%s", "");
  if (rank && rank_stride < 4) return fail("rank_stride must be >= 4%s", "");
  return 0;
}

}  // namespace pdht

using namespace pdht;

// ===================================================================== ABI ===
static_assert(PDHT_HIP_ABI_VERSION == 4, "bump the version string with the ABI");
PDHT_API const char *pdht_hip_version(void) { return "pdht-hip 0.4 (abi 4, gfx950, CityHash v1.0.x)"; }
PDHT_API const char *pdht_hip_last_error(void) { return g_err; }
PDHT_API const char *pdht_hip_last_kernel(void) { return g_kernel; }

PDHT_API int pdht_hip_device_count(int *count) {
  if (!count) return fail("null count%s", "");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e == hipErrorNoDevice) {
    (void)hipGetLastError();
    c = 0;
  } else if (e != hipSuccess) {
    *count = 0;
    return fail("%s (hipGetDeviceCount)", hipGetErrorString(e));
  }
  *count = c;
  return 0;
}

PDHT_API int pdht_hip_set_device(int device) {
  HIP_TRY(hipSetDevice(device));
  int dev;
  return current_device(&dev);
}

// ---------------------------------------------------- synthetic workloads ---
namespace pdht {
__device__ __forceinline__ u64 splitmix64_at(u64 seed, u64 k) {
  u64 z = seed + (k + 1) * 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(kBlock) void k_splitmix64(u64 seed, u64 first, u64 nwords, u64 *out) {
  const u64 stride = (u64)gridDim.x * kBlock;
  for (u64 w = (u64)blockIdx.x * kBlock + threadIdx.x; w < nwords; w += stride)
    out[w] = splitmix64_at(seed, first + w);
}
__global__ __launch_bounds__(kBlock) void k_mixed_lengths(u64 seed, u64 first, u64 n, u32 lo,
                                                          u32 span, u64 *lens) {
  const u64 stride = (u64)gridDim.x * kBlock;
  for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    lens[i] = lo + splitmix64_at(seed, first + i) % span;
}

// Read-only HBM stream (calibration), the same access shape as the hash
// kernels: a wave owns a contiguous 4 KiB tile = 4 wave-instructions of 1 KiB
// (16 B per lane); grid-stride over tiles, 2 workgroups per CU (the fastest
// read shape in tools/hbm_probe.hip: 7.0-7.2 TB/s with nt loads).
template <bool NT>
__global__ __launch_bounds__(kBlock) void k_read_stream(const u32x4 *__restrict__ p, u64 n16,
                                                        u64 *out) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  const u64 full = n16 >> 8;  // whole 4 KiB tiles
  u32x4 acc = {0, 0, 0, 0};
  for (u64 t = wave; t < full; t += nwaves) {
    const u32x4 *q = p + (t << 8) + lane;
    const u32x4 a = ld<NT>(q), b = ld<NT>(q + 64), c = ld<NT>(q + 128), d = ld<NT>(q + 192);
    acc ^= a ^ b ^ c ^ d;
  }
  for (u64 i = (full << 8) + wave * 64 + lane; i < n16; i += nwaves * 64) acc ^= ld<NT>(p + i);
  u64 v = ((u64)(acc.x ^ acc.z) << 32) | (acc.y ^ acc.w);
  for (int o = 32; o > 0; o >>= 1) v ^= __shfl_xor(v, o);
  // one atomic per workgroup: thousands of same-address atomics at the end of
  // the stream serialise in L2 and cost ~25 % of the launch (hbm_probe.hip)
  __shared__ u64 part[kWavesPerBlock];
  if (lane == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 b = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) b ^= part[w];
    atomicXor(reinterpret_cast<unsigned long long *>(out), b);
  }
}
}  // namespace pdht

PDHT_API int pdht_hip_read_stream_dev(const void *buf, size_t bytes, int nt, uint64_t *out,
                                      pdht_hip_stream_t s) {
  if (bytes == 0) return 0;
  if (!buf || !out || (bytes & 15) || ((uintptr_t)buf & 15)) return fail("bad buffer%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  const u64 n16 = bytes / 16;
  const unsigned g = grid_for(((n16 >> 8) + kWavesPerBlock) / kWavesPerBlock, 2, dev);
  const u32x4 *p = static_cast<const u32x4 *>(buf);
  if (nt)
    k_read_stream<true><<<g, kBlock, 0, ST(s)>>>(p, n16, out);
  else
    k_read_stream<false><<<g, kBlock, 0, ST(s)>>>(p, n16, out);
  HIP_TRY(hipGetLastError());
  return 0;
}

// Key-stream calibration: exactly the default 64-B kernel's data movement
// (k_fixed_xpose64, nt loads and stores, same grid) with the hash replaced by
// an XOR fold, so hash cost = kernel time - this time.
PDHT_API int pdht_hip_key_stream_dev(const void *keys, size_t n, uint64_t *out,
                                     pdht_hip_stream_t s) {
  if (n == 0) return 0;
  if (!keys || !out || ((uintptr_t)keys & 15)) return fail("bad buffer%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  Sink64T<true> sink{};
  sink.out = out;
  g_kernel = "k_fixed_xpose64<fold,nt,d2>@3";
  k_fixed_xpose64<AlgoFold64, Sink64T<true>, true, 2>
      <<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, ST(s)>>>(static_cast<const uint8_t *>(keys), n,
                                                                AlgoFold64{}, sink);
  HIP_TRY(hipGetLastError());
  return 0;
}

PDHT_API int pdht_hip_splitmix64_fill_dev(uint64_t seed, uint64_t first, size_t nwords,
                                          uint64_t *out, pdht_hip_stream_t s) {
  if (nwords == 0) return 0;
  if (!out) return fail("null out%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  k_splitmix64<<<grid_for((nwords + kBlock - 1) / kBlock, 8, dev), kBlock, 0, ST(s)>>>(seed, first,
                                                                                         nwords, out);
  HIP_TRY(hipGetLastError());
  return 0;
}

PDHT_API int pdht_hip_mixed_lengths_dev(uint64_t seed, uint64_t first, size_t n, uint32_t lo,
                                        uint32_t hi, uint64_t *lens, pdht_hip_stream_t s) {
  if (n == 0) return 0;
  if (!lens || hi < lo) return fail("bad arguments%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  k_mixed_lengths<<<grid_for((n + kBlock - 1) / kBlock, 8, dev), kBlock, 0, ST(s)>>>(
      seed, first, n, lo, hi - lo + 1, lens);
  HIP_TRY(hipGetLastError());
  return 0;
}
