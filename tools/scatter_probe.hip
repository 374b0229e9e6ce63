// scatter_probe.hip -- write-side ceiling of destination bucketing's store
// pattern (tuning tool, not product code).
//
// The bucketing scatter writes, per input tile, one run per bucket into every
// output array: run of bucket r from tile t goes to
//     out + (r * ntiles + t) * R          (bucket-major, tile-minor: exactly
// the layout a stable counting sort produces when every bucket gets the same
// number of keys per tile).  This probe writes that pattern with no hashing,
// no LDS and no loads: R bytes per (tile, bucket), nranks buckets, tiles
// dealt to XCDs in contiguous ranges (workgroup b on XCD b % 8), each
// workgroup's 256 threads writing its tile's runs with consecutive lanes
// covering consecutive bytes of a run.  Prints GB/s per (R, nranks, wg/CU).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/scatter_probe tools/scatter_probe.hip
//   tools/bin/scatter_probe [total_MiB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned long long u64;
typedef unsigned int u32;

// R bytes per run, written as R/4 dwords; 256 threads cover a tile's
// nranks runs: thread j writes dword j, j+256, ... of the tile's
// nranks*R/4 dwords (run r = dwords [r*R/4, (r+1)*R/4)).
// skew4: every run is shifted by skew4 dwords (runs of a real counting sort
// start wherever the prefix sums put them, not on a line).
__global__ __launch_bounds__(256) void scatter(u32 *__restrict__ out, u32 R4, u32 nranks, u64 ntiles, u32 skew4) {
  u64 t, end, step;
  if (gridDim.x >= 8 && gridDim.x % 8 == 0) {
    const u64 x = blockIdx.x % 8, per = gridDim.x / 8;
    t = x * ntiles / 8 + blockIdx.x / 8;
    end = (x + 1) * ntiles / 8;
    step = per;
  } else {
    t = blockIdx.x;
    end = ntiles;
    step = gridDim.x;
  }
  const u32 nd = nranks * R4;
  for (; t < end; t += step) {
    for (u32 d = threadIdx.x; d < nd; d += 256) {
      const u32 r = d / R4, k = d - r * R4;
      out[((u64)r * ntiles + t) * R4 + k + skew4] = (u32)t ^ d;
    }
  }
}

int main(int argc, char **argv) {
  const u64 total = (u64)(argc > 1 ? atoi(argv[1]) : 384) << 20;
  u32 *buf;
  CK(hipMalloc(&buf, total));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const u32 Rs[] = {16, 32, 64, 128, 256};
  const u32 NRs[] = {1024};
  const int PCs[] = {2};
  const u32 SKs[] = {0, 2, 7};  // dwords
  for (u32 sk : SKs)
  for (u32 nr : NRs)
    for (u32 R : Rs)
      for (int pc : PCs) {
        const u64 ntiles = total / ((u64)R * nr);
        const unsigned g = (unsigned)std::min<u64>(ntiles, (u64)cus * pc) & ~7u;
        scatter<<<g, 256>>>(buf, R / 4, nr, ntiles - 1, sk);
        CK(hipDeviceSynchronize());
        std::vector<float> ms;
        for (int i = 0; i < 10; ++i) {
          CK(hipEventRecord(a));
          scatter<<<g, 256>>>(buf, R / 4, nr, ntiles - 1, sk);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float m;
          CK(hipEventElapsedTime(&m, a, b));
          ms.push_back(m);
        }
        std::sort(ms.begin(), ms.end());
        const double bytes = (double)ntiles * R * nr;
        printf("{\"run_bytes\": %u, \"skew_bytes\": %u, \"nranks\": %u, \"per_cu\": %d, \"MiB\": %.0f, "
               "\"median_ms\": %.4f, \"GBps\": %.1f}\n",
               R, 4 * sk, nr, pc, bytes / 1048576, ms[5], bytes / ms[5] / 1e6);
      }
  CK(hipFree(buf));
  return 0;
}
