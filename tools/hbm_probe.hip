// hbm_probe.hip -- what HBM rate can the 64-B key stream reach on this box?
//
// Standalone calibration (not part of the product): sweeps the access shapes
// the CityHash kernels could use, over the same traffic as cfg2 (read 64 B,
// write 8 B per key), with HIP events, median of R launches, interleaved.
//
//   rd<T,NT>       read-only: a wave reads T KiB contiguous per iteration
//                  (T global_load_dwordx4 of 1 KiB), grid-stride
//   rdpf<NT>       read-only, 4 KiB tiles, next tile in VGPRs while this one
//                  is consumed (the k_fixed_xpose64 shape without the hash)
//   dma<D,AUX>     read-only via LDS-DMA (global_load_lds_dwordx4), a ring of
//                  D 4-KiB slots per wave, wait vmcnt(4(D-1))
//   kv<D,AUX>      key-shaped: LDS-DMA ring of D slots, each lane reads its
//                  64-B row back (ds_read_b128 x4), folds it to 8 B and stores
//                  it nt (72 B of traffic per key, no hash)
//
//   hipcc --offload-arch=gfx950 -O3 -o build/hbm_probe tools/hbm_probe.hip
//   build/hbm_probe [GiB]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <int T, bool NT>
__global__ __launch_bounds__(256) void rd(const u32x4 *__restrict__ p, u64 ntile, u64 *out) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  u32x4 acc = {0, 0, 0, 0};
  for (u64 t = wave; t < ntile; t += nw) {
    const u32x4 *q = p + t * (64 * T) + lane;
    u32x4 v[T];
#pragma unroll
    for (int j = 0; j < T; ++j) v[j] = ld<NT>(q + 64 * j);
#pragma unroll
    for (int j = 0; j < T; ++j) acc ^= v[j];
  }
  u64 s = ((u64)(acc.x ^ acc.z) << 32) | (acc.y ^ acc.w);
  if (s == 0x123456789ull) out[0] = s;  // keep the loads
}

// Per-lane walk (the long-key kernels' shape): a wave takes 64 rows of L
// bytes, lane l walks row l in spans of P 16-B pieces (P dwordx4 loads in
// flight per lane), every wave-instruction touching 64 different lines.
template <int L, int P>
__global__ __launch_bounds__(256) void walk(const u32x4 *__restrict__ p, u64 nrows, u64 *out) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  u32x4 acc = {0, 0, 0, 0};
  for (u64 t = wave; t * 64 < nrows; t += nw) {
    const u32x4 *q = p + (t * 64 + lane) * (L / 16);
#pragma unroll 1
    for (int o = 0; o < L / 16; o += P) {
      u32x4 v[P];
#pragma unroll
      for (int j = 0; j < P; ++j) v[j] = q[o + j];
#pragma unroll
      for (int j = 0; j < P; ++j) acc ^= v[j] * 3u;
    }
  }
  u64 s = ((u64)(acc.x ^ acc.z) << 32) | (acc.y ^ acc.w);
  if (s == 0x123456789ull) out[0] = s;
}

template <bool NT>
__global__ __launch_bounds__(256) void rdpf(const u32x4 *__restrict__ p, u64 ntile, u64 *out) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 a[4], b[4];
  u64 t = wave;
  if (t < ntile)
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = ld<NT>(p + t * 256 + 64 * j + lane);
  for (; t < ntile; t += 2 * nw) {
    if (t + nw < ntile)
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = ld<NT>(p + (t + nw) * 256 + 64 * j + lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= a[j] * 3u;
    if (t + nw >= ntile) break;
    if (t + 2 * nw < ntile)
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = ld<NT>(p + (t + 2 * nw) * 256 + 64 * j + lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= b[j] * 5u;
  }
  u64 s = ((u64)(acc.x ^ acc.z) << 32) | (acc.y ^ acc.w);
  if (s == 0x123456789ull) out[0] = s;
}

template <class T>
__device__ __forceinline__ u32 lds_addr(const T *p) {
  return (u32)(uintptr_t)(const __attribute__((address_space(3))) T *)(p);
}

// LDS-DMA ring: D slots of 4 KiB per wave; KEYS: consume as 64-B keys and
// write 8 B per key (nt).
template <int D, int AUX, bool KEYS>
__global__ __launch_bounds__(256) void dma(const uint8_t *__restrict__ p, u64 ntile, u64 *out) {
  __shared__ __attribute__((aligned(16))) u32 ring[4][D][1024];
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 nw = (u64)gridDim.x * 4;
  const u64 w0 = (u64)blockIdx.x * 4 + wave;
  auto issue = [&](u64 t, int s) {
    const uint8_t *base = p + (t << 12);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(base + 1024 * j + 16 * lane),
                                       (void __attribute__((address_space(3))) *)&ring[wave][s][256 * j], 16, 0, AUX);
  };
  // prologue: D-1 tiles in flight
#pragma unroll
  for (int s = 0; s < D - 1; ++s)
    if (w0 + s * nw < ntile) issue(w0 + s * nw, s);
  u32x4 acc = {0, 0, 0, 0};
  int s = 0;
  for (u64 t = w0; t < ntile; t += nw) {
    const u64 tn = t + (D - 1) * nw;
    const int sn = (s + D - 1) % D;
    if (tn < ntile) {
      issue(tn, sn);
      // D-1 tiles newer than t may be outstanding (4 instr each)
      if constexpr (D == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (D == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (D == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else if constexpr (D == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const u32 img = lds_addr(&ring[wave][s][0]);
    u32x4 v[4];
    if (KEYS) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const u32 a = img + 64 * lane + 16 * c;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v[c]) : "v"(a) : "memory");
      }
    } else {
      const u32 a = img + 16 * lane;
      asm volatile("ds_read_b128 %0, %1" : "=v"(v[0]) : "v"(a) : "memory");
      v[1] = v[2] = v[3] = v[0];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (KEYS) {
      u32x4 f = v[0] ^ v[1] * 3u ^ v[2] * 5u ^ v[3] * 7u;
      u64 h = ((u64)(f.x ^ f.z) << 32) | (f.y ^ f.w);
      __builtin_nontemporal_store(h, out + 1 + (t << 6) + lane);
    } else {
      acc ^= v[0];
    }
    s = (s + 1) % D;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  u64 sum = ((u64)(acc.x ^ acc.z) << 32) | (acc.y ^ acc.w);
  if (sum == 0x123456789ull) out[0] = sum;
}

// Key-shaped with register prefetch (xpose without transpose/hash): read a
// 4 KiB tile per wave, write 8 B per lane nt, DEPTH tiles in flight.
template <int DEPTH, bool NT>
__global__ __launch_bounds__(256) void kvreg(const u32x4 *__restrict__ p, u64 ntile, u64 *out) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  u32x4 pre[DEPTH][4];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (wave + d * nw < ntile)
#pragma unroll
      for (int j = 0; j < 4; ++j) pre[d][j] = ld<NT>(p + (wave + d * nw) * 256 + 64 * j + lane);
  for (u64 t = wave; t < ntile; t += DEPTH * nw) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const u64 tt = t + d * nw;
      if (tt >= ntile) break;
      u32x4 f = pre[d][0] ^ pre[d][1] * 3u ^ pre[d][2] * 5u ^ pre[d][3] * 7u;
      const u64 tn = tt + DEPTH * nw;
      if (tn < ntile)
#pragma unroll
        for (int j = 0; j < 4; ++j) pre[d][j] = ld<NT>(p + tn * 256 + 64 * j + lane);
      u64 h = ((u64)(f.x ^ f.z) << 32) | (f.y ^ f.w);
      __builtin_nontemporal_store(h, out + 1 + (tt << 6) + lane);
    }
  }
}

// Key-shaped, G consecutive 4-KiB tiles per wave per unit (one unit of
// prefetch in flight); digests stored after the unit.  SM: 0 = nt 8 B/lane,
// 1 = plain 8 B/lane, 2 = nt 16 B/lane (tile pairs via shuffles), 3 = plain
// 16 B/lane.
template <int G, int SM>
__global__ __launch_bounds__(256) void kvg(const u32x4 *__restrict__ p, u64 nunit, u64 *out) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  u32x4 pre[G][4];
  auto fetch = [&](u64 u) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 4; ++j) pre[g][j] = __builtin_nontemporal_load(p + (u * G + g) * 256 + 64 * j + lane);
  };
  if (wave < nunit) fetch(wave);
  for (u64 u = wave; u < nunit; u += nw) {
    u64 h[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      u32x4 f = pre[g][0] ^ pre[g][1] * 3u ^ pre[g][2] * 5u ^ pre[g][3] * 7u;
      h[g] = ((u64)(f.x ^ f.z) << 32) | (f.y ^ f.w);
    }
    if (u + nw < nunit) fetch(u + nw);
    u64 *o = out + 1 + u * G * 64;
    if constexpr (SM < 2) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        if constexpr (SM == 0) __builtin_nontemporal_store(h[g], o + g * 64 + lane);
        else o[g * 64 + lane] = h[g];
      }
    } else {
      typedef u64 u64x2 __attribute__((ext_vector_type(2)));
      static_assert(G % 2 == 0, "pairs");
#pragma unroll
      for (int g = 0; g < G; g += 2) {
        const int s0 = (2 * lane) & 63, s1 = (2 * lane + 1) & 63;
        const u64 a0 = __shfl(h[g], s0), a1 = __shfl(h[g], s1);
        const u64 b0 = __shfl(h[g + 1], s0), b1 = __shfl(h[g + 1], s1);
        const u64x2 v = lane < 32 ? u64x2{a0, a1} : u64x2{b0, b1};
        u64x2 *d = reinterpret_cast<u64x2 *>(o + g * 64) + lane;
        if constexpr (SM == 2) __builtin_nontemporal_store(v, d);
        else *d = v;
      }
    }
  }
}

// Write-only stream: 16 B per lane, 1 KiB per wave-instruction, 4 per tile.
template <bool NT>
__global__ __launch_bounds__(256) void wr(u32x4 *__restrict__ p, u64 ntile) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  const u32x4 v = {lane, (u32)wave, 7u, 9u};
  for (u64 t = wave; t < ntile; t += nw)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (NT) __builtin_nontemporal_store(v, p + t * 256 + 64 * j + lane);
      else p[t * 256 + 64 * j + lane] = v;
    }
}

// cfg3's byte mix with plain coalesced accesses, no LDS and no hash (VERDICT
// r05 item 3): per 64-key tile a wave reads the tile's u64 offsets (one per
// lane), the tile's contiguous key bytes in 16-B pieces (every lane folds its
// pieces), and writes one 8-B digest per lane.
//   cfg3mix<NT,PERWAVE>  uniform 136-B keys: the key range of tile t is
//                    [t*8704, (t+1)*8704), independent of the offsets (no
//                    dependent round trip): the byte mix's own ceiling
//   cfg3dep<NT>      the real cfg3 offsets: the key range is read from the
//                    offsets first (offsets -> bytes, one dependent round trip
//                    per tile, as every offset-indexed kernel must)
// NT: non-temporal loads and digest stores.  PERWAVE: tiles a wave has in
// flight (loads of all issued before any is folded).
template <bool NT, int PERWAVE>
__global__ __launch_bounds__(256) void cfg3mix(const uint8_t *__restrict__ keys, const u64 *__restrict__ offs,
                                               u64 ntiles, u64 *__restrict__ dig) {
  constexpr u32 kTileBytes = 64 * 136;  // 8704 B = 544 pieces of 16 B
  constexpr int kPieces = kTileBytes / 16, kPer = (kPieces + 63) / 64;
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  for (u64 t0 = wave * PERWAVE; t0 < ntiles; t0 += nw * PERWAVE) {
    u32x4 v[PERWAVE][kPer];
    u64 o[PERWAVE];
#pragma unroll
    for (int w = 0; w < PERWAVE; ++w) {
      const u64 t = min(t0 + w, ntiles - 1);
      o[w] = NT ? __builtin_nontemporal_load(offs + t * 64 + lane) : offs[t * 64 + lane];
      const u32x4 *q = reinterpret_cast<const u32x4 *>(keys + t * kTileBytes);
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int pc = j * 64 + lane;
        v[w][j] = pc < kPieces ? ld<NT>(q + pc) : u32x4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int w = 0; w < PERWAVE; ++w) {
      if (t0 + w >= ntiles) break;
      u32x4 f = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < kPer; ++j) f ^= v[w][j] * (u32)(2 * j + 1);
      const u64 h = (((u64)(f.x ^ f.z) << 32) | (f.y ^ f.w)) ^ o[w];
      if (NT) __builtin_nontemporal_store(h, dig + (t0 + w) * 64 + lane);
      else dig[(t0 + w) * 64 + lane] = h;
    }
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void cfg3dep(const uint8_t *__restrict__ keys, const u64 *__restrict__ offs,
                                               u64 n, u64 *__restrict__ dig) {
  const u32 lane = threadIdx.x & 63;
  const u64 wave = (u64)blockIdx.x * 4 + (threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * 4;
  const u64 ntiles = (n + 63) / 64;
  for (u64 t = wave; t < ntiles; t += nw) {
    const u64 k = min(t * 64 + lane, n - 1);
    const u64 o = NT ? __builtin_nontemporal_load(offs + k) : offs[k];
    const u64 hi_k = min(t * 64 + 64, n);
    const u64 end = __shfl(NT ? __builtin_nontemporal_load(offs + hi_k) : offs[hi_k], 0);
    const u64 beg = __shfl(o, 0);
    const u64 a0 = beg & ~15ull, a1 = (end + 15) & ~15ull;
    const u32x4 *q = reinterpret_cast<const u32x4 *>(keys + a0);
    const u64 np = (a1 - a0) / 16;
    u32x4 f = {0, 0, 0, 0};
    for (u64 j0 = 0; j0 < np; j0 += 64 * 8) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const u64 pc = j0 + j * 64 + lane;
        v[j] = pc < np ? ld<NT>(q + pc) : u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) f ^= v[j] * (u32)(2 * j + 1);
    }
    const u64 h = (((u64)(f.x ^ f.z) << 32) | (f.y ^ f.w)) ^ o;
    if (t * 64 + lane < n) {
      if (NT) __builtin_nontemporal_store(h, dig + t * 64 + lane);
      else dig[t * 64 + lane] = h;
    }
  }
}

static u64 splitmix64_at(u64 seed, u64 k) {
  u64 z = seed + (k + 1) * 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

int main(int argc, char **argv) {
  const char *set0 = getenv("PROBE_SET");
  if (set0 && std::string(set0) == "cfg3") {
    // cfg3: 64M keys of 16..256 B (bench.py mixed_lengths: 16 + splitmix64(SEED_LENS, i) % 241),
    // offsets[n+1], digests[n]; and the uniform 136-B form of the same byte mix
    const u64 n = 64ull << 20;
    std::vector<u64> hoff(n + 1);
    hoff[0] = 0;
    for (u64 i = 0; i < n; ++i) hoff[i + 1] = hoff[i] + 16 + splitmix64_at(0x1E575EED1E575EEDull, i) % 241;
    const u64 total = hoff[n], uni = n * 136;
    const u64 kbytes = std::max(total, uni) + 4096;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint8_t *keys;
    u64 *offs, *uoffs, *dig;
    CK(hipMalloc(&keys, kbytes));
    CK(hipMalloc(&offs, (n + 1) * 8));
    CK(hipMalloc(&uoffs, (n + 1) * 8));
    CK(hipMalloc(&dig, n * 8));
    CK(hipMemset(keys, 0x5a, kbytes));
    CK(hipMemcpy(offs, hoff.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    for (u64 i = 0; i <= n; ++i) hoff[i] = i * 136;
    CK(hipMemcpy(uoffs, hoff.data(), (n + 1) * 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    const double real_b = (double)total + 16.0 * n + 8, uni_b = (double)uni + 16.0 * n + 8;
    struct C3 {
      std::string name;
      int pc;
      double bytes;
      std::function<void(unsigned)> go;
      std::vector<float> ms;
    };
    std::vector<C3> cs;
    const u64 ntiles = n / 64;
    for (int pc : {2, 4, 8}) {
      cs.push_back({"cfg3dep<nt>", pc, real_b, [=](unsigned g) { cfg3dep<true><<<g, 256>>>(keys, offs, n, dig); }, {}});
      cs.push_back({"cfg3dep<plain>", pc, real_b, [=](unsigned g) { cfg3dep<false><<<g, 256>>>(keys, offs, n, dig); }, {}});
      cs.push_back({"cfg3mix<nt,1>", pc, uni_b, [=](unsigned g) { cfg3mix<true, 1><<<g, 256>>>(keys, uoffs, ntiles, dig); }, {}});
      cs.push_back({"cfg3mix<plain,1>", pc, uni_b, [=](unsigned g) { cfg3mix<false, 1><<<g, 256>>>(keys, uoffs, ntiles, dig); }, {}});
    }
    for (int pc : {2, 4}) {
      cs.push_back({"cfg3mix<nt,2>", pc, uni_b, [=](unsigned g) { cfg3mix<true, 2><<<g, 256>>>(keys, uoffs, ntiles, dig); }, {}});
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto &c : cs) c.go(cus * c.pc);
    CK(hipDeviceSynchronize());
    CK(hipGetLastError());
    const int reps = argc > 2 ? atoi(argv[2]) : 10;
    for (int r = 0; r < reps; ++r)
      for (auto &c : cs) {
        CK(hipEventRecord(e0));
        c.go(cus * c.pc);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        c.ms.push_back(ms);
      }
    CK(hipGetLastError());
    printf("{\"cfg3_key_bytes\": %llu, \"uniform_key_bytes\": %llu, \"keys\": %llu}\n", (unsigned long long)total,
           (unsigned long long)uni, (unsigned long long)n);
    for (auto &c : cs) {
      std::vector<float> v = c.ms;
      std::sort(v.begin(), v.end());
      const float med = v[v.size() / 2];
      printf("{\"case\": \"%s\", \"per_cu\": %d, \"median_ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f, \"frac\": %.4f}\n",
             c.name.c_str(), c.pc, med, v[0], c.bytes / med / 1e6, c.bytes / med / 1e6 / 8000.0);
    }
    return 0;
  }
  const double gib = argc > 1 ? atof(argv[1]) : 1.0;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const u64 bytes = (u64)(gib * (1ull << 30)) & ~4095ull;
  const u64 ntile = bytes >> 12;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t *buf;
  u64 *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, (ntile * 64 + 1) * 8));
  CK(hipMemset(buf, 0x5a, bytes));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));

  struct Case {
    std::string name;
    int percu;
    double bytes_per_launch;
    std::function<void(unsigned)> launch;
    std::vector<float> ms;
  };
  std::vector<Case> cases;
  const u32x4 *p4 = reinterpret_cast<const u32x4 *>(buf);
  const double rdb = (double)bytes, kvb = (double)bytes * 72.0 / 64.0;
#define ADD(nm, pc, b, ...) cases.push_back({nm, pc, b, [=](unsigned g) { __VA_ARGS__; }, {}})
  const char *set = getenv("PROBE_SET");
  const std::string which = set ? set : "read";
  if (which == "read") {
    for (int pc : {2, 4, 8}) {
      ADD("rd<4,plain>", pc, rdb, rd<4, false><<<g, 256>>>(p4, ntile, out));
      ADD("rd<4,nt>", pc, rdb, rd<4, true><<<g, 256>>>(p4, ntile, out));
    }
    for (int pc : {2, 4}) {
      ADD("rd<8,plain>", pc, rdb, (rd<8, false><<<g, 256>>>(p4, ntile / 2, out)));
      ADD("rd<8,nt>", pc, rdb, (rd<8, true><<<g, 256>>>(p4, ntile / 2, out)));
    }
    for (int pc : {2, 3, 4}) {
      ADD("rdpf<plain>", pc, rdb, rdpf<false><<<g, 256>>>(p4, ntile, out));
      ADD("rdpf<nt>", pc, rdb, rdpf<true><<<g, 256>>>(p4, ntile, out));
    }
    for (int pc : {1, 2, 3, 4}) {
      ADD("dma<2,def>", pc, rdb, (dma<2, 0, false><<<g, 256>>>(buf, ntile, out)));
      ADD("dma<2,nt>", pc, rdb, (dma<2, 2, false><<<g, 256>>>(buf, ntile, out)));
      ADD("dma<4,def>", pc, rdb, (dma<4, 0, false><<<g, 256>>>(buf, ntile, out)));
      ADD("dma<4,nt>", pc, rdb, (dma<4, 2, false><<<g, 256>>>(buf, ntile, out)));
    }
    for (int pc : {1, 2}) {
      ADD("dma<5,nt>", pc, rdb, (dma<5, 2, false><<<g, 256>>>(buf, ntile, out)));
      ADD("kv-dma<5,nt>", pc, kvb, (dma<5, 2, true><<<g, 256>>>(buf, ntile, out)));
    }
    for (int pc : {2, 3, 4}) {
      ADD("kv-dma<2,nt>", pc, kvb, (dma<2, 2, true><<<g, 256>>>(buf, ntile, out)));
      ADD("kv-dma<3,nt>", pc, kvb, (dma<3, 2, true><<<g, 256>>>(buf, ntile, out)));
      ADD("kv-dma<4,nt>", pc, kvb, (dma<4, 2, true><<<g, 256>>>(buf, ntile, out)));
      ADD("kv-dma<4,def>", pc, kvb, (dma<4, 0, true><<<g, 256>>>(buf, ntile, out)));
      ADD("kvreg<2,nt>", pc, kvb, (kvreg<2, true><<<g, 256>>>(p4, ntile, out)));
      ADD("kvreg<2,plain>", pc, kvb, (kvreg<2, false><<<g, 256>>>(p4, ntile, out)));
      ADD("kvreg<3,nt>", pc, kvb, (kvreg<3, true><<<g, 256>>>(p4, ntile, out)));
    }
  } else if (which == "walk") {  // per-lane walks over 1 KiB rows vs the coalesced read
    const u64 rows = bytes / 1024;
    for (int pc : {2, 4, 8}) {
      ADD("rd<4,plain>", pc, rdb, rd<4, false><<<g, 256>>>(p4, ntile, out));
      ADD("walk<1024,16>", pc, rdb, (walk<1024, 16><<<g, 256>>>(p4, rows, out)));
      ADD("walk<1024,8>", pc, rdb, (walk<1024, 8><<<g, 256>>>(p4, rows, out)));
      ADD("walk<1024,4>", pc, rdb, (walk<1024, 4><<<g, 256>>>(p4, rows, out)));
    }
  } else {  // "write": store shapes next to the 64-B key stream
    u32x4 *w4 = reinterpret_cast<u32x4 *>(out + 2);  // 16-B aligned
    const u64 wtile = (ntile * 64 * 8) >> 12;        // digest-sized write stream
    for (int pc : {2, 4, 8}) {
      ADD("wr<nt>", pc, (double)wtile * 4096, (wr<true><<<g, 256>>>(w4, wtile)));
      ADD("wr<plain>", pc, (double)wtile * 4096, (wr<false><<<g, 256>>>(w4, wtile)));
    }
    for (int pc : {1, 2, 3}) {
      ADD("kvg<1,nt8>", pc, kvb, (kvg<1, 0><<<g, 256>>>(p4, ntile, out)));
      ADD("kvg<1,plain8>", pc, kvb, (kvg<1, 1><<<g, 256>>>(p4, ntile, out)));
      ADD("kvg<2,nt8>", pc, kvb, (kvg<2, 0><<<g, 256>>>(p4, ntile / 2, out)));
      ADD("kvg<2,nt16>", pc, kvb, (kvg<2, 2><<<g, 256>>>(p4, ntile / 2, out)));
      ADD("kvg<2,plain16>", pc, kvb, (kvg<2, 3><<<g, 256>>>(p4, ntile / 2, out)));
      ADD("kvg<4,nt8>", pc, kvb, (kvg<4, 0><<<g, 256>>>(p4, ntile / 4, out)));
      ADD("kvg<4,nt16>", pc, kvb, (kvg<4, 2><<<g, 256>>>(p4, ntile / 4, out)));
      ADD("kvg<4,plain16>", pc, kvb, (kvg<4, 3><<<g, 256>>>(p4, ntile / 4, out)));
      ADD("kvreg<2,nt>", pc, kvb, (kvreg<2, true><<<g, 256>>>(p4, ntile, out)));
    }
  }
#undef ADD
  // warm + interleaved rounds
  for (auto &c : cases) c.launch(cus * c.percu);
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  for (int r = 0; r < reps; ++r) {
    for (auto &c : cases) {
      CK(hipEventRecord(e0));
      c.launch(cus * c.percu);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      c.ms.push_back(ms);
    }
  }
  CK(hipGetLastError());
  std::sort(cases.begin(), cases.end(), [](const Case &a, const Case &b) {
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    return a.bytes_per_launch / med(a.ms) > b.bytes_per_launch / med(b.ms);
  });
  for (auto &c : cases) {
    std::vector<float> v = c.ms;
    std::sort(v.begin(), v.end());
    const float med = v[v.size() / 2];
    printf("{\"case\": \"%s\", \"per_cu\": %d, \"GiB\": %.2f, \"median_ms\": %.4f, \"min_ms\": %.4f, \"GBps\": %.1f}\n",
           c.name.c_str(), c.percu, gib, med, v[0], c.bytes_per_launch / med / 1e6);
  }
  return 0;
}
