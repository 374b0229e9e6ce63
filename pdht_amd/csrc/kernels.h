// kernels.h -- gfx950 kernels of the batch key-hashing engine.
//
// Layout of the work:
//   * one key per lane, 64 keys per wave, digests stored lane-contiguous
//     (8 B or 16 B per lane -> 512 B / 1 KiB per wave-instruction);
//   * k_fixed_direct<L>: packed keys of a compile-time length L (8/16/32/64):
//     each lane pulls its own key with L/16 global_load_dwordx4 straight into
//     VGPRs (a wave's 4 instructions cover one contiguous 4 KiB span), the
//     algorithm runs with every offset constant-folded;
//   * k_fixed_lds<64>: same, but the wave's 4 KiB tile arrives by 4
//     LDS-DMA instructions (global_load_lds_dwordx4, fully contiguous 1 KiB
//     per instruction, no VGPR staging) and each lane reads its 64-byte row
//     back with ds_read_b128 through an XOR swizzle (conflict-free);
//   * k_window: any key length, fixed stride or offset-indexed: the wave's
//     contiguous byte range is DMA'd into a per-wave LDS window and each lane
//     hashes its key out of LDS with byte-aligned fetches
//     (v_alignbyte_b32); keys that do not fit the window are read from
//     global memory directly.
// All kernels are grid-stride persistent loops (grid ~ CUs x residency) and
// carry no inter-workgroup communication.
#pragma once

#include <type_traits>

#include "city_core.h"

namespace pdht {

typedef u32 u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;  // 4 waves
constexpr int kWavesPerBlock = kBlock / 64;

// --------------------------------------------------------------- readers ---
// Key bytes in LDS at an arbitrary byte offset.  A span of N bytes is one run
// of N/4+1 dword reads from one base address (ds_read2_b32 with immediate
// offsets, a single wait) funnelled by v_alignbyte_b32; the window carries
// 16 B of slack so the trailing dword read stays in the array.
struct LdsReader {
  const u32 *lds;
  u32 base;
  template <int N>
  __device__ __forceinline__ Words<N / 4> span(u32 o) const {
    const u32 a = base + o;
    const u32 *p = lds + (a >> 2);
    const u32 r = a & 3u;
    u32 raw[N / 4 + 1];
#pragma unroll
    for (int j = 0; j <= N / 4; ++j) raw[j] = p[j];
    Words<N / 4> w;
#pragma unroll
    for (int j = 0; j < N / 4; ++j) w.d[j] = __builtin_amdgcn_alignbyte(raw[j + 1], raw[j], r);
    return w;
  }
  __device__ __forceinline__ u32 w32(u32 o) const { return span<4>(o).d[0]; }
  __device__ __forceinline__ u32 b8(u32 o) const {
    const u32 a = base + o;
    return (lds[a >> 2] >> (8 * (a & 3u))) & 0xffu;
  }
};

// Key bytes straight from global memory (keys outside the LDS window): the
// same dword-run + funnel shape on the dword-aligned address.  The extra
// trailing dword is only read when the span is misaligned (it then holds key
// bytes), so no read leaves the key's dwords.
// Loads go through explicit global-address-space pointers: a generic (flat)
// load would make the compiler drain vmcnt AND lgkmcnt at every join after
// it, i.e. wait for the next tile's prefetch on the common path too.
typedef const __attribute__((address_space(1))) u32 gu32;
typedef const __attribute__((address_space(1))) uint8_t gu8;
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
template <bool A16 = false>
struct GlobalReaderT {
  const uint8_t *p;
  template <int N>
  __device__ __forceinline__ Words<N / 4> span(u32 o) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    if constexpr (A16 && N % 16 == 0) {
      // packed keys at a 16-B multiple stride: 16-B aligned spans (every
      // lane alike) load as dwordx4, a quarter of the instructions
      if ((a & 15) == 0) {
        gu32x4 *q = reinterpret_cast<gu32x4 *>(a);
        Words<N / 4> w;
#pragma unroll
        for (int j = 0; j < N / 16; ++j) {
          const u32x4 v = q[j];
          w.d[4 * j + 0] = v.x;
          w.d[4 * j + 1] = v.y;
          w.d[4 * j + 2] = v.z;
          w.d[4 * j + 3] = v.w;
        }
        return w;
      }
    }
    gu32 *q = reinterpret_cast<gu32 *>(a & ~(uintptr_t)3);
    const u32 r = (u32)(a & 3);
    u32 raw[N / 4 + 1];
#pragma unroll
    for (int j = 0; j < N / 4; ++j) raw[j] = q[j];
    raw[N / 4] = r ? q[N / 4] : 0u;
    Words<N / 4> w;
#pragma unroll
    for (int j = 0; j < N / 4; ++j) w.d[j] = __builtin_amdgcn_alignbyte(raw[j + 1], raw[j], r);
    return w;
  }
  __device__ __forceinline__ u32 w32(u32 o) const { return span<4>(o).d[0]; }
  __device__ __forceinline__ u32 b8(u32 o) const {
    return reinterpret_cast<gu8 *>(reinterpret_cast<uintptr_t>(p))[o];
  }
};
typedef GlobalReaderT<false> GlobalReader;

// ------------------------------------------------------------ algorithms ---
struct AlgoCity64 {
  typedef u64 Out;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const { return city64(r, len); }
};
struct AlgoCity64Seeds {
  typedef u64 Out;
  u64 s0, s1;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const {
    return city64_seeds(r, len, s0, s1);
  }
};
struct AlgoCity128 {
  typedef u128 Out;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const { return city128(r, len); }
};
struct AlgoCity128Seed {
  typedef u128 Out;
  u64 lo, hi;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const {
    return city128_seed(r, len, u128{lo, hi});
  }
};
struct AlgoCrc128 {
  typedef u128 Out;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const { return crc128(r, len); }
};
struct AlgoCrc128Seed {
  typedef u128 Out;
  u64 lo, hi;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const {
    return crc128_seed(r, len, u128{lo, hi});
  }
};

// CRC-32C slicing tables in LDS (8 KiB per workgroup) for batches that may
// hold keys > 900 B (CityHashCrc256 path, city.c:407-517): one lookup per key
// byte, 64 lanes at random table words.  From constant memory those lookups
// are per-lane vector loads through the TA, 4x slower (tools/longbench.py).
struct CrcLdsTab {
  const u32 *t;
  __device__ __forceinline__ u32 operator()(u32 slice, u32 byte) const { return t[slice * 256 + byte]; }
};
template <class Base>
struct CrcLds : Base {
  static constexpr bool kCrcLds = true;
  const u32 *tab = nullptr;  // set by algo_init() inside the kernel
  template <class R>
  __device__ __forceinline__ typename Base::Out operator()(const R &r, u64 len) const;
};
template <>
template <class R>
__device__ __forceinline__ u128 CrcLds<AlgoCrc128>::operator()(const R &r, u64 len) const {
  return crc128(r, len, CrcLdsTab{tab});
}
template <>
template <class R>
__device__ __forceinline__ u128 CrcLds<AlgoCrc128Seed>::operator()(const R &r, u64 len) const {
  return crc128_seed(r, len, u128{this->lo, this->hi}, CrcLdsTab{tab});
}

template <class A, class = void>
struct HasCrcLds {
  static constexpr bool value = false;
};
template <class A>
struct HasCrcLds<A, decltype((void)A::kCrcLds)> {
  static constexpr bool value = A::kCrcLds;
};

// Per-workgroup algorithm setup, reached by every thread of the block.
template <class Algo>
__device__ __forceinline__ void algo_init(Algo &a) {
  if constexpr (HasCrcLds<Algo>::value) {
    __shared__ u32 tab[8 * 256];
    for (u32 k = threadIdx.x; k < 8 * 256; k += blockDim.x) tab[k] = kCrcDev.t[k >> 8][k & 255];
    __syncthreads();
    a.tab = tab;
  }
}

// Calibration only (pdht_hip_key_stream_dev): the data movement of a hash
// kernel with the hash replaced by an XOR fold of the key's 64 bytes.
struct AlgoFold64 {
  typedef u64 Out;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64) const {
    const Words<16> w = r.template span<64>(0);
    u32 a = 0, b = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a ^= w.d[2 * j];
      b ^= w.d[2 * j + 1];
    }
    return ((u64)b << 32) | a;
  }
};

// Calibration only (pdht_hip_key_stream_var_dev): every byte of a key read
// through the same reader (16-B spans, then single bytes), XOR-folded.
struct AlgoFoldVar {
  typedef u64 Out;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const {
    u32 a = (u32)len, b = 0;
    u32 o = 0;
    for (; o + 16 <= len; o += 16) {
      const Words<4> w = r.template span<16>(o);
      a ^= w.d[0] ^ w.d[2];
      b ^= w.d[1] ^ w.d[3];
    }
    for (; o < len; ++o) a ^= r.b8(o) << (8 * (o & 3));
    return ((u64)b << 32) | a;
  }
};

// ----------------------------------------------------------------- sinks ---
// Where a digest goes.  init()/flush() run once per workgroup around the
// grid-stride loop (every thread reaches both).
template <bool NT, class T>
__device__ __forceinline__ void st(T v, T *p) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// NTS: non-temporal digest stores (cache-policy experiment knob).
template <bool NTS = false>
struct Sink64T {
  static constexpr u32 kHist = 1;  // LDS histogram words this sink needs
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64 i, u64 h) { st<NTS>(h, out + i); }
  __device__ __forceinline__ void flush() {}
};
template <bool NTS = false>
struct Sink128T {
  static constexpr u32 kHist = 1;
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64 i, u128 h) {
    typedef u64 u64x2 __attribute__((ext_vector_type(2)));
    u64x2 v = {h.lo, h.hi};
    st<NTS>(v, reinterpret_cast<u64x2 *>(out) + i);
  }
  __device__ __forceinline__ void flush() {}
};
typedef Sink64T<false> Sink64;
typedef Sink128T<false> Sink128;

// The same sink with non-temporal stores (identity for other sinks).
template <class S>
struct NtSink {
  typedef S type;
  static __device__ __host__ S make(S s) { return s; }
};
template <>
struct NtSink<Sink64> {
  typedef Sink64T<true> type;
  static __host__ type make(Sink64 s) { return type{s.lds_hist, s.out}; }
};
template <>
struct NtSink<Sink128> {
  typedef Sink128T<true> type;
  static __host__ type make(Sink128 s) { return type{s.lds_hist, s.out}; }
};

// u64 remainder by a run-time invariant divisor: Granlund & Montgomery
// (PLDI'94, fig. 4.1): q = (t + ((n - t) >> 1)) >> (l - 1), t = mulhi(m', n),
// m' = floor(2^64 (2^l - d) / d) + 1, l = ceil(log2 d); exact for every n.
struct FastMod {
  u64 d, m;
  u32 sh, pow2;
  __device__ __forceinline__ u64 mod(u64 n) const {
    if (pow2) return n & (d - 1);
    const u64 t = __umul64hi(m, n);
    const u64 q = (t + ((n - t) >> 1)) >> sh;
    return n - q * d;
  }
};

constexpr u32 kHistLds = 4096;  // per-workgroup LDS bins before going global

// pdht_hash placement (libpdht/hash.c:26-29) + rankputs histogram
// (putget.c:55).
template <bool NTS = false>
struct SinkPlaceT {
  static constexpr u32 kHist = kHistLds;
  u32 *lds_hist;  // set by the kernel
  u64 *mbits;
  u32 *ptindex;
  uint8_t *rank;
  u64 rank_stride;
  u64 *hist;
  FastMod pt, rk;
  u32 nranks;
  __device__ __forceinline__ void init() {
    if (hist && nranks <= kHistLds) {
      for (u32 r = threadIdx.x; r < nranks; r += blockDim.x) lds_hist[r] = 0;
      __syncthreads();
    }
  }
  __device__ __forceinline__ void put(u64 i, u64 h) {
    st<NTS>(h, mbits + i);
    if (ptindex) st<NTS>((u32)pt.mod(h), ptindex + i);
    if (rank || hist) {
      const u32 r = (u32)rk.mod(h);
      if (rank) st<NTS>(r, reinterpret_cast<u32 *>(rank + i * rank_stride));
      if (hist) {
        if (nranks <= kHistLds)
          atomicAdd(lds_hist + r, 1u);
        else
          atomicAdd(reinterpret_cast<unsigned long long *>(hist + r), 1ull);
      }
    }
  }
  __device__ __forceinline__ void flush() {
    if (hist && nranks <= kHistLds) {
      __syncthreads();
      // one device-scope atomic per bin per workgroup (a two-level variant,
      // partial rows + a reduce kernel, measured no faster: r01 placebench)
      for (u32 r = threadIdx.x; r < nranks; r += blockDim.x)
        if (lds_hist[r]) atomicAdd(reinterpret_cast<unsigned long long *>(hist + r), (unsigned long long)lds_hist[r]);
    }
  }
};
typedef SinkPlaceT<false> SinkPlace;
template <>
struct NtSink<SinkPlace> {
  typedef SinkPlaceT<true> type;
  static __host__ type make(SinkPlace s) {
    return type{s.lds_hist, s.mbits, s.ptindex, s.rank, s.rank_stride, s.hist, s.pt, s.rk, s.nranks};
  }
};

// ------------------------------------------------------------ key loads ---

template <bool NT, class T>
__device__ __forceinline__ T ld(const T *p) {
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <int L, bool NT = false>
__device__ __forceinline__ void load_key_regs(const uint8_t *__restrict__ keys, u64 i,
                                              RegReader<L / 4> &r) {
  static_assert(L == 8 || L % 16 == 0, "direct path: L = 8 or a multiple of 16");
  if constexpr (L == 8) {
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = ld<NT>(reinterpret_cast<const u32x2 *>(keys) + i);
    r.d[0] = v.x;
    r.d[1] = v.y;
  } else {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(keys + i * (u64)L);
#pragma unroll
    for (int j = 0; j < L / 16; ++j) {
      const u32x4 v = ld<NT>(p + j);
      r.d[4 * j + 0] = v.x;
      r.d[4 * j + 1] = v.y;
      r.d[4 * j + 2] = v.z;
      r.d[4 * j + 3] = v.w;
    }
  }}

// ------------------------------------------------------- direct kernel ---
// U keys per lane per iteration (all loads issued before any hashing).  BS =
// workgroup size: fused placement with a histogram uses 1024 so that a quarter
// as many workgroups flush their LDS bins with device-scope atomics.
template <int L, int U, class Algo, class Sink, bool NT = false, int BS = kBlock>
__global__ __launch_bounds__(BS) void k_fixed_direct(const uint8_t *__restrict__ keys, u64 n,
                                                     Algo algo, Sink sink) {
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  sink.init();
  const u64 stride = (u64)gridDim.x * BS;
  for (u64 i = (u64)blockIdx.x * BS + threadIdx.x; i < n; i += stride * U) {
    RegReader<L / 4> r[U];
    // unconditional (clamped) loads: a load under a lane-divergent branch is
    // followed by its own vmcnt(0), which would serialise the U keys
#pragma unroll
    for (int u = 0; u < U; ++u) load_key_regs<L, NT>(keys, min(i + u * stride, n - 1), r[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) sink.put(i + u * stride, algo(r[u], (u64)L));
  }
  sink.flush();
}

// -------------------------------------------------- LDS-transposed 64 B ---
// A wave's 64 keys (one contiguous 4 KiB tile) are brought in as fully
// contiguous 1 KiB pieces (piece j = bytes [1024j, 1024j+1024), lane l's
// 16 B = chunk g = 64j + l = key g>>2, quarter g&3) and transposed through a
// per-wave LDS image so each lane ends up with its own 64-byte key in VGPRs.
// Image slot of (key k, quarter c) = 4k + (c ^ ((k >> 2) & 3)): the XOR keeps
// the 16-lane groups of ds_read_b128 (row reads, lane = key) and the 8-lane
// groups of ds_write_b128 conflict-free.
__device__ __forceinline__ u32 xpose_slot(u32 k, u32 c) { return 4 * k + (c ^ ((k >> 2) & 3)); }

// LDS byte address of a __shared__ object (for hand-issued ds_* / M0).
template <class T>
__device__ __forceinline__ u32 lds_addr(const T *p) {
  return (u32)(uintptr_t)(const __attribute__((address_space(3))) T *)(p);
}

// Row read of lane `lane`'s key from an image at LDS byte address `img`,
// hand-issued so the compiler does not tie it to outstanding LDS-DMA (it
// would otherwise wait vmcnt(0) on every DMA in flight, prefetch included).
__device__ __forceinline__ void read_row_asm(u32 img, u32 lane, RegReader<16> &r) {
  const u32 sw = (lane >> 2) & 3;
  u32x4 v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const u32 a = img + 16 * (4 * lane + (c ^ sw));
    asm volatile("ds_read_b128 %0, %1" : "=v"(v[c]) : "v"(a) : "memory");
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    r.d[4 * c + 0] = v[c].x;
    r.d[4 * c + 1] = v[c].y;
    r.d[4 * c + 2] = v[c].z;
    r.d[4 * c + 3] = v[c].w;
  }}

// Variant "lds": pieces arrive by LDS-DMA (global_load_lds_dwordx4, no VGPR
// staging); the SOURCE address is permuted so that the linear DMA image is
// the swizzled one; the next tile's DMA is in flight while this one hashes.
template <class Algo, class Sink>
__global__ __launch_bounds__(kBlock) void k_fixed_lds64(const uint8_t *__restrict__ keys, u64 n,
                                                        Algo algo, Sink sink) {
  __shared__ __attribute__((aligned(16))) u32 tile[kWavesPerBlock][2][1024];  // 2 x 4 KiB per wave
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 full = n >> 6;  // tiles with 64 valid keys (DMA path)
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;

  auto issue = [&](u64 t, int b) {
    const uint8_t *base = keys + (t << 12);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32 g = 64 * j + lane;               // image slot this lane fills
      const u32 k = g >> 2, cq = g & 3;            // slot holds quarter cq ^ swz(k) of key k
      const uint8_t *src = base + k * 64 + ((cq ^ ((k >> 2) & 3)) << 4);
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)src,
                                       (void __attribute__((address_space(3))) *)&tile[wave][b][256 * j],
                                       16, 0, 0);
    }
  };

  u64 t = (u64)blockIdx.x * kWavesPerBlock + wave;
  int b = 0;
  if (t < full) issue(t, 0);
  for (; t < ntiles; t += nwaves) {
    const u64 tn = t + nwaves;
    const u64 i = (t << 6) + lane;
    RegReader<16> r;    if (t < full) {
      if (tn < full) {
        issue(tn, b ^ 1);  // next tile streams in while this one hashes
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      read_row_asm(lds_addr(&tile[wave][b][0]), lane, r);
    } else if (i < n) {
      load_key_regs<64>(keys, i, r);
    }
    if (i < n) sink.put(i, algo(r, (u64)64));
    b ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sink.flush();
}

// Variant "xpose": the same transpose with register staging: each lane loads
// 4 contiguous 16-B pieces of the NEXT tile (global_load_dwordx4, 1 KiB per
// wave-instruction) while the current tile hashes, then writes them into the
// image with ds_write_b128.
template <class Algo, class Sink, bool LNT = false, int DEPTH = 1>
__global__ __launch_bounds__(kBlock) void k_fixed_xpose64(const uint8_t *__restrict__ keys, u64 n,
                                                          Algo algo, Sink sink) {
  __shared__ __attribute__((aligned(16))) u32x4 img[kWavesPerBlock][256];  // 4 KiB per wave
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 full = n >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  // DEPTH tiles of prefetch in flight per wave (register sets, static index)
  u32x4 pre[DEPTH][4];
  auto fetch = [&](int d, u64 t) {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(keys + (t << 12));
#pragma unroll
    for (int j = 0; j < 4; ++j) pre[d][j] = ld<LNT>(src + 64 * j + lane);
  };
  const u64 t0 = (u64)blockIdx.x * kWavesPerBlock + wave;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (t0 + d * nwaves < full) fetch(d, t0 + d * nwaves);
  for (u64 t = t0; t < ntiles; t += DEPTH * nwaves) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const u64 tt = t + d * nwaves;
      if (tt >= ntiles) break;  // wave-uniform
      const u64 i = (tt << 6) + lane;
      RegReader<16> r;
      if (tt < full) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const u32 g = 64 * j + lane;
          img[wave][xpose_slot(g >> 2, g & 3)] = pre[d][j];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const u64 tn = tt + DEPTH * nwaves;
        if (tn < full) fetch(d, tn);  // refill this register set while hashing
        const u32 sw = (lane >> 2) & 3;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const u32x4 v = img[wave][4 * lane + (c ^ sw)];
          r.d[4 * c + 0] = v.x;
          r.d[4 * c + 1] = v.y;
          r.d[4 * c + 2] = v.z;
          r.d[4 * c + 3] = v.w;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      } else if (i < n) {
        load_key_regs<64>(keys, i, r);
      }
      if (i < n) sink.put(i, algo(r, (u64)64));
    }
  }
  sink.flush();
}

// --------------------------------------------- chunk-streamed long keys ---
// Fixed keys too long for a 64-key LDS window (keylen > 255 B; 16-B multiple
// length and stride, 16-B aligned rows), CityHash64 and its seeded form.  The
// >64-byte loop (city.c:236-260) consumes a key 64 bytes at a time, so a wave
// streams the s-th 64-byte chunk of each of its 64 keys through a 4 KiB LDS
// image per step: 4 LDS-DMA instructions of 16 keys x 64 B (the xpose64
// swizzle applied on the source side, as in k_fixed_lds64), double-buffered
// so chunk s+1 is in flight while chunk s is hashed, and each lane reads its
// row back with 4 ds_read_b128.  Step 0 is the tail [L-64, L) (tail-first
// initialisation), steps 1..R the chunks 0..R-1.  k_global (each lane walking
// its own key with per-lane loads) is the fallback for other lengths.
template <class A>
struct IsCity64Algo {
  static constexpr bool value = std::is_same<A, AlgoCity64>::value || std::is_same<A, AlgoCity64Seeds>::value;
};

template <class Algo, class Sink, int AUX = 0>
__global__ __launch_bounds__(kBlock) void k_fixed_chunks(const uint8_t *__restrict__ keys, u64 stride, u32 L,
                                                         u64 n, Algo algo, Sink sink) {
  __shared__ __attribute__((aligned(16))) u32 tile[kWavesPerBlock][2][1024];  // 2 x 4 KiB per wave
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  const u32 rounds = (L - 1) >> 6;
  // image slot g = 64j + lane holds quarter (g&3) ^ swz(k) of key k = g>>2
  auto issue = [&](u64 t, u32 off, int b) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32 g = 64 * j + lane;
      const u32 k = g >> 2, cq = g & 3;
      const u64 key = min((t << 6) + k, n - 1);
      const uint8_t *src = keys + key * stride + off + ((cq ^ ((k >> 2) & 3)) << 4);
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)src,
                                       (void __attribute__((address_space(3))) *)&tile[wave][b][256 * j], 16, 0,
                                       AUX);
    }
  };
  for (u64 t = (u64)blockIdx.x * kWavesPerBlock + wave; t < ntiles; t += nwaves) {
    const u64 i = (t << 6) + lane;
    issue(t, L - 64, 0);  // the tail
    issue(t, 0, 1);       // chunk 0
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    RegReader<16> r;
    read_row_asm(lds_addr(&tile[wave][0][0]), lane, r);
    LongState st;
    city64_long_init(r.template span<64>(0), L, st);
    for (u32 q = 0; q < rounds; ++q) {
      const int cb = (q + 1) & 1;  // chunk q sits in buffer (q+1)&1
      if (q + 1 < rounds) {
        issue(t, (q + 1) << 6, cb ^ 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      read_row_asm(lds_addr(&tile[wave][cb][0]), lane, r);
      const Words<16> c = r.template span<64>(0);
      if (q == 0) st.x += c.w64(0);  // "x * k1 + Fetch64(s)" (city.c:243)
      round64(st, c);
    }
    u64 h = city64_long_final(st);
    if constexpr (std::is_same<Algo, AlgoCity64Seeds>::value) h = mix16(h - algo.s0, algo.s1);
    if (i < n) sink.put(i, h);
  }
  sink.flush();
}

// --------------------------------------------------------- window kernel ---
// Any key length.  VAR: key i = bytes[offsets[i]-obase, offsets[i+1]-obase);
// otherwise key i = bytes[i*stride, i*stride+keylen).  WIN = LDS bytes per
// wave.  AUX = cache-policy bits of the LDS-DMA (2 = non-temporal).
template <int WIN, bool VAR, class Algo, class Sink, int AUX = 0>
__global__ __launch_bounds__(kBlock) void k_window(const uint8_t *__restrict__ bytes,
                                                   const u64 *__restrict__ offsets, u64 obase,
                                                   u64 stride, u64 keylen, u64 n, Algo algo,
                                                   Sink sink) {
  static_assert(WIN % 16 == 0, "window = whole 16-B DMA lanes");
  // Windows of the 4 waves back to back; a span's trailing dword read may run
  // past a window's end only when it is not used (aligned span), so only the
  // array as a whole needs the 16 B of slack.  WIN need not be a multiple of
  // 1 KiB: 10224 B keeps a workgroup under 40 KiB = 4 workgroups per CU.
  __shared__ __attribute__((aligned(16))) u32 win_all[kWavesPerBlock * (WIN / 4) + 4];
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  u32 *lds = win_all + wave * (WIN / 4);
  for (u64 t = (u64)blockIdx.x * kWavesPerBlock + wave; t < ntiles; t += nwaves) {
    const u64 k0 = t << 6;
    const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;  // one past the tile's last key
    const u64 i = k0 + lane;
    const bool valid = i < n;
    u64 start = 0, end = 0, whi;
    if constexpr (VAR) {
      if (valid) {
        start = offsets[i] - obase;
        end = offsets[i + 1] - obase;
      }
      whi = offsets[kend] - obase;
    } else {
      start = i * stride;
      end = start + keylen;
      whi = (kend - 1) * stride + keylen;
    }
    // One pass: the window starts at the tile's first key; keys that end
    // beyond WIN bytes (only in tiles of long keys) are read from global
    // memory instead (a multi-pass variant that re-staged the remainder was
    // measured slower: each extra pass is a serialised DMA round trip).
    u64 wlo;
    if constexpr (VAR)
      wlo = offsets[k0] - obase;
    else
      wlo = k0 * stride;
    wlo &= ~(u64)15;
    const u64 span = whi - wlo;
    const u32 wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
    // DMA the window: piece j moves 1 KiB, lane l's 16 B to LDS 1024j+16l.
    // 16-B-aligned pieces never cross a page the key bytes do not touch.
    const uint8_t *src = bytes + wlo;
#pragma unroll
    for (int j = 0; j < (WIN + 1023) / 1024; ++j) {
      if ((u32)j * 1024 < wbytes) {  // wave-uniform
        if ((u32)j * 1024 + lane * 16 < wbytes)
          __builtin_amdgcn_global_load_lds(
              (const void __attribute__((address_space(1))) *)(src + j * 1024 + lane * 16),
              (void __attribute__((address_space(3))) *)(lds + 256 * j), 16, 0, AUX);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const u64 len = end - start;
      typename Algo::Out h;
      if (end - wlo <= wbytes)
        h = algo(LdsReader{lds, (u32)(start - wlo)}, len);
      else
        h = algo(GlobalReader{bytes + start}, len);
      sink.put(i, h);
    }
    __builtin_amdgcn_wave_barrier();  // window reused by the next tile
  }
  sink.flush();
}

// ---------------------------------------------------------- long keys ---
// Keys far longer than a 64-key LDS window can hold (fixed L > 255 B): each
// lane walks its own key straight from global memory (GlobalReader); the
// other lanes' reads of the same 128-B lines arrive through L2.  VAR: key i =
// bytes[offsets[i]-obase, offsets[i+1]-obase); else bytes[i*stride, +keylen).
template <bool VAR, class Algo, class Sink, bool A16 = false>
__global__ __launch_bounds__(kBlock) void k_global(const uint8_t *__restrict__ bytes,
                                                   const u64 *__restrict__ offsets, u64 obase,
                                                   u64 stride, u64 keylen, u64 n, Algo algo,
                                                   Sink sink) {
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u64 step = (u64)gridDim.x * kBlock;
  for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += step) {
    u64 st, len;
    if constexpr (VAR) {
      st = offsets[i] - obase;
      len = offsets[i + 1] - obase - st;
    } else {
      st = i * stride;
      len = keylen;
    }
    sink.put(i, algo(GlobalReaderT<A16>{bytes + st}, len));
  }
  sink.flush();
}

// ------------------------------------------- double-buffered window kernel ---
// Offset-indexed keys.  k_window with two LDS windows per wave: while tile t
// hashes out of one window, the LDS-DMA of tile t+nwaves streams into the
// other, and the offsets of tile t+2*nwaves are already on their way.  The
// windows are two distinct __shared__ objects and the loop is unrolled by two,
// so every LDS read names its window and the compiler's LDS-DMA wait tracking
// (alias scopes per LDS object) only waits for the DMA into THAT window.
// Per tile, one vector load of offsets[k0+lane] (a key's end = its right
// neighbour's start) and one uniform load of offsets[kend].
template <int WIN>
struct WinGeo {
  u64 wlo;     // 16-B aligned window start (bytes index, relative to obase)
  u64 start;   // this lane's key
  u64 end;
  u32 wbytes;  // bytes staged (<= WIN)
};

template <int WIN, class Algo, class Sink, int AUX = 2>
__global__ __launch_bounds__(kBlock) void k_window2(const uint8_t *__restrict__ bytes,
                                                    const u64 *__restrict__ offsets, u64 obase,
                                                    u64 n, Algo algo, Sink sink) {
  static_assert(WIN % 16 == 0, "window = whole 16-B DMA lanes");
  __shared__ __attribute__((aligned(16))) u32 winA[kWavesPerBlock * (WIN / 4) + 4];
  __shared__ __attribute__((aligned(16))) u32 winB[kWavesPerBlock * (WIN / 4) + 4];
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  u32 *const wa = winA + wave * (WIN / 4);
  u32 *const wb = winB + wave * (WIN / 4);

  // offsets of tile t: this lane's start, and the tile's end (uniform)
  auto load_offs = [&](u64 t, u64 &a, u64 &hi) {
    const u64 k0 = t << 6;
    const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;
    a = offsets[(k0 + lane < n) ? k0 + lane : n];
    hi = offsets[kend];
  };
  auto geometry = [&](u64 a, u64 hi) {
    WinGeo<WIN> g;
    const u64 nb = __shfl_down(a, 1);
    g.start = a - obase;
    g.end = (lane == 63 ? hi : nb) - obase;
    // readfirstlane returns int: widen through u32 (no sign extension)
    const u64 a0 = (u64)(u32)__builtin_amdgcn_readfirstlane((u32)a) |
                   ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(a >> 32)) << 32);
    g.wlo = a0 - obase;
    g.wlo &= ~(u64)15;
    const u64 span = (hi - obase) - g.wlo;
    g.wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
    return g;
  };
  auto issue = [&](const WinGeo<WIN> &g, u32 *w) {
    const uint8_t *src = bytes + g.wlo;
#pragma unroll
    for (int j = 0; j < (WIN + 1023) / 1024; ++j) {
      if ((u32)j * 1024 < g.wbytes) {  // wave-uniform
        if ((u32)j * 1024 + lane * 16 < g.wbytes)
          __builtin_amdgcn_global_load_lds(
              (const void __attribute__((address_space(1))) *)(src + j * 1024 + lane * 16),
              (void __attribute__((address_space(3))) *)(w + 256 * j), 16, 0, AUX);
      }
    }
  };
  // a tile's digests are stored one step late, right after the next DMA is
  // issued: the wait at the top of a step then only covers operations issued
  // a whole tile of hashing earlier (on CDNA a load wait also waits for every
  // older store)
  typename Algo::Out h{};
  u64 hi_pend = ~0ull;  // index of the digest held in h (~0: none)
  auto hash = [&](u64 t, const WinGeo<WIN> &g, const u32 *w) {
    const u64 i = (t << 6) + lane;
    hi_pend = ~0ull;
    if (i < n) {
      const u64 len = g.end - g.start;
      if (g.end - g.wlo <= g.wbytes)
        h = algo(LdsReader{w, (u32)(g.start - g.wlo)}, len);
      else
        h = algo(GlobalReader{bytes + g.start}, len);
      hi_pend = i;
    }
  };
  auto put_pending = [&] {
    if (hi_pend != ~0ull) sink.put(hi_pend, h);
  };

  u64 t = (u64)blockIdx.x * kWavesPerBlock + wave;
  if (t < ntiles) {
    u64 a, hi, an, hin;
    load_offs(t, a, hi);
    WinGeo<WIN> g = geometry(a, hi), gn;
    issue(g, wa);
    // offsets loads are unconditional (clamped tile): a conditional load
    // merges with the old value through a register copy, and the copy waits
    // vmcnt(0) for the DMA issued just before it
    const u64 last = ntiles - 1;
    load_offs(min(t + nwaves, last), an, hin);
    // one step: hash tile t out of `cur` while tile t+nwaves streams into `nxt`
    auto step = [&](u32 *cur, u32 *nxt) -> bool {
      const u64 tn = t + nwaves;
      const bool more = tn < ntiles;  // wave-uniform
      // tile t's DMA (issued one step ago) has landed; the compiler does not
      // order LDS reads after LDS-DMA by itself, so this wait is what makes
      // `cur` readable (it also covers the offsets loads of the same step)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (more) {
        gn = geometry(an, hin);
        issue(gn, nxt);
      }
      put_pending();
      if (more) load_offs(min(tn + nwaves, last), an, hin);
      hash(t, g, cur);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // `cur` is the DMA target two tiles on
      g = gn;
      t = tn;
      return more;
    };
    while (step(wa, wb) && step(wb, wa)) {
    }
    put_pending();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sink.flush();
}

// ------------------------------------------------- pipelined window kernel ---
// k_window with the next tile's window prefetched into VGPRs (WIN/1024
// global_load_dwordx4 per lane, contiguous 1 KiB per wave-instruction) while
// the current tile hashes out of LDS; the prefetched pieces are written into
// the (single) per-wave LDS window with ds_write_b128 at the top of the next
// iteration.  Ordinary loads, so the compiler's waits stay exact (LDS-DMA
// would make it drain every outstanding DMA before each LDS read).
template <int WIN, bool VAR, class Algo, class Sink>
__global__ __launch_bounds__(kBlock) void k_window_pf(const uint8_t *__restrict__ bytes,
                                                      const u64 *__restrict__ offsets, u64 obase,
                                                      u64 stride, u64 keylen, u64 n, Algo algo,
                                                      Sink sink) {
  static_assert(WIN % 1024 == 0, "window = whole 1 KiB pieces");
  constexpr int P = WIN / 1024;
  __shared__ __attribute__((aligned(16))) u32 win[kWavesPerBlock][WIN / 4 + 4];
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  u32 *lds = win[wave];
  u32x4 *lds4 = reinterpret_cast<u32x4 *>(lds);

  struct Tile {
    u64 wlo;      // 16-B aligned window start (byte offset into `bytes`)
    u32 wbytes;   // bytes of the window actually staged (<= WIN)
    u64 start, end;
  };
  auto geometry = [&](u64 t) {
    Tile g;
    const u64 k0 = t << 6;
    const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;
    const u64 i = k0 + lane;
    u64 whi;
    if constexpr (VAR) {
      g.wlo = (offsets[k0] - obase) & ~(u64)15;
      whi = offsets[kend] - obase;
      g.start = i < n ? offsets[i] - obase : 0;
      g.end = i < n ? offsets[i + 1] - obase : 0;
    } else {
      g.wlo = (k0 * stride) & ~(u64)15;
      whi = (kend - 1) * stride + keylen;
      g.start = i * stride;
      g.end = g.start + keylen;
    }
    const u64 span = whi - g.wlo;
    g.wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
    return g;
  };
  u32x4 pre[P];
  auto prefetch = [&](const Tile &g) {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(bytes + g.wlo) + lane;
#pragma unroll
    for (int j = 0; j < P; ++j)
      if ((u32)j * 1024 + lane * 16 < g.wbytes) pre[j] = __builtin_nontemporal_load(src + 64 * j);
  };

  u64 t = (u64)blockIdx.x * kWavesPerBlock + wave;
  Tile cur{};
  if (t < ntiles) {
    cur = geometry(t);
    prefetch(cur);
  }
  for (; t < ntiles; t += nwaves) {
#pragma unroll
    for (int j = 0; j < P; ++j)
      if ((u32)j * 1024 + lane * 16 < cur.wbytes) lds4[64 * j + lane] = pre[j];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const Tile g = cur;
    const u64 tn = t + nwaves;
    if (tn < ntiles) {  // next tile streams in while this one hashes
      cur = geometry(tn);
      prefetch(cur);
    }
    const u64 i = (t << 6) + lane;
    if (i < n) {
      const u64 len = g.end - g.start;
      typename Algo::Out h;
      if (g.end - g.wlo <= g.wbytes)
        h = algo(LdsReader{lds, (u32)(g.start - g.wlo)}, len);
      else
        h = algo(GlobalReader{bytes + g.start}, len);
      sink.put(i, h);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the window is rewritten by the next tile
  }
  sink.flush();
}

// ------------------------------------------------ class-sorted var keys ---
// Cost class of a key: which code path CityHash takes (city.c:225-233) and,
// for long keys, how many 64-byte rounds (city.c:246).
__device__ __forceinline__ u32 len_class(u64 len) {
  if (len <= 16) return 0;
  if (len <= 32) return 1;
  if (len <= 64) return 2;
  const u64 r = (len - 1) >> 6;  // 1.. rounds
  return r >= 4 ? 6u : (u32)(2 + r);
}

// Variable-length keys, block tiles of 256 keys.  The tile's contiguous byte
// range is DMA'd into one LDS window shared by the block; the tile's keys are
// counting-sorted by cost class in LDS and thread t hashes the t-th key of
// that order, so a wave runs (mostly) one code path with one trip count
// instead of every path its 64 lanes' lengths touch.  Digests go back to
// their original index.  Keys not inside the window (tile bytes > WINB) are
// read from global memory.
template <int WINB, class Algo, class Sink>
__global__ __launch_bounds__(kBlock) void k_var_sorted(const uint8_t *__restrict__ bytes,
                                                       const u64 *__restrict__ offsets, u64 obase,
                                                       u64 n, Algo algo, Sink sink) {
  static_assert(WINB % 1024 == 0, "window = whole 1 KiB DMA pieces");
  __shared__ __attribute__((aligned(16))) u32 win[WINB / 4 + 4];
  __shared__ u32 s_rel[kBlock], s_len[kBlock], s_perm[kBlock], s_cnt[8];
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u32 tid = threadIdx.x;
  const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u32 lane = tid & 63;
  const u64 ntiles = (n + kBlock - 1) / kBlock;
  for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const u64 k0 = t * kBlock;
    const u64 kend = (k0 + kBlock < n) ? k0 + kBlock : n;
    const u64 i = k0 + tid;
    const bool valid = i < n;
    const u64 wlo = (offsets[k0] - obase) & ~(u64)15;
    const u64 whi = offsets[kend] - obase;
    const u64 span = whi - wlo;
    const u32 wbytes = span < (u64)WINB ? (u32)span : (u32)WINB;
    // DMA the window: pieces of 1 KiB, wave w takes pieces w, w+4, ...
    const uint8_t *src = bytes + wlo;
    for (u32 j = wave; j * 1024 < wbytes; j += kWavesPerBlock) {
      if (j * 1024 + lane * 16 < wbytes)
        __builtin_amdgcn_global_load_lds(
            (const void __attribute__((address_space(1))) *)(src + j * 1024 + lane * 16),
            (void __attribute__((address_space(3))) *)(win + 256 * j), 16, 0, 0);
    }
    // key geometry + class while the DMA is in flight
    u32 cls = 7;
    if (valid) {
      const u64 st = offsets[i] - obase, en = offsets[i + 1] - obase;
      s_rel[tid] = (u32)(st - wlo);
      s_len[tid] = (u32)(en - st);
      cls = len_class(en - st);
    }
    if (tid < 8) s_cnt[tid] = 0;
    __syncthreads();
    const u32 pos = atomicAdd(&s_cnt[cls], 1u);
    __syncthreads();
    u32 base = 0;
#pragma unroll
    for (u32 c = 0; c < 7; ++c) base += (c < cls) ? s_cnt[c] : 0u;
    s_perm[base + pos] = tid;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < kend - k0) {
      const u32 me = s_perm[tid];
      const u32 rel = s_rel[me], len = s_len[me];
      typename Algo::Out h;
      if (span <= 0xffffffffull && (u64)rel + len <= wbytes) {
        h = algo(LdsReader{win, rel}, (u64)len);
      } else {  // outside the window: straight from global memory
        h = algo(GlobalReader{bytes + (offsets[k0 + me] - obase)}, (u64)len);
      }
      sink.put(k0 + me, h);
    }
    __syncthreads();  // window, perm and geometry are rewritten by the next tile
  }
  sink.flush();
}

// ------------------------------------------------- synthetic workloads ---
__global__ __launch_bounds__(kBlock) void k_splitmix64(u64 seed, u64 first, u64 nwords, u64 *out);
__global__ __launch_bounds__(kBlock) void k_mixed_lengths(u64 seed, u64 first, u64 n, u32 lo,
                                                          u32 span, u64 *lens);

}  // namespace pdht
