// kernels.h -- gfx950 kernels of the batch key-hashing engine.
//
// Layout of the work:
//   * one key per lane, 64 keys per wave, digests stored lane-contiguous
//     (8 B or 16 B per lane -> 512 B / 1 KiB per wave-instruction);
//   * k_fixed_direct<L>: packed keys of a compile-time length L (8/16/32):
//     each lane pulls its own key straight into VGPRs, U keys in flight, the
//     algorithm runs with every offset constant-folded;
//   * k_fixed_xpose64: packed 64-byte keys: the wave's contiguous 4 KiB tile
//     arrives as 4 x 1 KiB global_load_dwordx4 (two tiles of prefetch in
//     flight) and is transposed through a swizzled per-wave LDS image so each
//     lane holds its own key in VGPRs;
//   * k_window: any key length, fixed stride or offset-indexed: the wave's
//     contiguous byte range is DMA'd into a per-wave LDS window and each lane
//     hashes its key out of LDS with unaligned ds_read_b128 spans; keys that
//     do not fit the window are read from global memory directly;
//   * k_global: fixed keys too long for a 64-key window, each lane walking
//     its own key in global memory.
// All kernels are grid-stride persistent loops (grid ~ CUs x residency) and
// carry no inter-workgroup communication.
#pragma once

#include <type_traits>

#include "city_core.h"

namespace pdht {

typedef u32 u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;  // 4 waves
constexpr int kWavesPerBlock = kBlock / 64;

// Orders one wave's LDS writes before its later LDS reads (and the reverse)
// without a workgroup barrier: waves own their LDS regions.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// --------------------------------------------------------------- readers ---
// Key bytes in LDS at an arbitrary byte offset (product, r04): spans as
// UNALIGNED LDS loads.  gfx950 serves ds_read_b128 / ds_read_b64 /
// ds_read_b32 at any byte address (HSA runs with unaligned access mode;
// hipcc emits them for under-aligned LDS types on its own), so a span needs
// no v_alignbyte_b32 at all -- 64 B = 4 ds_read_b128 instead of 9
// ds_read2_b32 + 16 VALU funnel shifts (window kernel: static VALU 1145 ->
// 1030; cfg3 +2.5 / +2.8 % on two boxes, interleaved, profiles/r04/ab/).
// Reads stay inside the key's bytes.
struct LdsReader {
  const u32 *lds;
  u32 base;
  template <int N>
  __device__ __forceinline__ Words<N / 4> span(u32 o) const {
    typedef u32x4 u32x4u __attribute__((aligned(1)));
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    typedef u32x2 u32x2u __attribute__((aligned(1)));
    typedef u32 u32u __attribute__((aligned(1)));
    const uint8_t *p = reinterpret_cast<const uint8_t *>(lds) + base + o;
    Words<N / 4> w;
#pragma unroll
    for (int j = 0; j < N / 16; ++j) {
      const u32x4 v = *reinterpret_cast<const u32x4u *>(p + 16 * j);
      w.d[4 * j + 0] = v.x;
      w.d[4 * j + 1] = v.y;
      w.d[4 * j + 2] = v.z;
      w.d[4 * j + 3] = v.w;
    }
    if constexpr (N % 16 >= 8) {
      const u32x2 v = *reinterpret_cast<const u32x2u *>(p + N / 16 * 16);
      w.d[N / 16 * 4] = v.x;
      w.d[N / 16 * 4 + 1] = v.y;
    }
    if constexpr (N % 8 == 4) w.d[N / 4 - 1] = *reinterpret_cast<const u32u *>(p + N - 4);
    return w;
  }
  __device__ __forceinline__ u32 w32(u32 o) const { return span<4>(o).d[0]; }
  __device__ __forceinline__ u32 b8(u32 o) const {
    return reinterpret_cast<const uint8_t *>(lds)[base + o];
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
// A16: every key starts 16-B aligned (fixed keys, aligned base and stride):
// spans at 16-B aligned offsets load as dwordx4, a quarter of the
// instructions (the CRC-256 rounds read 240-B blocks at multiples of 240).
// NT = kLongLines (the long-key kernels): every span a lane reads covers
// whole 128-B lines of its key where the algorithm allows -- CityHash64's
// long loop two rounds (128 B) per span (kPairs), CityHashCrc256's 240-B
// blocks with the line remainder carried in registers (kLines) -- and 8-B
// aligned spans load as dwordx2.  A lane's 8 dwordx4 pieces of one line then
// leave together and meet in L2; split over two spans a compute round apart,
// the line was fetched twice (tools/abbench.py long64: 0.577 -> 0.679, long:
// 0.530 -> 0.567).  (r02 also measured non-temporal span loads -- 2x
// slower: every 16-B piece refetched its line -- and CityHash128's 16-B
// shifted loop on line spans -- 5 % slower; both removed in r03.)
constexpr int kLongLines = 5;
// NT = kLongStream (r04): as kLongLines for CityHash64 and CityHash128, and
// CityHashCrc256Long's block loop as a stream of whole 128-B lines
// (city_core.h crc256_stream_blocks) instead of 256-B line spans.
constexpr int kLongStream = 6;
template <bool A16 = false, int NT = 0>
struct GlobalReaderT {
  static constexpr bool kLines = NT == kLongLines;
  static constexpr bool kPairs = NT == kLongLines || NT == kLongStream;
  static constexpr bool kStream = A16 && NT == kLongStream;
  const uint8_t *p;
  // N bytes at o (16-B aligned key and offset), only the 16-B pieces that
  // start below lim (the rest zero): a key's last partial line without a
  // read past round16(len), which the 16-B aligned row stride still covers
  template <int N>
  __device__ __forceinline__ Words<N / 4> line_lim(u32 o, u32 lim) const {
    static_assert(N % 16 == 0, "whole 16-B pieces");
    gu32x4 *q = reinterpret_cast<gu32x4 *>(reinterpret_cast<uintptr_t>(p + o));
    Words<N / 4> w;
#pragma unroll
    for (int j = 0; j < N / 16; ++j) {
      const u32x4 v = o + 16 * j < lim ? q[j] : u32x4{0, 0, 0, 0};
      w.d[4 * j + 0] = v.x;
      w.d[4 * j + 1] = v.y;
      w.d[4 * j + 2] = v.z;
      w.d[4 * j + 3] = v.w;
    }
    return w;
  }
  template <int N>
  __device__ __forceinline__ Words<N / 4> span(u32 o) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    if constexpr (A16 && NT == kLongLines && N % 8 == 0 && N % 16 != 0) {
      if ((a & 7) == 0) {
        typedef u32 u32x2 __attribute__((ext_vector_type(2)));
        typedef const __attribute__((address_space(1))) u32x2 gu32x2;
        gu32x2 *q = reinterpret_cast<gu32x2 *>(a);
        Words<N / 4> w;
#pragma unroll
        for (int j = 0; j < N / 8; ++j) {
          const u32x2 v = q[j];
          w.d[2 * j] = v.x;
          w.d[2 * j + 1] = v.y;
        }
        return w;
      }
    }
    if constexpr (A16 && N % 16 == 0) {
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

// CRC-32C tables in LDS for batches that may hold keys > 900 B
// (CityHashCrc256 path, city.c:407-517): the slicing-by-8 byte tables below,
// 8 KiB per workgroup.  r02's 6-bit-slice tables (city_core.h Crc32c6Tables,
// 11 x 64 entries, conflict-free but 11 lookups per word; tuning/ variant
// 150) and 5-bit slices measured slower on the r03 line-span kernel, which
// spends more on VALU than on bank conflicts; from constant memory the
// lookups are per-lane vector loads through the TA, 4x slower.
// The product form (r03): plain slicing-by-8 byte tables (8 KiB, one copy),
// each address one byte select: 8 lookups of ~2 VALU per word against the
// 6-bit form's 11 of ~3.  Byte-indexed tables conflict in LDS (+72 % bank
// conflicts), but the long-key loop is VALU-heavy and the byte tables run
// 3-4 % faster (interleaved, `profiles/r03/ab/long_bytetab_*.log`).
// Late r05: the eight lookups are folded with gfx950's three-input v_bitop3
// (XOR3) -- 4 VALU instead of 7 per word; the long-key loop spends most of
// its VALU on these folds (PDHT_CRC_XOR3=0: the plain xor chain, A/B only).
#ifndef PDHT_CRC_XOR3
#define PDHT_CRC_XOR3 1
#endif
__device__ __forceinline__ u32 xor3(u32 a, u32 b, u32 c) {
#if PDHT_CRC_XOR3
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // truth table of a ^ b ^ c
#else
  return a ^ b ^ c;
#endif
}
struct CrcLdsByteTab {
  const u32 *t;  // [8][256], table k for byte k of the word (= slice-8 table 7-k)
  __device__ __forceinline__ u32 rd(u32 k, u32 b) const { return t[256 * k + b]; }
  __device__ __forceinline__ u32 crc64(u64 x) const {
    const u32 lo = (u32)x, hi = (u32)(x >> 32);
    const u32 a = xor3(rd(0, lo & 255), rd(1, (lo >> 8) & 255), rd(2, (lo >> 16) & 255));
    const u32 b = xor3(rd(3, lo >> 24), rd(4, hi & 255), rd(5, (hi >> 8) & 255));
    return xor3(a, b, rd(6, (hi >> 16) & 255) ^ rd(7, hi >> 24));
  }
};

template <int SB>
struct CrcLdsSlices;
template <>
struct CrcLdsSlices<8> {  // CrcLdsByteTab: the product tables
  typedef CrcLdsByteTab Tab;
  static constexpr u32 kWords = 8 * 256;
  __device__ static void fill(u32 *tab) {
    for (u32 k = threadIdx.x; k < kWords; k += blockDim.x) tab[k] = kCrcDev.t[7 - (k >> 8)][k & 255];
  }
  __device__ __forceinline__ static Tab make(const u32 *t) { return Tab{t}; }
};
constexpr int kCrcSlices = 8;  // the product's CRC-32C tables
template <class Base, int SB = kCrcSlices>
struct CrcLds : Base {
  static constexpr bool kCrcLds = true;
  typedef CrcLdsSlices<SB> Slices;
  const u32 *tab = nullptr;  // set by algo_init() inside the kernel
  template <class R>
  __device__ __forceinline__ typename Base::Out operator()(const R &r, u64 len) const {
    const auto T = Slices::make(tab);
    if constexpr (std::is_same<Base, AlgoCrc128>::value)
      return crc128(r, len, T);
    else
      return crc128_seed(r, len, u128{this->lo, this->hi}, T);
  }
};

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
    typedef typename Algo::Slices S;
    __shared__ __attribute__((aligned(16))) u32 tab[S::kWords];
    S::fill(tab);
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
  __host__ Sink64T shift(u64 k0) const { return Sink64T{lds_hist, out + k0}; }  // keys from k0 on
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
  __host__ Sink128T shift(u64 k0) const { return Sink128T{lds_hist, out + 2 * k0}; }
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
  __host__ SinkPlaceT shift(u64 k0) const {
    SinkPlaceT s = *this;
    s.mbits += k0;
    if (s.ptindex) s.ptindex += k0;
    if (s.rank) s.rank += k0 * s.rank_stride;
    return s;
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

// Variant "xpose": the same transpose with register staging: each lane loads
// 4 contiguous 16-B pieces of the NEXT tile (global_load_dwordx4, 1 KiB per
// wave-instruction) while the current tile hashes, then writes them into the
// image with ds_write_b128.
template <class Algo, class Sink, bool LNT = false, int DEPTH = 1, int BLOCK = kBlock, int PRIO = 0>
__global__ __launch_bounds__(BLOCK) void k_fixed_xpose64(const uint8_t *__restrict__ keys, u64 n,
                                                         Algo algo, Sink sink) {
  constexpr int kWavesPerBlock = BLOCK / 64;
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
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(PRIO);
        if (tn < full) fetch(d, tn);  // refill this register set while hashing
        if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
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

// --------------------------------------------------------- window kernel ---
// Any key length.  VAR: key i = bytes[offsets[i]-obase, offsets[i+1]-obase);
// otherwise key i = bytes[i*stride, i*stride+keylen).  WIN = LDS bytes per
// wave.  AUX = cache-policy bits of the LDS-DMA (2 = non-temporal).
// PRIO (tuning): the wave raises its issue priority while it fetches the
// next tile's offsets and issues the window DMA, and drops it to hash.
template <int WIN, bool VAR, class Algo, class Sink, int AUX = 0, int ALIGN = 16, class LR = LdsReader,
          int PRIO = 0>
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
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(PRIO);
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
    // Window bounds are ABSOLUTE addresses: wlo is the 16-B block holding the
    // tile's first key byte, so every 16-B DMA piece below lies in a block
    // that holds key bytes, and no piece reaches a page the keys do not
    // touch, whatever the alignment of `bytes` (zero-copy host buffers).
    const u64 base = (u64)(uintptr_t)bytes;
    u64 first;
    if constexpr (VAR)
      first = offsets[k0] - obase;
    else
      first = k0 * stride;
    const u64 wlo = (base + first) & ~(u64)(ALIGN - 1);
    const u64 span = whi > first ? base + whi - wlo : 0;  // a tile of empty keys reads nothing
    const u32 wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
    // DMA the window: piece j moves 1 KiB, lane l's 16 B to LDS 1024j+16l.
    const uint8_t *src = reinterpret_cast<const uint8_t *>((uintptr_t)wlo);
#pragma unroll
    for (int j = 0; j < (WIN + 1023) / 1024; ++j) {
      if ((u32)j * 1024 < wbytes) {  // wave-uniform
        if ((u32)j * 1024 + lane * 16 < wbytes)
          __builtin_amdgcn_global_load_lds(
              (const void __attribute__((address_space(1))) *)(src + j * 1024 + lane * 16),
              (void __attribute__((address_space(3))) *)(lds + 256 * j), 16, 0, AUX);
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const u64 len = end - start;
      typename Algo::Out h;
      if (base + end - wlo <= wbytes)
        h = algo(LR{lds, (u32)(base + start - wlo)}, len);
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
template <bool VAR, class Algo, class Sink, bool A16 = false, int NT = 0>
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
    sink.put(i, algo(GlobalReaderT<A16, NT>{bytes + st}, len));
  }
  sink.flush();
}

// ------------------------------------------------- synthetic workloads ---
__global__ __launch_bounds__(kBlock) void k_splitmix64(u64 seed, u64 first, u64 nwords, u64 *out);
__global__ __launch_bounds__(kBlock) void k_mixed_lengths(u64 seed, u64 first, u64 n, u32 lo,
                                                          u32 span, u64 *lens);

}  // namespace pdht
