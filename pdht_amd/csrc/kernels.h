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
//     hashes its key out of LDS with byte-aligned fetches
//     (v_alignbyte_b32); keys that do not fit the window are read from
//     global memory directly;
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
// 0.530 -> 0.567).
// Tuning only: 1 = every dwordx4 span load non-temporal (2x slower: each
// 16-B piece refetches its line); 2 = all but the span's last 128 B; 3 =
// kLines alone; 4 = kPairs alone; 7 = kLongLines + CityHash128's 16-B
// shifted loop on line spans as well (carry in registers); 6 = 7 with the
// carry in one register array (moves on the loop's back edge).
constexpr int kLongLines = 5;
template <bool A16 = false, int NT = 0>
struct GlobalReaderT {
  static constexpr bool kLines = NT == 3 || NT == 7 || NT == kLongLines;
  static constexpr bool kPairs = NT == 4 || NT == 6 || NT == 7 || NT == kLongLines;
  static constexpr bool kOneCarry = NT == 6;
  static constexpr bool kLines16 = NT == 6 || NT == 7;
  const uint8_t *p;
  template <int N>
  __device__ __forceinline__ Words<N / 4> span(u32 o) const {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p + o);
    if constexpr (A16 && (NT == 3 || NT == kLongLines) && N % 8 == 0 && N % 16 != 0) {
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
          const u32x4 v = (NT == 1 || (NT == 2 && j < N / 16 - 8)) ? __builtin_nontemporal_load(q + j) : q[j];
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
// (CityHashCrc256 path, city.c:407-517): the 5-bit-slice tables of
// city_core.h, 13 x 32 entries = 1664 B per workgroup, every lookup
// conflict-free.  (r01 kept the slicing-by-8 tables here, 8 KiB: one lookup
// per byte but 4.3x bank conflicts; from constant memory those lookups are
// per-lane vector loads through the TA, 4x slower again.)
struct CrcLdsTab {
  const u32 *t;  // [13][32]
  __device__ __forceinline__ u32 crc64(u64 x) const {
    const u32 lo = (u32)x, hi = (u32)(x >> 32);
    u32 r = t[0 * 32 + (lo & 31)] ^ t[1 * 32 + ((lo >> 5) & 31)] ^ t[2 * 32 + ((lo >> 10) & 31)] ^
            t[3 * 32 + ((lo >> 15) & 31)] ^ t[4 * 32 + ((lo >> 20) & 31)] ^ t[5 * 32 + ((lo >> 25) & 31)];
    r ^= t[6 * 32 + (__builtin_amdgcn_alignbit(hi, lo, 30) & 31)];
    r ^= t[7 * 32 + ((hi >> 3) & 31)] ^ t[8 * 32 + ((hi >> 8) & 31)] ^ t[9 * 32 + ((hi >> 13) & 31)] ^
         t[10 * 32 + ((hi >> 18) & 31)] ^ t[11 * 32 + ((hi >> 23) & 31)] ^ t[12 * 32 + (hi >> 28)];
    return r;
  }
};
// The 6-bit-slice form (city_core.h Crc32c6Tables): 11 lookups per word.
struct CrcLds6Tab {
  const u32 *t;  // [11][64]
  __device__ __forceinline__ u32 crc64(u64 x) const {
    const u32 lo = (u32)x, hi = (u32)(x >> 32);
    u32 r = t[0 * 64 + (lo & 63)] ^ t[1 * 64 + ((lo >> 6) & 63)] ^ t[2 * 64 + ((lo >> 12) & 63)] ^
            t[3 * 64 + ((lo >> 18) & 63)] ^ t[4 * 64 + ((lo >> 24) & 63)];
    r ^= t[5 * 64 + (__builtin_amdgcn_alignbit(hi, lo, 30) & 63)];
    r ^= t[6 * 64 + ((hi >> 4) & 63)] ^ t[7 * 64 + ((hi >> 10) & 63)] ^ t[8 * 64 + ((hi >> 16) & 63)] ^
         t[9 * 64 + ((hi >> 22) & 63)] ^ t[10 * 64 + (hi >> 28)];
    return r;
  }
};
template <int SB>
struct CrcLdsSlices;
template <>
struct CrcLdsSlices<5> {
  typedef CrcLdsTab Tab;
  static constexpr u32 kWords = 13 * 32;
  __device__ static u32 word(u32 k) { return kCrc5Dev.t[k >> 5][k & 31]; }
};
template <>
struct CrcLdsSlices<6> {
  typedef CrcLds6Tab Tab;
  static constexpr u32 kWords = 11 * 64;
  __device__ static u32 word(u32 k) { return kCrc6Dev.t[k >> 6][k & 63]; }
};

template <class Base, int SB = 6>
struct CrcLds : Base {
  static constexpr bool kCrcLds = true;
  typedef CrcLdsSlices<SB> Slices;
  const u32 *tab = nullptr;  // set by algo_init() inside the kernel
  template <class R>
  __device__ __forceinline__ typename Base::Out operator()(const R &r, u64 len) const {
    typedef typename Slices::Tab Tab;
    if constexpr (std::is_same<Base, AlgoCrc128>::value)
      return crc128(r, len, Tab{tab});
    else
      return crc128_seed(r, len, u128{this->lo, this->hi}, Tab{tab});
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
    __shared__ u32 tab[S::kWords];
    for (u32 k = threadIdx.x; k < S::kWords; k += blockDim.x) tab[k] = S::word(k);
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

#ifdef PDHT_HIP_TUNING
// Tuning-only calibrations of the variable-length window kernel: the digest
// is the key length (no key byte is read from LDS), so the kernel is its
// window DMA, offsets loads and digest stores alone.
struct AlgoLenOnly {
  typedef u64 Out;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &, u64 len) const {
    return len;
  }
};
// Timing only: CityHash64 twice per key (the second over the key minus its
// first byte), to see what the hash arithmetic itself costs a kernel.
struct AlgoCity64x2 {
  typedef u64 Out;
  template <class R>
  __device__ __forceinline__ Out operator()(const R &r, u64 len) const {
    return city64(r, len) ^ (len ? city64(Shifted<R>{r, 1u}, len - 1) : 0);
  }
};
#endif

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
template <class Algo, class Sink, bool LNT = false, int DEPTH = 1, int BLOCK = kBlock>
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

// --------------------------------------------------------- window kernel ---
// Any key length.  VAR: key i = bytes[offsets[i]-obase, offsets[i+1]-obase);
// otherwise key i = bytes[i*stride, i*stride+keylen).  WIN = LDS bytes per
// wave.  AUX = cache-policy bits of the LDS-DMA (2 = non-temporal).
template <int WIN, bool VAR, class Algo, class Sink, int AUX = 0, int ALIGN = 16>
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
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const u64 len = end - start;
      typename Algo::Out h;
      if (base + end - wlo <= wbytes)
        h = algo(LdsReader{lds, (u32)(base + start - wlo)}, len);
      else
        h = algo(GlobalReader{bytes + start}, len);
      sink.put(i, h);
    }
    __builtin_amdgcn_wave_barrier();  // window reused by the next tile
  }
  sink.flush();
}

// ---------------------------- digest stores that never need a branch ---
// A tile's digests through a buffer resource whose size is the tile's valid
// digests: lanes past the batch's end store out of range and the hardware
// drops the store, so the store is ONE unconditional instruction per tile.
// (A store under a lane-divergent branch may be skipped by the wave, and the
// compiler can then no longer count it: every later load wait became
// vmcnt(0), which also waited for the stores.)  Word 3 = 0x00020000 for
// gfx9 (ck/ck.hpp CK_BUFFER_RESOURCE_3RD_DWORD).
template <class Sink>
struct BufStore {
  static constexpr bool kOk = false;
};
template <bool NTS>
struct BufStore<Sink64T<NTS>> {
  static constexpr bool kOk = true;
  __device__ static void put(const Sink64T<NTS> &s, u64 k0, u64 cnt, u32 lane, u64 h) {
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(s.out + k0, 0, (int)(cnt * 8), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{(u32)h, (u32)(h >> 32)}, r, (int)(lane * 8), 0, NTS ? 2 : 0);
  }
};
template <bool NTS>
struct BufStore<Sink128T<NTS>> {
  static constexpr bool kOk = true;
  __device__ static void put(const Sink128T<NTS> &s, u64 k0, u64 cnt, u32 lane, u128 h) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(s.out + 2 * k0, 0, (int)(cnt * 16), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{(u32)h.lo, (u32)(h.lo >> 32), (u32)h.hi, (u32)(h.hi >> 32)}, r,
                                           (int)(lane * 16), 0, NTS ? 2 : 0);
  }
};

// --------------------------- window kernel, next window in registers (var) ---
// Offset-indexed keys, one 64-key tile per wave as in k_window, with the
// NEXT tile's window travelling in VGPRs while this one hashes: the window
// of tile t+nw (NP dwordx4 global loads per lane, 1 KiB per wave-instruction,
// non-temporal) is issued right after tile t's window has been copied from
// registers into the wave's LDS window, so the memory latency of every window
// hides under a tile of hashing, at the LDS footprint of the single window
// (4 workgroups per CU).  Offsets run two tiles ahead.  Everything on the
// common path is straight-line so the compiler can count the memory
// operations: the window loads are global (not flat) loads with addresses
// clamped into the window (no branch), the copy writes all NP pieces, and
// the digests leave through one unconditional buffer store (BufStore).  The
// wait for tile t+nw's registers then covers only loads issued a whole tile
// of hashing earlier -- not this tile's digest stores.  (k_window_rp, the r02
// form of the idea, loaded through flat pointers and stored under a branch:
// every wait was vmcnt(0), and it measured no faster than k_window.)
template <int WS, class Algo, class Sink>
__global__ __launch_bounds__(kBlock) void k_window_pf(const uint8_t *__restrict__ bytes,
                                                      const u64 *__restrict__ offsets, u64 obase, u64 n, Algo algo,
                                                      Sink sink) {
  // WS = LDS bytes per wave, a whole number of 1 KiB pieces; the window
  // holds WS - 16 bytes of keys (the last 16 B are the slack of the span
  // reads), so 4 waves x 10 KiB fill 40 KiB: 4 workgroups per CU.  Digest
  // sinks only: no LDS histogram is declared.
  static_assert(WS % 1024 == 0, "window = whole 1 KiB pieces");
  static_assert(BufStore<Sink>::kOk, "digest sinks only");
  constexpr int NP = WS / 1024;
  constexpr u32 WIN = WS - 16;
  __shared__ __attribute__((aligned(16))) u32 win_all[kWavesPerBlock * (WS / 4)];
  algo_init(algo);
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  u32 *const lds = win_all + wave * (WS / 4);
  u32x4 *const lds4 = reinterpret_cast<u32x4 *>(lds);
  const u64 base = (u64)(uintptr_t)bytes;
  const u64 lastt = ntiles - 1;
  // a tile's offsets, both vector loads (a scalar load would make every LDS
  // wait of the hash an lgkmcnt(0)): this lane's key is [a, e)
  auto load_offs = [&](u64 t, u64 &a, u64 &e) {
    const u64 k = (t << 6) + lane;
    a = offsets[k < n ? k : n];
    e = offsets[k + 1 < n ? k + 1 : n];
  };
  struct Geo {
    u64 wlo;     // absolute, 16-B aligned
    u32 wbytes;  // bytes of the window that hold the tile
  };
  auto geometry = [&](u64 a, u64 e) {
    Geo g;
    const u64 first = ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)a) |
                       ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(a >> 32)) << 32)) - obase;
    const u64 whi = ((u64)(u32)__builtin_amdgcn_readlane((u32)e, 63) |
                     ((u64)(u32)__builtin_amdgcn_readlane((u32)(e >> 32), 63) << 32)) - obase;
    g.wlo = (base + first) & ~(u64)15;
    const u64 span = whi > first ? base + whi - g.wlo : 0;
    g.wbytes = span < (u64)WIN ? (u32)span : WIN;
    return g;
  };
  u32x4 pre[NP];
  auto issue = [&](const Geo &g) {
    gu32x4 *src = reinterpret_cast<gu32x4 *>((uintptr_t)g.wlo);
    const u32 last = g.wbytes ? (g.wbytes - 1) >> 4 : 0;  // last 16-B piece holding key bytes
#pragma unroll
    for (int j = 0; j < NP; ++j) pre[j] = __builtin_nontemporal_load(src + min((u32)(64 * j) + lane, last));
  };
  u64 t = (u64)blockIdx.x * kWavesPerBlock + wave;
  if (t < ntiles) {
    // a/e: tile t's offsets; a1/e1: tile t+nw's (in flight one tile ahead)
    u64 a, e, a1, e1;
    load_offs(t, a, e);
    load_offs(min(t + nwaves, lastt), a1, e1);
    Geo g = geometry(a, e);
    issue(g);
    for (;;) {
      // tile t's window: registers -> LDS (all NP pieces; the ones past the
      // tile repeat its last piece and are never read)
#pragma unroll
      for (int j = 0; j < NP; ++j) lds4[64 * j + lane] = pre[j];
      wave_lds_sync();
      const u64 tn = t + nwaves;
      const bool more = tn < ntiles;  // wave-uniform
      const u64 an = a1, en = e1;      // tile t+nw's offsets (landed a tile ago)
      Geo gn{};
      if (more) {
        gn = geometry(an, en);
        issue(gn);                                // tile t+nw's window, in flight while tile t hashes
        load_offs(min(tn + nwaves, lastt), a1, e1);  // and tile t+2nw's offsets
      }
      const u64 k0 = t << 6;
      const u64 start = a - obase, end = e - obase;
      const u64 len = end - start;  // 0 past the batch's end (clamped offsets)
      typename Algo::Out h;
      if (base + end - g.wlo <= g.wbytes)
        h = algo(LdsReader{lds, (u32)(base + start - g.wlo)}, len);
      else
        h = algo(GlobalReader{bytes + start}, len);
      BufStore<Sink>::put(sink, k0, (n - k0 < 64 ? n - k0 : 64), lane, h);
      wave_lds_sync();  // window read before the next copy overwrites it
      if (!more) break;
      t = tn;
      g = gn;
      a = an;
      e = en;
    }
  }
}

// ------------------------------------ length-sorted window kernel (var) ---
// Offset-indexed keys of mixed lengths.  One lane per key leaves a wave as
// slow as its longest key: CityHash64 runs the 17-32 B, 33-64 B and >64 B
// paths one after the other when a wave holds all three, and the 64-B round
// loop as often as the wave's longest key needs -- for cfg3's 16..256 B keys
// every wave runs all of them (3 rounds, where a key needs 1.6 on average),
// about twice the arithmetic the keys need.  Here a workgroup of W waves
// takes a tile of 64W consecutive keys, stages their bytes in ONE shared LDS
// window, sorts the tile's keys by cost class (length bin, below) with a
// stable counting sort in LDS, and wave w hashes sorted keys [64g, 64g+64)
// (g = w rotated by the tile number, so that no SIMD always gets the longest
// group): every wave then runs one length class with one round count.
// Digests go to their keys' own positions (scattered 8/16-B stores inside
// the tile's range; L2 merges the lines).  Keys that do not fit the window
// (rare: the window holds a 64W-key tile of mean length WINB/64W with
// room to spare) are read from global memory, in a bin of their own.
// Four workgroup barriers per tile: window landed, bin counts, sorted order,
// window free.
constexpr u32 kSortBins = 32;
__device__ __forceinline__ u32 sort_len_bin(u64 len) {
  // 0: <= 16 B, 1: 17-32, 2: 33-64, then one bin per 64-B round count
  if (len <= 16) return 0;
  if (len <= 32) return 1;
  if (len <= 64) return 2;
  const u64 r = (len - 1) >> 6;  // rounds (>= 1)
  return r < kSortBins - 4 ? 2 + (u32)r : kSortBins - 3;
}
template <int W, int WINB>
struct SortedLds {
  static constexpr int T = 64 * W;
  u32 win[WINB / 4 + 4];  // the tile's window (+16 B slack for span reads)
  u32 kst[T];             // key start in the window, ~0 = not in it
  u32 klen[T];
  uint16_t sidx[T];       // sorted position -> key of the tile
  u32 cnt[W][kSortBins];  // per wave and bin: keys
};
template <int W, int WINB, class Algo, class Sink, int AUX = 2>
__global__ __launch_bounds__(W * 64) void k_window_sorted(const uint8_t *__restrict__ bytes,
                                                          const u64 *__restrict__ offsets, u64 obase, u64 n,
                                                          Algo algo, Sink sink) {
  static_assert(WINB % 16 == 0, "window = whole 16-B DMA lanes");
  constexpr int T = 64 * W;
  constexpr int NP = (WINB + 1023) / 1024;  // 1 KiB DMA pieces
  __shared__ __attribute__((aligned(16))) SortedLds<W, WINB> S;
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u32 tid = threadIdx.x;
  const u32 wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const u32 lane = tid & 63;
  const u64 ntiles = (n + T - 1) / T;
  const u64 base = (u64)(uintptr_t)bytes;
  // this thread's key and the tile's first / end offsets: loaded one tile
  // ahead, so they land while the previous tile hashes
  u64 o_st = 0, o_en = 0, o_first = 0, o_last = 0;
  auto load_offs = [&](u64 t) {
    const u64 k = t * T + tid;
    o_st = offsets[k < n ? k : n];
    o_en = offsets[k + 1 < n ? k + 1 : n];
    o_first = offsets[t * T];                         // uniform
    o_last = offsets[t * T + T < n ? t * T + T : n];  // uniform
  };
  u64 t = blockIdx.x;
  if (t < ntiles) load_offs(t);
  for (; t < ntiles; t += gridDim.x) {
    const u64 k0 = t * T;
    const u64 first = o_first - obase, last = o_last - obase;
    const u64 wlo = (base + first) & ~(u64)15;                          // absolute, as in k_window
    const u64 span = last > first ? base + last - wlo : 0;
    const u32 wbytes = span < (u64)WINB ? (u32)span : (u32)WINB;
    const uint8_t *src = reinterpret_cast<const uint8_t *>((uintptr_t)wlo);
#pragma unroll
    for (int jj = 0; jj < (NP + W - 1) / W; ++jj) {
      const u32 j = (u32)jj * W + wave;  // wave-uniform
      if (j < (u32)NP && j * 1024 < wbytes) {
        if (j * 1024 + lane * 16 < wbytes)
          __builtin_amdgcn_global_load_lds(
              (const void __attribute__((address_space(1))) *)(src + j * 1024 + lane * 16),
              (void __attribute__((address_space(3))) *)(S.win + 256 * j), 16, 0, AUX);
      }
    }
    // this thread's key: bin, window position, rank among equal bins of the wave
    const u64 k = k0 + tid;
    const bool valid = k < n;
    const u64 st = o_st - obase, en = o_en - obase;
    const u64 len = valid ? en - st : 0;
    const bool fits = valid && base + en - wlo <= wbytes;
    const u32 b = !valid ? kSortBins - 1 : !fits ? kSortBins - 2 : sort_len_bin(len);
    S.kst[tid] = fits ? (u32)(base + st - wlo) : ~0u;
    S.klen[tid] = (u32)len;
    u64 same = ~0ull;
#pragma unroll
    for (int bit = 0; bit < 5; ++bit) {
      const u64 m = __ballot((b >> bit) & 1u);
      same &= ((b >> bit) & 1u) ? m : ~m;
    }
    const u32 r = (u32)__popcll(same & ((1ull << lane) - 1));
    if (lane < kSortBins) S.cnt[wave][lane] = 0;
    wave_lds_sync();
    if (r == 0) S.cnt[wave][b] = (u32)__popcll(same);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA pieces landed
    __syncthreads();                                  // every wave's pieces, and the counts
    // bin bases: lane j < 32 sums bin j over the waves (all / the earlier
    // ones), an exclusive scan over the 32 lanes gives this wave's base of bin j
    u32 tot = 0, pre = 0;
    if (lane < kSortBins) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const u32 c = S.cnt[w][lane];
        tot += c;
        pre += (u32)w < wave ? c : 0u;
      }
    }
    u32 inc = tot;
#pragma unroll
    for (int d = 1; d < (int)kSortBins; d <<= 1) {
      const u32 v = __shfl_up(inc, d);
      if (lane >= (u32)d) inc += v;
    }
    const u32 pos = (u32)__shfl(inc - tot + pre, (int)b) + r;
    S.sidx[pos] = (uint16_t)tid;
    __syncthreads();  // the sorted order
    if (t + gridDim.x < ntiles) load_offs(t + gridDim.x);  // lands while this tile hashes
    const u32 g = (wave + (u32)t) % (u32)W;
    const u32 idx = S.sidx[64 * g + lane];
    const u64 ki = k0 + idx;
    if (ki < n) {
      const u32 ws = S.kst[idx];
      typename Algo::Out h;
      if (ws != ~0u) {
        h = algo(LdsReader{S.win, ws}, (u64)S.klen[idx]);
      } else {
        const u64 a = offsets[ki] - obase;
        h = algo(GlobalReader{bytes + a}, offsets[ki + 1] - obase - a);
      }
      sink.put(ki, h);
    }
    __syncthreads();  // window and tables free for the next tile
  }
  sink.flush();
}

// ------------------------------------- window kernel, offsets prefetched ---
// Offset-indexed keys, as k_window<WIN, true>, with the next tile's offsets
// loaded while this tile's window streams in: the window DMA of tile t+1 is
// issued as soon as tile t is hashed, instead of after another round trip
// for its offsets (k_window: offsets -> DMA -> hash, two dependent memory
// latencies per tile).  One vector load per tile and lane (offsets[k0+lane];
// a key's end is its right neighbour's start) plus one uniform load of
// offsets[kend].
template <int WIN, class Algo, class Sink, int AUX = 2>
__global__ __launch_bounds__(kBlock) void k_window_var(const uint8_t *__restrict__ bytes,
                                                       const u64 *__restrict__ offsets, u64 obase, u64 n,
                                                       Algo algo, Sink sink) {
  static_assert(WIN % 16 == 0, "window = whole 16-B DMA lanes");
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
  const u64 base = (u64)(uintptr_t)bytes;
  auto load = [&](u64 t, u64 &a, u64 &hi) {
    const u64 k0 = t << 6;
    const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;
    a = offsets[(k0 + lane < n) ? k0 + lane : n];
    hi = offsets[kend];
  };
  u64 t = (u64)blockIdx.x * kWavesPerBlock + wave;
  u64 a = 0, hi = 0;
  if (t < ntiles) load(t, a, hi);
  for (; t < ntiles; t += nwaves) {
    const u64 i = (t << 6) + lane;
    const bool valid = i < n;
    const u64 nb = __shfl_down(a, 1);
    const u64 start = a - obase;
    const u64 end = (lane == 63 ? hi : nb) - obase;
    // lane 0 holds offsets[k0]; readfirstlane returns int: widen through u32
    const u64 first = ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)a) |
                       ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(a >> 32)) << 32)) - obase;
    const u64 whi = hi - obase;
    const u64 wlo = (base + first) & ~(u64)15;  // absolute, as in k_window
    const u64 span = whi > first ? base + whi - wlo : 0;
    const u32 wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
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
    // the next tile's offsets travel with this tile's window
    const u64 tn = t + nwaves;
    if (tn < ntiles) load(tn, a, hi);  // wave-uniform
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const u64 len = end - start;
      typename Algo::Out h;
      if (base + end - wlo <= wbytes)
        h = algo(LdsReader{lds, (u32)(base + start - wlo)}, len);
      else
        h = algo(GlobalReader{bytes + start}, len);
      sink.put(i, h);
    }
    __builtin_amdgcn_wave_barrier();  // window reused by the next tile
  }
  sink.flush();
}

// ----------------------------------- double-buffered window kernel (var) ---
// Offset-indexed keys with two LDS windows per wave: while tile t hashes out
// of one window, the LDS-DMA of tile t+nwaves streams into the other, and
// the offsets of tile t+2*nwaves are on their way.  The windows are two
// distinct __shared__ objects and the loop is unrolled by two, so every LDS
// read names its window.  A tile's digests are stored one step late, right
// after the next DMA is issued, so the wait at the top of a step only covers
// operations issued a whole tile of hashing earlier (on CDNA a load wait is
// a vmcnt wait and also waits for every older store).  Window bounds are
// absolute addresses, as in k_window.
template <int WIN, class Algo, class Sink, int AUX = 2>
__global__ __launch_bounds__(kBlock) void k_window_db(const uint8_t *__restrict__ bytes,
                                                      const u64 *__restrict__ offsets, u64 obase, u64 n,
                                                      Algo algo, Sink sink) {
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
  const u64 base = (u64)(uintptr_t)bytes;
  struct Geo {
    u64 wlo, start, end;  // wlo absolute; start/end relative to bytes
    u32 wbytes;
  };
  auto load_offs = [&](u64 t, u64 &a, u64 &hi) {
    const u64 k0 = t << 6;
    const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;
    a = offsets[(k0 + lane < n) ? k0 + lane : n];
    hi = offsets[kend];
  };
  auto geometry = [&](u64 a, u64 hi) {
    Geo g;
    const u64 nb = __shfl_down(a, 1);
    g.start = a - obase;
    g.end = (lane == 63 ? hi : nb) - obase;
    // readfirstlane returns int: widen through u32 (no sign extension)
    const u64 first = ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)a) |
                       ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(a >> 32)) << 32)) - obase;
    const u64 whi = hi - obase;
    g.wlo = (base + first) & ~(u64)15;
    const u64 span = whi > first ? base + whi - g.wlo : 0;
    g.wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
    return g;
  };
  auto issue = [&](const Geo &g, u32 *w) {
    const uint8_t *src = reinterpret_cast<const uint8_t *>((uintptr_t)g.wlo);
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
  typename Algo::Out h{};
  u64 hi_pend = ~0ull;  // index of the digest held in h (~0: none)
  auto hash = [&](u64 t, const Geo &g, const u32 *w) {
    const u64 i = (t << 6) + lane;
    hi_pend = ~0ull;
    if (i < n) {
      const u64 len = g.end - g.start;
      if (base + g.end - g.wlo <= g.wbytes)
        h = algo(LdsReader{w, (u32)(base + g.start - g.wlo)}, len);
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
    Geo g = geometry(a, hi), gn;
    issue(g, wa);
    // offsets loads are unconditional (clamped tile): a conditional load
    // merges with the old value through a register copy, and the copy waits
    // vmcnt(0) for the DMA issued just before it
    const u64 last = ntiles - 1;
    load_offs(min(t + nwaves, last), an, hin);
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

// ------------------------- window kernel, next window prefetched in VGPRs ---
// Offset-indexed keys, as k_window<WIN, true>, but the window of tile
// t+nwaves is loaded into registers (plain dwordx4 loads, NP x 16 B per lane)
// while tile t hashes out of the one LDS window, and written to LDS at the
// top of the next step: the window's memory latency hides under a tile of
// hashing at the LDS footprint (and occupancy) of the single-window kernel,
// which the double-LDS-window kernel (k_window_db) halved.  Loads past the
// window's last 16-B piece re-read that piece (clamped address: no load under
// a lane-divergent branch, none outside the 16-B blocks holding key bytes).
template <int WIN, class Algo, class Sink, bool LNT = true>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))
void k_window_rp(const uint8_t *__restrict__ bytes, const u64 *__restrict__ offsets, u64 obase, u64 n, Algo algo,
                 Sink sink) {
  static_assert(WIN % 16 == 0, "window = whole 16-B pieces");
  constexpr int NP = (WIN + 1023) / 1024;
  __shared__ __attribute__((aligned(16))) u32 win_all[kWavesPerBlock * (WIN / 4) + 4];
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  u32 *const lds = win_all + wave * (WIN / 4);
  u32x4 *const lds4 = reinterpret_cast<u32x4 *>(lds);
  const u64 base = (u64)(uintptr_t)bytes;
  struct Geo {
    u64 wlo, start, end;  // wlo absolute; start/end relative to bytes
    u32 wbytes;
  };
  auto load_offs = [&](u64 t, u64 &a, u64 &hi) {
    const u64 k0 = t << 6;
    const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;
    a = offsets[(k0 + lane < n) ? k0 + lane : n];
    hi = offsets[kend];
  };
  auto geometry = [&](u64 a, u64 hi) {
    Geo g;
    const u64 nb = __shfl_down(a, 1);
    g.start = a - obase;
    g.end = (lane == 63 ? hi : nb) - obase;
    const u64 first = ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)a) |
                       ((u64)(u32)__builtin_amdgcn_readfirstlane((u32)(a >> 32)) << 32)) - obase;
    const u64 whi = hi - obase;
    g.wlo = (base + first) & ~(u64)15;
    const u64 span = whi > first ? base + whi - g.wlo : 0;
    g.wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
    return g;
  };
  u32x4 pre[NP];
  auto issue = [&](const Geo &g) {
    const u32x4 *src = reinterpret_cast<const u32x4 *>((uintptr_t)g.wlo);
    const u32 last = g.wbytes ? (g.wbytes - 1) >> 4 : 0;  // last 16-B piece
#pragma unroll
    for (int j = 0; j < NP; ++j)
      if ((u32)j * 1024 < g.wbytes) {  // wave-uniform
        const u32 p = min((u32)(64 * j) + lane, last);
        pre[j] = ld<LNT>(src + p);
      }
  };
  auto stage = [&](const Geo &g) {
#pragma unroll
    for (int j = 0; j < NP; ++j)
      if ((u32)j * 1024 < g.wbytes && (u32)(64 * j) + lane < (g.wbytes + 15) >> 4) lds4[64 * j + lane] = pre[j];
  };
  u64 t = (u64)blockIdx.x * kWavesPerBlock + wave;
  if (t < ntiles) {
    const u64 lastt = ntiles - 1;
    u64 a, hi, an, hin;
    load_offs(t, a, hi);
    Geo g = geometry(a, hi), gn;
    issue(g);
    load_offs(min(t + nwaves, lastt), an, hin);
    for (;;) {
      stage(g);
      wave_lds_sync();
      const u64 tn = t + nwaves;
      const bool more = tn < ntiles;  // wave-uniform
      if (more) {
        gn = geometry(an, hin);
        issue(gn);  // in flight while tile t hashes
        load_offs(min(tn + nwaves, lastt), an, hin);
      }
      const u64 i = (t << 6) + lane;
      if (i < n) {
        const u64 len = g.end - g.start;
        typename Algo::Out h;
        if (base + g.end - g.wlo <= g.wbytes)
          h = algo(LdsReader{lds, (u32)(base + g.start - g.wlo)}, len);
        else
          h = algo(GlobalReader{bytes + g.start}, len);
        sink.put(i, h);
      }
      wave_lds_sync();  // the window is rewritten by the next stage()
      if (!more) break;
      t = tn;
      g = gn;
    }
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
