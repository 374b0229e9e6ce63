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

#include "city_core.h"

namespace pdht {

constexpr int kBlock = 256;  // 4 waves
constexpr int kWavesPerBlock = kBlock / 64;

// --------------------------------------------------------------- readers ---
// Key bytes in LDS at an arbitrary byte offset.  Each dword fetch reads the
// two covering dwords and funnels them with v_alignbyte_b32; the window
// carries 16 B of slack so the trailing dword read stays in the array.
struct LdsReader {
  const u32 *lds;
  u32 base;
  __device__ __forceinline__ u32 dw(u32 o) const {
    o += base;
    const u32 q = o >> 2;
    return __builtin_amdgcn_alignbyte(lds[q + 1], lds[q], o & 3u);
  }
  __device__ __forceinline__ u64 w64(u32 o) const { return ((u64)dw(o + 4) << 32) | dw(o); }
  __device__ __forceinline__ u32 w32(u32 o) const { return dw(o); }
  __device__ __forceinline__ u32 b8(u32 o) const {
    o += base;
    return (lds[o >> 2] >> (8 * (o & 3u))) & 0xffu;
  }
  __device__ __forceinline__ LdsReader at(u32 o) const { return LdsReader{lds, base + o}; }
};

// Key bytes straight from global memory (keys larger than the LDS window).
struct GlobalReader {
  const uint8_t *p;
  __device__ __forceinline__ u64 w64(u32 o) const {
    u64 v;
    __builtin_memcpy(&v, p + o, 8);
    return v;
  }
  __device__ __forceinline__ u32 w32(u32 o) const {
    u32 v;
    __builtin_memcpy(&v, p + o, 4);
    return v;
  }
  __device__ __forceinline__ u32 b8(u32 o) const { return p[o]; }
  __device__ __forceinline__ GlobalReader at(u32 o) const { return GlobalReader{p + o}; }
};

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

// ----------------------------------------------------------------- sinks ---
// Where a digest goes.  init()/flush() run once per workgroup around the
// grid-stride loop (every thread reaches both).
struct Sink64 {
  static constexpr u32 kHist = 1;  // LDS histogram words this sink needs
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64 i, u64 h) { __builtin_nontemporal_store(h, out + i); }
  __device__ __forceinline__ void flush() {}
};
struct Sink128 {
  static constexpr u32 kHist = 1;
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64 i, u128 h) {
    typedef u64 u64x2 __attribute__((ext_vector_type(2)));
    u64x2 v = {h.lo, h.hi};
    __builtin_nontemporal_store(v, reinterpret_cast<u64x2 *>(out) + i);
  }
  __device__ __forceinline__ void flush() {}
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
struct SinkPlace {
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
    __builtin_nontemporal_store(h, mbits + i);
    if (ptindex) __builtin_nontemporal_store((u32)pt.mod(h), ptindex + i);
    if (rank || hist) {
      const u32 r = (u32)rk.mod(h);
      if (rank) *reinterpret_cast<u32 *>(rank + i * rank_stride) = r;
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
      for (u32 r = threadIdx.x; r < nranks; r += blockDim.x)
        if (lds_hist[r]) atomicAdd(reinterpret_cast<unsigned long long *>(hist + r), (unsigned long long)lds_hist[r]);
    }
  }
};

// ------------------------------------------------------------ key loads ---
template <int L>
__device__ __forceinline__ void load_key_regs(const uint8_t *__restrict__ keys, u64 i,
                                              RegReader<L / 4> &r) {
  static_assert(L == 8 || L % 16 == 0, "direct path: L = 8 or a multiple of 16");
  if constexpr (L == 8) {
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(keys) + i);
    r.d[0] = v.x;
    r.d[1] = v.y;
  } else {
    typedef u32 u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 *p = reinterpret_cast<const u32x4 *>(keys + i * (u64)L);
#pragma unroll
    for (int j = 0; j < L / 16; ++j) {
      const u32x4 v = __builtin_nontemporal_load(p + j);
      r.d[4 * j + 0] = v.x;
      r.d[4 * j + 1] = v.y;
      r.d[4 * j + 2] = v.z;
      r.d[4 * j + 3] = v.w;
    }
  }
  r.base = 0;
}

// ------------------------------------------------------- direct kernel ---
// U keys per lane per iteration (all loads issued before any hashing).
template <int L, int U, class Algo, class Sink>
__global__ __launch_bounds__(kBlock) void k_fixed_direct(const uint8_t *__restrict__ keys, u64 n,
                                                         Algo algo, Sink sink) {
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  sink.init();
  const u64 stride = (u64)gridDim.x * kBlock;
  for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride * U) {
    RegReader<L / 4> r[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) load_key_regs<L>(keys, i + u * stride, r[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * stride < n) sink.put(i + u * stride, algo(r[u], (u64)L));
  }
  sink.flush();
}

// -------------------------------------------------- LDS-transposed 64 B ---
// A wave's 64 keys (4 KiB) arrive by 4 LDS-DMA instructions: instruction j
// moves bytes [1024j, 1024j+1024) of the tile, lane l's 16 B landing at
// LDS byte 1024j + 16l (linear).  Key k's chunk c (16 B) therefore sits at
// slot 4k + c.  Lane k reads its 4 chunks with ds_read_b128; to keep the
// 16-lane groups of ds_read_b128 conflict-free the SOURCE is permuted so the
// image holds chunk c of key k at slot 4k + (c ^ ((k >> 2) & 3)) (the read
// applies the same involution).
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
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  typedef u32 u32x4 __attribute__((ext_vector_type(4)));

  // DMA of tile t into buffer b (only full tiles; the ragged last tile is
  // loaded through registers below).
  auto issue = [&](u64 t, int b) {
    const uint8_t *base = keys + (t << 12);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32 slot = 64 * j + lane;              // image slot written by this lane
      const u32 k = slot >> 2, c = slot & 3;        // image holds chunk c ^ swz(k) of key k
      const u32 src_chunk = c ^ ((k >> 2) & 3);
      const uint8_t *src = base + k * 64 + src_chunk * 16;
      __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)src,
                                       (void __attribute__((address_space(3))) *)&tile[wave][b][256 * j],
                                       16, 0, 0);
    }
  };

  u64 t = (u64)blockIdx.x * kWavesPerBlock + wave;
  const u64 full = n >> 6;  // tiles with 64 valid keys
  int b = 0;
  if (t < full) issue(t, 0);
  for (; t < ntiles; t += nwaves) {
    const u64 tn = t + nwaves;
    if (tn < full) issue(tn, b ^ 1);  // prefetch next tile into the other buffer
    const u64 i = (t << 6) + lane;
    RegReader<16> r;
    r.base = 0;
    if (t < full) {
      // wait for this tile's 4 DMAs (the next tile's 4 may stay in flight)
      if (tn < full)
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const u32x4 *row = reinterpret_cast<const u32x4 *>(&tile[wave][b][0]) + 4 * lane;
      const u32 sw = (lane >> 2) & 3;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const u32x4 v = row[c ^ sw];
        r.d[4 * c + 0] = v.x;
        r.d[4 * c + 1] = v.y;
        r.d[4 * c + 2] = v.z;
        r.d[4 * c + 3] = v.w;
      }
    } else if (i < n) {
      load_key_regs<64>(keys, i, r);
    }
    if (i < n) sink.put(i, algo(r, (u64)64));
    b ^= 1;
    __builtin_amdgcn_wave_barrier();  // all lanes done reading buffer b before it is refilled
  }
  sink.flush();
}

// --------------------------------------------------------- window kernel ---
// Any key length.  VAR: key i = bytes[offsets[i]-obase, offsets[i+1]-obase);
// otherwise key i = bytes[i*stride, i*stride+keylen).  WIN = LDS bytes per
// wave.
template <int WIN, bool VAR, class Algo, class Sink>
__global__ __launch_bounds__(kBlock) void k_window(const uint8_t *__restrict__ bytes,
                                                   const u64 *__restrict__ offsets, u64 obase,
                                                   u64 stride, u64 keylen, u64 n, Algo algo,
                                                   Sink sink) {
  static_assert(WIN % 1024 == 0, "window = whole 1 KiB DMA pieces");
  __shared__ __attribute__((aligned(16))) u32 win[kWavesPerBlock][WIN / 4 + 4];
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  u32 *lds = win[wave];
  for (u64 t = (u64)blockIdx.x * kWavesPerBlock + wave; t < ntiles; t += nwaves) {
    const u64 k0 = t << 6;
    const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;  // one past the tile's last key
    const u64 i = k0 + lane;
    const bool valid = i < n;
    u64 start = 0, end = 0, wlo, whi;
    if constexpr (VAR) {
      if (valid) {
        start = offsets[i] - obase;
        end = offsets[i + 1] - obase;
      }
      wlo = offsets[k0] - obase;
      whi = offsets[kend] - obase;
    } else {
      start = i * stride;
      end = start + keylen;
      wlo = k0 * stride;
      whi = (kend - 1) * stride + keylen;
    }
    wlo &= ~(u64)15;
    const u64 span = whi - wlo;
    const u32 wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
    // DMA the window: piece j moves 1 KiB, lane l's 16 B to LDS 1024j+16l.
    // 16-B-aligned pieces never cross a page the key bytes do not touch.
    const uint8_t *src = bytes + wlo;
#pragma unroll
    for (int j = 0; j < WIN / 1024; ++j) {
      if ((u32)j * 1024 < wbytes) {  // wave-uniform
        if ((u32)j * 1024 + lane * 16 < wbytes)
          __builtin_amdgcn_global_load_lds(
              (const void __attribute__((address_space(1))) *)(src + j * 1024 + lane * 16),
              (void __attribute__((address_space(3))) *)(lds + 256 * j), 16, 0, 0);
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

// ------------------------------------------------- synthetic workloads ---
__global__ __launch_bounds__(kBlock) void k_splitmix64(u64 seed, u64 first, u64 nwords, u64 *out);
__global__ __launch_bounds__(kBlock) void k_mixed_lengths(u64 seed, u64 first, u64 n, u32 lo,
                                                          u32 span, u64 *lens);

}  // namespace pdht
