// tuning/kernels_tuning.h -- the TUNING build's alternative kernels, readers,
// sinks and algorithms (libpdht_hip_tuning.so, -DPDHT_HIP_TUNING; used by
// tools/abbench.py and the `--tuning` GPU tests only, never by the product
// library).  Each was measured against the product form and lost, or is a
// calibration (a kernel with part of its work removed, wrong digests) that
// DESIGN.md §4 quotes; the product headers (kernels.h, bucket.h) hold only
// what ships.  Included by tuning/launch_tuning.h and the tuning hooks of the
// C-ABI sources.
#pragma once
#include "../kernels.h"

namespace pdht {

// Key bytes in LDS at an arbitrary byte offset, r01-r03 form (tuning variant
// 175 now): a span of N bytes is one run of N/4+1 dword reads from one base
// address (ds_read2_b32 with immediate offsets, a single wait) funnelled by
// v_alignbyte_b32; the window carries 16 B of slack so the trailing dword
// read stays in the array.
struct LdsReaderFunnel {
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

// r02's 6-bit-slice CRC-32C tables (tuning variant 150): 11 x 64 entries =
// 2816 B; a 64-word table covers each of the 64 banks once, so random
// indices stay conflict-free, at 11 lookups per word against 8.
struct CrcLds6Tab {
  const u32 *t;  // [11][64]
  __device__ __forceinline__ u32 crc64(u64 x) const {  // (late r05: XOR3 folds, as the byte tables)
    const u32 lo = (u32)x, hi = (u32)(x >> 32);
    const u32 a = xor3(t[0 * 64 + (lo & 63)], t[1 * 64 + ((lo >> 6) & 63)], t[2 * 64 + ((lo >> 12) & 63)]);
    const u32 b = xor3(t[3 * 64 + ((lo >> 18) & 63)], t[4 * 64 + ((lo >> 24) & 63)],
                       t[5 * 64 + (__builtin_amdgcn_alignbit(hi, lo, 30) & 63)]);
    const u32 c = xor3(t[6 * 64 + ((hi >> 4) & 63)], t[7 * 64 + ((hi >> 10) & 63)], t[8 * 64 + ((hi >> 16) & 63)]);
    return xor3(xor3(a, b, c), t[9 * 64 + ((hi >> 22) & 63)], t[10 * 64 + (hi >> 28)]);
  }
};

template <>
struct CrcLdsSlices<6> {
  typedef CrcLds6Tab Tab;
  static constexpr u32 kWords = 11 * 64;
  __device__ static void fill(u32 *tab) {
    for (u32 k = threadIdx.x; k < kWords; k += blockDim.x) tab[k] = kCrc6Dev.t[k >> 6][k & 63];
  }
  __device__ __forceinline__ static Tab make(const u32 *t) { return Tab{t}; }
};

// r06 (tuning 303): 11-bit slices -- CRC-32C of a word as the XOR of 6
// lookups (bits 0-10, 11-21, 22-32, 33-43, 44-54: 2048-entry tables; 55-63:
// 512 entries; 42 KiB) instead of 8 byte lookups: 25 % fewer LDS reads, at
// ~2 VALU per address (an 11-bit field has no byte-select form).
struct Crc32c11Tables {
  u32 t[5 * 2048 + 512];
};
constexpr Crc32c11Tables make_crc32c11_tables() {
  Crc32c11Tables F{};
  const Crc32cTables S = make_crc32c_tables();
  for (u32 k = 0; k < 6; ++k)
    for (u32 v = 0; v < (k < 5 ? 2048u : 512u); ++v) {
      const u64 x = (u64)v << (11 * k);
      F.t[2048 * k + v] = S.t[7][x & 0xff] ^ S.t[6][(x >> 8) & 0xff] ^ S.t[5][(x >> 16) & 0xff] ^
                          S.t[4][(x >> 24) & 0xff] ^ S.t[3][(x >> 32) & 0xff] ^ S.t[2][(x >> 40) & 0xff] ^
                          S.t[1][(x >> 48) & 0xff] ^ S.t[0][x >> 56];
    }
  return F;
}
__device__ __constant__ const Crc32c11Tables kCrc11Dev = make_crc32c11_tables();
struct CrcLds11Tab {
  const u32 *t;
  __device__ __forceinline__ u32 crc64(u64 x) const {
    const u32 lo = (u32)x, hi = (u32)(x >> 32);
    const u32 a = xor3(t[lo & 2047], t[2048 + ((lo >> 11) & 2047)],
                       t[4096 + (__builtin_amdgcn_alignbit(hi, lo, 22) & 2047)]);
    const u32 b = xor3(t[6144 + ((hi >> 1) & 2047)], t[8192 + ((hi >> 12) & 2047)], t[10240 + (hi >> 23)]);
    return a ^ b;
  }
};
template <>
struct CrcLdsSlices<11> {
  typedef CrcLds11Tab Tab;
  static constexpr u32 kWords = 5 * 2048 + 512;
  __device__ static void fill(u32 *tab) {
    for (u32 k = threadIdx.x; k < kWords; k += blockDim.x) tab[k] = kCrc11Dev.t[k];
  }
  __device__ __forceinline__ static Tab make(const u32 *t) { return Tab{t}; }
};

// Timing only: the CRC-32C of a word replaced by a fold (no table lookups):
// what the lookups cost the long-key kernel (wrong digests).
struct CrcNullTab {
  const u32 *t;
  __device__ __forceinline__ u32 crc64(u64 x) const { return (u32)x ^ (u32)(x >> 32) ^ t[0]; }
};

template <>
struct CrcLdsSlices<0> {  // CrcNullTab: the 6-bit form's launch shape, no lookups
  typedef CrcNullTab Tab;
  static constexpr u32 kWords = 64;
  __device__ static void fill(u32 *tab) {
    for (u32 k = threadIdx.x; k < kWords; k += blockDim.x) tab[k] = 0;
  }
  __device__ __forceinline__ static Tab make(const u32 *t) { return Tab{t}; }
};

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

// 64-bit digests stored 16 B per lane: every even lane takes its odd
// neighbour's digest (two DPP row_shl:1 moves) and stores both with one
// dwordx4, so a wave's 512 B of digests leave as 32 lane-stores instead of
// 64 (i must be 64-aligned tile base + lane, as in every kernel here; a lane
// whose partner is inactive -- past the batch's end, or in another branch of
// a divergent hash -- stores its own digest alone).
template <bool NTS = true>
struct Sink64x2T {
  static constexpr u32 kHist = 1;
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64 i, u64 h) {
    const u32 lo = (u32)h, hi = (u32)(h >> 32);
    const u32 lo1 = __builtin_amdgcn_mov_dpp(lo, 0x101, 0xf, 0xf, false);  // row_shl:1: lane l <- l+1
    const u32 hi1 = __builtin_amdgcn_mov_dpp(hi, 0x101, 0xf, 0xf, false);
    const u32 lane = (u32)i & 63;
    // partner = the other lane of the pair; the two may sit in different
    // divergent branches (then each stores its own digest)
    const bool partner = (__builtin_amdgcn_read_exec() >> (lane ^ 1)) & 1;
    if ((lane & 1) == 0 && partner)
      st<NTS>(u32x4{lo, hi, lo1, hi1}, reinterpret_cast<u32x4 *>(out + i));
    else if (!partner)
      st<NTS>(h, out + i);
  }
  __device__ __forceinline__ void flush() {}
  __host__ Sink64x2T shift(u64 k0) const { return Sink64x2T{lds_hist, out + k0}; }
};

// Calibration only: digests dropped (a kernel's loads alone).
struct SinkNone {
  static constexpr u32 kHist = 1;
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64, u64 h) {
    if (h == 0x0123456789abcdefull) out[0] = h;  // keeps the digest live, never taken
  }
  __device__ __forceinline__ void flush() {}
};
// Calibration only: every digest stored, but into the first 32 KiB of out
// (L2-resident): the store instructions without their HBM writes.
struct SinkSmall {
  static constexpr u32 kHist = 1;
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64 i, u64 h) { out[i & 4095] = h; }
  __device__ __forceinline__ void flush() {}
};
// Calibration only: nt digest stores wrapped into the first 2^BITS digests
// of out (2^BITS x 8 B: L2-sized to Infinity-Cache-sized destinations).
template <int BITS>
struct SinkRing {
  static constexpr u32 kHist = 1;
  u32 *lds_hist;
  u64 *out;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ void put(u64 i, u64 h) { st<true>(h, out + (i & ((1ull << BITS) - 1))); }
  __device__ __forceinline__ void flush() {}
  __host__ SinkRing shift(u64) const { return *this; }
};

// ------------------------------------------------ pipelined window kernel ---
// Offset-indexed keys with 64-bit digests, one LDS window per wave as in
// k_window, but with every memory latency except the window DMA's taken off a
// tile's critical path.  k_window's tile is a chain of four dependent memory
// round trips -- offsets (a vmcnt(0) wait that also waits for the previous
// tile's digest store to be acknowledged), two scalar loads of the window
// bounds, then the DMA.  Here:
//   * the offsets of the wave's next tile are loaded while this tile's window
//     streams in: one dwordx4 per lane = offsets[i], offsets[i+1] (index
//     clamped to n-1, so the load is always issued and the clamped lanes read
//     offsets[n]); the window is [lane 0's start, lane 63's end) by readlane --
//     no scalar loads, whose lgkmcnt wait would meet the LDS reads;
//   * a tile's digests are stored one tile late, right after the next tile's
//     DMA and offsets load are issued, as a raw buffer store whose range
//     check drops the lanes past n (always issued, even with no valid lane);
//   * so the wait for a window is s_waitcnt vmcnt(2): on gfx950 loads, stores
//     and LDS-DMA count together in issue order (MI355X_MICROARCH.md,
//     "s_waitcnt vmcnt(N)"), and the two youngest operations are exactly that
//     offsets load and that store -- the wait never includes a store.
// G = tiles a wave takes in a row before jumping by the grid (1: the grid
// stride of k_window; 16: r02's grouped order, consecutive windows per wave).
// RING (calibration only): digests of tile t go to out + 64 * (t % RING), an
// L2-resident destination -- the kernel without its HBM writes.
// SAUX: cache-policy bits of the digest stores (gfx950: 1 = sc0, 2 = nt, 16 = sc1).
template <int WIN, int G, class Algo, int AUX = 2, class LR = LdsReader, u64 RING = 0, int SAUX = AUX>
__global__ __launch_bounds__(kBlock) void k_window_pipe(const uint8_t *__restrict__ bytes,
                                                        const u64 *__restrict__ offsets, u64 obase, u64 n,
                                                        Algo algo, u64 *__restrict__ out) {
  static_assert(WIN % 16 == 0, "window = whole 16-B DMA lanes");
  __shared__ __attribute__((aligned(16))) u32 win_all[kWavesPerBlock * (WIN / 4) + 4];
  algo_init(algo);
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) >> 6;
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  u32 *lds = win_all + wave * (WIN / 4);
  const u64 base = (u64)(uintptr_t)bytes;
  // tile order: runs of G consecutive tiles, run r of wave w = gw + r * nwaves
  const u64 gw = (u64)blockIdx.x * kWavesPerBlock + wave;
  auto next = [&](u64 t) -> u64 {
    if (G > 1 && (t + 1) % G != 0) return t + 1;
    return (t / G + nwaves) * G;
  };
  u64 t = gw * G;
  if (t >= ntiles) return;
  // key i's bounds: offsets[min(i, n-1)] and the next entry (n >= 1 here)
  auto bounds = [&](u64 tt, u64 &a, u64 &e) {
    const u64 *p = offsets + ((tt << 6) + lane < n ? (tt << 6) + lane : n - 1);
    a = p[0];
    e = p[1];
  };
  auto rd64 = [](u64 v, u32 l) -> u64 {
    return (u64)(u32)__builtin_amdgcn_readlane((u32)v, l) |
           ((u64)(u32)__builtin_amdgcn_readlane((u32)(v >> 32), l) << 32);
  };
  u64 a, e;
  bounds(t, a, e);
  u64 hprev = 0, tprev = ~0ull;  // digest of the previous tile (none yet)
  typedef u32 u32x2 __attribute__((ext_vector_type(2)));
  while (true) {
    const u64 k0 = t << 6;
    const u64 i = k0 + lane;
    const bool valid = i < n;
    const u64 start = a - obase;
    const u64 end = e - obase;
    const u64 first = rd64(a, 0) - obase;
    const u64 whi = rd64(e, 63) - obase;
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
    __builtin_amdgcn_sched_barrier(0);
    // the next tile's offsets (always issued: clamped index; past the end the
    // loop stops before they are used)
    const u64 tn = next(t);
    u64 an, en;
    bounds(tn, an, en);
    __builtin_amdgcn_sched_barrier(0);
    // the previous tile's digests (always issued; records past n dropped)
    {
      const u64 pk = tprev << 6;
      const u32 nrec = tprev == ~0ull ? 0u : (u32)((n - pk < 64 ? n - pk : 64) * 8);
      const u64 dst = tprev == ~0ull ? 0 : RING ? (tprev % RING) << 6 : pk;
      __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + dst, 0, nrec, 0x00020000);
      const u32x2 w = {(u32)hprev, (u32)(hprev >> 32)};
      __builtin_amdgcn_raw_buffer_store_b64(w, r, lane * 8, 0, SAUX);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (valid) {
      const u64 len = end - start;
      if (base + end - wlo <= wbytes)
        hprev = algo(LR{lds, (u32)(base + start - wlo)}, len);
      else
        hprev = algo(GlobalReader{bytes + start}, len);
    }
    tprev = t;
    __builtin_amdgcn_wave_barrier();  // window reused by the next tile
    if (tn >= ntiles) break;
    t = tn;
    a = an;
    e = en;
  }
  // the last tile's digests
  const u64 pk = tprev << 6;
  const u32 nrec = (u32)((n - pk < 64 ? n - pk : 64) * 8);
  __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(out + (RING ? (tprev % RING) << 6 : pk), 0, nrec, 0x00020000);
  const u32x2 w = {(u32)hprev, (u32)(hprev >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(w, r, lane * 8, 0, SAUX);
}

// ------------------------------------------------ 64-B tile-order probe ---
// k_fixed_xpose64 (kernels.h) with the wave -> tile order as a parameter
// (r05 experiment on the allocation-dependent speed of the 64-B stream,
// DESIGN.md §4.1): ORDER 1 = tile t at position (t * 0x9E3779B1) mod ntiles
// (ntiles a power of two: a bijection that scatters the tiles in flight over
// the whole batch instead of one contiguous window); ORDER 2 = each wave a
// contiguous run of ceil(ntiles / nwaves) tiles.
// Digests go where their keys' tile is.
template <class Algo, class Sink, int ORDER>
__global__ __launch_bounds__(kBlock) void k_fixed_xpose64_order(const uint8_t *__restrict__ keys, u64 n, Algo algo,
                                                                Sink sink) {
  constexpr int DEPTH = 2;
  __shared__ __attribute__((aligned(16))) u32x4 img[kWavesPerBlock][256];
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 ntiles = n >> 6;  // the launcher passes whole tiles only
  const u64 nwaves = (u64)gridDim.x * kWavesPerBlock;
  const u64 gw = (u64)blockIdx.x * kWavesPerBlock + wave;
  const u64 per = (ntiles + nwaves - 1) / nwaves;  // ORDER 2: tiles per wave (the last waves fewer)
  // k-th tile of this wave (k = 0, 1, ...) -> physical tile
  auto tile = [&](u64 k) -> u64 {
    if constexpr (ORDER == 2) return gw * per + k;
    const u64 t = gw + k * nwaves;
    return ORDER == 1 ? (t * 0x9E3779B1ull) & (ntiles - 1) : t;
  };
  const u64 nk = ORDER == 2 ? (gw * per < ntiles ? min(per, ntiles - gw * per) : 0)
                            : (ntiles > gw ? (ntiles - gw + nwaves - 1) / nwaves : 0);
  u32x4 pre[DEPTH][4];
  auto fetch = [&](int d, u64 t) {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(keys + (t << 12));
#pragma unroll
    for (int j = 0; j < 4; ++j) pre[d][j] = ld<true>(src + 64 * j + lane);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if ((u64)d < nk) fetch(d, tile(d));
  for (u64 k = 0; k < nk; k += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      if (k + d >= nk) break;  // wave-uniform
      const u64 tt = tile(k + d);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u32 g = 64 * j + lane;
        img[wave][xpose_slot(g >> 2, g & 3)] = pre[d][j];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (k + d + DEPTH < nk) fetch(d, tile(k + d + DEPTH));
      RegReader<16> r;
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
      sink.put((tt << 6) + lane, algo(r, (u64)64));
    }
  }
  sink.flush();
}

// ------------------------------------- workgroup write-combined window ---
// k_window for offset-indexed keys with 64-bit
// digests, where the 4 waves of a workgroup take 4 CONSECUTIVE tiles (a
// 256-key super-tile), stage their digests in LDS and the workgroup stores
// the super-tile's 2 KiB of digests as one contiguous run (256 threads x 8 B,
// non-temporal), instead of each wave storing its own 512 B when its tile is
// done.  Two barriers per super-tile couple the 4 waves.
template <int WIN, class Algo>
__global__ __launch_bounds__(kBlock) void k_window_wc(const uint8_t *__restrict__ bytes,
                                                      const u64 *__restrict__ offsets, u64 obase, u64 n, Algo algo,
                                                      u64 *__restrict__ out) {
  static_assert(WIN % 16 == 0, "window = whole 16-B DMA lanes");
  __shared__ __attribute__((aligned(16))) u32 win_all[kWavesPerBlock * (WIN / 4) + 4];
  __shared__ u64 dig[kBlock];
  algo_init(algo);
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lane = threadIdx.x & 63;
  const u64 nsuper = (n + kBlock - 1) / kBlock;
  u32 *lds = win_all + wave * (WIN / 4);
  const u64 base = (u64)(uintptr_t)bytes;
  for (u64 sp = blockIdx.x; sp < nsuper; sp += gridDim.x) {
    __builtin_amdgcn_s_setprio(1);
    const u64 k0 = sp * kBlock + wave * 64;  // this wave's tile
    const u64 i = k0 + lane;
    const bool valid = i < n;
    u64 start = 0, end = 0;
    if (valid) {
      start = offsets[i] - obase;
      end = offsets[i + 1] - obase;
    }
    u32 wbytes = 0;
    u64 wlo = 0;
    if (k0 < n) {
      const u64 kend = (k0 + 64 < n) ? k0 + 64 : n;
      const u64 whi = offsets[kend] - obase;
      const u64 first = offsets[k0] - obase;
      wlo = (base + first) & ~(u64)15;
      const u64 span = whi > first ? base + whi - wlo : 0;
      wbytes = span < (u64)WIN ? (u32)span : (u32)WIN;
      const uint8_t *src = reinterpret_cast<const uint8_t *>((uintptr_t)wlo);
#pragma unroll
      for (int j = 0; j < (WIN + 1023) / 1024; ++j) {
        if ((u32)j * 1024 < wbytes) {
          if ((u32)j * 1024 + lane * 16 < wbytes)
            __builtin_amdgcn_global_load_lds(
                (const void __attribute__((address_space(1))) *)(src + j * 1024 + lane * 16),
                (void __attribute__((address_space(3))) *)(lds + 256 * j), 16, 0, 2);
        }
      }
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    u64 h = 0;
    if (valid) {
      const u64 len = end - start;
      if (base + end - wlo <= wbytes)
        h = algo(LdsReader{lds, (u32)(base + start - wlo)}, len);
      else
        h = algo(GlobalReader{bytes + start}, len);
    }
    dig[threadIdx.x] = h;
    __syncthreads();
    const u64 j = sp * kBlock + threadIdx.x;
    if (j < n) __builtin_nontemporal_store(dig[threadIdx.x], out + j);  // the super-tile's 2 KiB in one run
    __syncthreads();  // windows and dig reused by the next super-tile
  }
}


// ------------------------------------------- long keys through an LDS ring ---
// r05 experiment (tuning 279-282): fixed keys of L = 1024 / 2048 / 4096 B on
// the CityHashCrc256 path.  The product walks each lane's key with per-lane
// loads (every wave instruction touches 64 lines).  Here the wave's 64 keys
// stream through a ring of R line-rounds in LDS (a round = one 128-B line of
// each of the 64 keys, 8 KiB), filled by COALESCED LDS-DMA: in DMA
// instruction i, lanes 8j..8j+7 fetch the 8 pieces of key 8i+j's line, in an
// order rotated by i + j so that the per-lane reads that follow are free of
// bank conflicts (piece p of key k = 8i+j sits at slot ((p - i - j) & 7)).
// The hash runs Crc256Stream (line-by-line), reading each line from the ring
// into registers; the moment a line is read its slot takes the line R ahead
// (the next tile's first lines at the end of a tile), so R - 1 rounds are
// always in flight and no VGPR holds them.  Waits are exact: when line l is
// read, the lines issued after it are l+1 .. l+R-1 (8 DMA instructions
// each; a digest store in between only makes the wait stricter); the last
// tile waits for everything.
__device__ __forceinline__ void lds_dma16(const void *g, u32 lds) {
  lds = __builtin_amdgcn_readfirstlane(lds);
  u32 save;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(save)
      : "v"(g), "s"(lds)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait_c() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int L, int R>
struct LongRing {
  static constexpr int NL = L / 128;                                  // lines per key
  static constexpr int kBlocks = L / 240;
  static constexpr int kStreamLines = (240 * kBlocks + 127) / 128;  // lines the block loop streams
  static constexpr int kLate = kStreamLines - 1;                     // first line kept for the tail
  static_assert(L % 128 == 0 && L > 900, "whole lines, CityHashCrc256 path");
  static_assert(R >= NL - kStreamLines + 1 && R <= NL && R * 8 <= 63, "ring depth");
  static constexpr int kTailWait = 8 * (R + kStreamLines - NL - 1);
};

// A wave's view of its ring (every member wave-uniform except the lane's own
// offsets).  line_lim() reads line l of the lane's key and hands the slot to
// the line R ahead; span() serves the tail chunks from the late lines.
template <int L, int R>
struct RingReader {
  typedef LongRing<L, R> G;
  static constexpr bool kStream = true;
  uint8_t *ring;        // this wave's R slots of 8 KiB (LDS)
  u32 ring_lds;         // the same, as an LDS byte address (DMA base)
  u32 kofs, rot;        // lane's key row inside a slot; its piece rotation
  u32 seq0;             // ring sequence number of this tile's line 0
  const uint8_t *cur;   // keys of this tile's DMA rows (lane-specific, clamped), line 0
  const uint8_t *nxt;   // the next tile's (nullptr: this is the wave's last tile)
  u32 dma_rot;          // lane's DMA piece rotation base: (lane & 7) + (lane >> 3)
  u64 dma_step;         // bytes from DMA instruction i's row to i+1's (8 keys)
  u64 last_row_off;     // clamp: offset of the batch's last row from `cur` / `nxt` (per tile)
  u64 nxt_last_row_off;

  __device__ __forceinline__ u32 slot(u32 l) const { return ((seq0 + l) % R) * 8192u; }
  __device__ __forceinline__ void wait_line(u32 l) const {
    if (nxt == nullptr)
      vm_wait_c<0>();
    else
      vm_wait_c<8 * (R - 1)>();
  }
  // DMA line l of the tile whose rows start at base (lane-specific) into slot s
  __device__ __forceinline__ void issue(const uint8_t *base, u64 last_off, u32 l, u32 s) const {
#pragma unroll
    for (u32 i = 0; i < 8; ++i) {
      const u64 off = min((u64)i * dma_step, last_off);
      const u32 p = (dma_rot + i) & 7;
      lds_dma16(base + off + 128u * l + 16u * p, ring_lds + s + i * 1024u);
    }
  }
  // the slot of line l is free: fetch the line R ahead into it
  __device__ __forceinline__ void release(u32 l) const {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's reads have landed
    const u32 ahead = l + R;
    if (ahead < (u32)G::NL)
      issue(cur, last_row_off, ahead, slot(l));
    else if (nxt)
      issue(nxt, nxt_last_row_off, ahead - G::NL, slot(l));
  }
  __device__ __forceinline__ const uint8_t *at(u32 o) const {  // byte o of the lane's key (resident line)
    const u32 l = o >> 7, p = (o >> 4) & 7;
    return ring + slot(l) + kofs + ((p - rot) & 7) * 16 + (o & 15);
  }
  template <int N>
  __device__ __forceinline__ Words<N / 4> line_lim(u32 o, u32) const {
    static_assert(N == 128, "whole lines");
    const u32 l = o >> 7;
    wait_line(l);
    Words<32> w;
    typedef u32 u32x4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (u32 p = 0; p < 8; ++p) {
      const u32x4v v = *reinterpret_cast<const u32x4v *>(ring + slot(l) + kofs + ((p - rot) & 7) * 16);
      w.d[4 * p] = v.x;
      w.d[4 * p + 1] = v.y;
      w.d[4 * p + 2] = v.z;
      w.d[4 * p + 3] = v.w;
    }
    if (l < (u32)G::kLate) release(l);
    return w;
  }
  template <int N>
  __device__ __forceinline__ Words<N / 4> span(u32 o) const {
    Words<N / 4> w;
    if ((o + N - 1) >> 7 > (u32)G::kLate) {  // a line only the tail reads: its DMA
      if (nxt == nullptr)
        vm_wait_c<0>();
      else
        vm_wait_c<G::kTailWait>();
    }
    if ((o & 7) == 0 && N % 8 == 0) {
#pragma unroll
      for (int j = 0; j < N / 8; ++j) {
        const u64 v = *reinterpret_cast<const u64 *>(at(o + 8 * j));
        w.d[2 * j] = (u32)v;
        w.d[2 * j + 1] = (u32)(v >> 32);
      }
    } else {
#pragma unroll
      for (int j = 0; j < N / 4; ++j) w.d[j] = w32(o + 4 * j);
    }
    return w;
  }
  __device__ __forceinline__ u32 b8(u32 o) const { return *at(o); }
  __device__ __forceinline__ u32 w32(u32 o) const {
    return b8(o) | (b8(o + 1) << 8) | (b8(o + 2) << 16) | (b8(o + 3) << 24);
  }
};

template <int L, int R, class Algo, class Sink>
__global__ __launch_bounds__(256) void k_long_ring(const uint8_t *__restrict__ keys, u64 n, Algo algo, Sink sink) {
  typedef LongRing<L, R> G;
  extern __shared__ __attribute__((aligned(16))) uint8_t ring_all[];  // [4 waves][R][8 KiB]
  __shared__ u32 lds_hist[Sink::kHist];
  sink.lds_hist = lds_hist;
  algo_init(algo);
  sink.init();
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const u64 ntiles = (n + 63) / 64, nwaves = (u64)gridDim.x * 4;
  u64 t = (u64)blockIdx.x * 4 + wave;
  if (t < ntiles) {
    RingReader<L, R> rd;
    rd.ring = ring_all + wave * (R * 8192);
    rd.ring_lds = (u32)(uintptr_t)rd.ring;
    rd.kofs = (lane >> 3) * 1024 + (lane & 7) * 128;
    rd.rot = (lane >> 3) + (lane & 7);
    rd.dma_rot = (lane & 7) + (lane >> 3);
    rd.dma_step = 8ull * L;
    // DMA rows of tile tt for this lane: key 64 tt + 8 i + (lane >> 3) in instruction i
    auto rows = [&](u64 tt, u64 &last_off) {
      const u64 first = tt * 64 + (lane >> 3);
      last_off = (n - 1 >= first ? n - 1 - first : 0) * (u64)L;  // rows past the batch re-read its last key
      return keys + min(first, n - 1) * (u64)L;
    };
    rd.seq0 = 0;
    rd.cur = rows(t, rd.last_row_off);
    u64 tn = t + nwaves;
    rd.nxt = tn < ntiles ? rows(tn, rd.nxt_last_row_off) : nullptr;
    // the first tile's first R lines
#pragma unroll
    for (u32 l = 0; l < (u32)R; ++l) rd.issue(rd.cur, rd.last_row_off, l, l * 8192u);
    while (true) {
      const u64 i = t * 64 + lane;
      const auto h = algo(rd, (u64)L);
      // the tail has read the late lines: their slots take the lines R ahead
      if (rd.nxt == nullptr)
        vm_wait_c<0>();
#pragma unroll
      for (u32 l = G::kLate; l < (u32)G::NL; ++l) rd.release(l);
      if (i < n) sink.put(i, h);
      if (rd.nxt == nullptr) break;
      t = tn;
      tn = t + nwaves;
      rd.seq0 += G::NL;
      rd.cur = rd.nxt;
      rd.last_row_off = rd.nxt_last_row_off;
      rd.nxt = tn < ntiles ? rows(tn, rd.nxt_last_row_off) : nullptr;
    }
  }
  sink.flush();
}

}  // namespace pdht
