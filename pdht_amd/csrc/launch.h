// launch.h -- kernel choice and launch of the hash paths:
// fixed-length keys (launch_fixed), variable-length keys (launch_var).
// Included by the translation units that instantiate them.
#pragma once
#include "runtime.h"

namespace pdht {

constexpr int kWinBytes = 12288;  // k_window over fixed keys: LDS window per wave (12 KiB)
}  // namespace pdht
// one A/B hook per launch path below (product/pdht_hooks_launch.h: none taken)
#include "pdht_hooks_launch.h"
namespace pdht {
// Kernel tags (pdht_hip_last_kernel): the kernel and its launch shape, so a
// profile taken of one shape (profiles/traffic_*.json) is never attributed to
// another.

// Packed 8/16/32-byte keys: each lane loads its own key (lane-adjacent rows,
// so 8- and 16-byte keys are fully coalesced), U keys in flight per lane.
// r01 interleaved A/B (profiles/r01/placebench_*): 8-B keys with non-temporal
// stores (+26 % on fused placement), 16-B keys with non-temporal loads and
// stores (+6-11 %).  Late r04 re-measured the shapes with the keys rotated
// over buffers larger than the 256 MiB Infinity Cache (bench.py rot_copies;
// r01 had re-read one cache-resident key buffer): every width now loads
// non-temporally -- 8-B placement 0.605 -> 0.640, 8-B hashing 0.659 -> 0.712,
// 32-B 0.628 -> 0.688 (with nt stores) -- and 8-B placement keeps 8 keys per
// lane in flight (0.621 -> 0.681) (profiles/r04/ab/*rot*.log).
#ifndef PDHT_PLACE8_NT
#define PDHT_PLACE8_NT true
#endif
template <class Algo, class Sink>
static void launch_small(size_t keylen, const uint8_t *k, size_t n, Algo algo, Sink sink,
                         hipStream_t st, int dev, u64 blocks) {
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt snt = NtSink<Sink>::make(sink);
  if (hook_small(keylen, k, n, algo, sink, st, dev, blocks) != kNoVariant) return;
  if constexpr (std::is_same<Sink, SinkPlace>::value) {
    // With a histogram: 1024-thread workgroups, 2 per CU.  Every workgroup
    // flushes its LDS bins with one device-scope atomic per bin, and those
    // run at the memory-side atomic rate (~1.3 TB/s of added bytes): 2048
    // workgroups x 1024 bins x 8 B took ~16 us of an 85-us launch; a quarter
    // as many workgroups measured +24 % (8-B keys) and +29 % (16-B keys) on
    // 16M keys, 1024 ranks (profiles/r01/placebench_*).
    // (r02, tools/abbench.py place8_*: 8-B keys stream best at ONE such
    // workgroup per CU -- 0.80 of the roofline against 0.74 at two, half the
    // flushes again; 16-B keys stay at two)
    // 8 keys per lane in flight (late r04, HBM-resident keys: 0.621 -> 0.681
    // against 4; 16: 0.629; profiles/r04/ab/ab_placerot_shapes.log)
    if (sink.hist && keylen == 8) {
      g_kernel = PDHT_PLACE8_NT ? "k_fixed_direct<8,8,nt,1024>@1" : "k_fixed_direct<8,8,nt-store,1024>@1";
      k_fixed_direct<8, 8, Algo, SinkNt, PDHT_PLACE8_NT, 1024>
          <<<grid_for((blocks + 31) / 32, 1, dev), 1024, 0, st>>>(k, n, algo, snt);
      return;
    }
    if (sink.hist && keylen == 16) {
      g_kernel = "k_fixed_direct<16,2,nt,1024>@2";
      k_fixed_direct<16, 2, Algo, SinkNt, true, 1024>
          <<<grid_for((blocks + 7) / 8, 2, dev), 1024, 0, st>>>(k, n, algo, snt);
      return;
    }
  }
  if (keylen == 8) {
    // non-temporal loads since late r04: 0.659 -> 0.712 with HBM-resident
    // keys (r01's plain loads were chosen on a cache-resident buffer;
    // profiles/r04/ab/ab_city8rot.log)
    g_kernel = "k_fixed_direct<8,4,nt>@8";
    k_fixed_direct<8, 4, Algo, SinkNt, true><<<grid_for((blocks + 3) / 4, 8, dev), kBlock, 0, st>>>(
        k, n, algo, snt);
  } else if (keylen == 16) {
    g_kernel = "k_fixed_direct<16,2,nt>@8";
    k_fixed_direct<16, 2, Algo, SinkNt, true><<<grid_for((blocks + 1) / 2, 8, dev), kBlock, 0, st>>>(
        k, n, algo, snt);
  } else {
    // non-temporal loads and stores since late r04: 0.628 -> 0.688 with
    // HBM-resident keys (profiles/r04/ab/ab_city32rot.log)
    g_kernel = "k_fixed_direct<32,2,nt>@8";
    k_fixed_direct<32, 2, Algo, SinkNt, true><<<grid_for((blocks + 1) / 2, 8, dev), kBlock, 0, st>>>(k, n, algo,
                                                                                                    snt);
  }
}

template <class Sink>
static bool sink_has_hist(const Sink &s) {
  if constexpr (std::is_same<Sink, SinkPlace>::value) return s.hist != nullptr;
  return false;
}

// Fixed-length keys: the register-direct / LDS-transposed kernels for the
// specialised lengths when the layout allows them, else the window kernel
// (a 64-key tile fits 12 or 16 KiB of LDS), else per-lane global reads.
// Batches larger than this many key bytes go out as consecutive launches of
// about this size.  One persistent launch over a large batch streams slower
// than the same keys in shorter launches: over a long launch the waves drift
// apart and the memory the chip has in flight spreads over ever more of the
// buffer.  Interleaved A/B (tools/abbench.py, r03), 64-B keys, ms per batch:
//   chunk               cfg5 128M keys (8 GiB)    cfg2 16M keys (1 GiB)
//   one launch          1.806 (0.669)             0.2034 (0.742)
//   4 GiB / 2 GiB       -     / 1.675             -
//   1 GiB               1.614 (0.749)             0.2031
//   512 MiB             1.579 (0.765)             0.1999 (0.755)
//   256 MiB             1.592                     0.2011
// (cfg3's window kernel is indifferent: 1.92 ms at 0.5-2 GiB, 1.94 in one.)
constexpr u64 kLaunchBytes = 512ull << 20;
static u64 launch_chunk_bytes() { return hook_chunk_bytes(kLaunchBytes); }

template <class Algo, class Sink>
static int launch_fixed_one(const void *keys, size_t stride, size_t keylen, size_t n, Algo algo, Sink sink,
                            hipStream_t st);

// Fixed-length keys in launches of about launch_chunk_bytes() each.
template <class Algo, class Sink>
static int launch_fixed(const void *keys, size_t stride, size_t keylen, size_t n, Algo algo, Sink sink,
                        hipStream_t st) {
  const u64 per = std::max<u64>(1, launch_chunk_bytes() / std::max<u64>(stride, 1));
  // Keys too long for a 64-key window (k_global: per-lane walks, compute-
  // heavy) go out in ONE launch: every launch ends in a tail of idle CUs, and
  // these kernels gain nothing from short launches (r03 A/B, 1M x 1 KiB:
  // Crc128 0.544 -> 0.566, CityHash64 0.659 -> 0.672; profiles/r03/ab).
  const bool long_keys = 63 * (u64)stride + keylen + 16 > 16384;
  if (n <= per || stride == 0 || long_keys) return launch_fixed_one(keys, stride, keylen, n, algo, sink, st);
  const u64 step = (per + 4095) & ~(u64)4095;  // whole 64-key tiles (and 4096-key blocks)
  const char *tag = "";
  for (u64 k0 = 0; k0 < n; k0 += step) {
    const u64 c = std::min<u64>(step, n - k0);
    if (int rc = launch_fixed_one(static_cast<const uint8_t *>(keys) + k0 * stride, stride, keylen, c, algo,
                                  sink.shift(k0), st))
      return rc;
    if (k0 == 0) tag = g_kernel;
  }
  g_kernel = tag;  // the tag of the full-size launches
  return 0;
}

template <class Algo, class Sink>
static int launch_fixed_one(const void *keys, size_t stride, size_t keylen, size_t n, Algo algo,
                        Sink sink, hipStream_t st) {
  if (n == 0) return 0;
  if (!keys && keylen) return fail("null key pointer%s", "");  // empty keys read nothing
  if (stride < keylen) return fail("stride < keylen%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  const uint8_t *k = static_cast<const uint8_t *>(keys);
  const bool packed = stride == keylen;
  const bool al16 = ((uintptr_t)k & 15) == 0;
  const bool al8 = ((uintptr_t)k & 7) == 0;
  const u64 blocks = (n + kBlock - 1) / kBlock;
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt sink_nt = NtSink<Sink>::make(sink);
  // the CRC-table algorithms serve keys > 900 B only: window / global kernels
  constexpr bool kShort = !HasCrcLds<Algo>::value;
  if (kShort && packed && keylen == 64 && al16) {
    if constexpr (kShort)
      if (int rc = hook_xpose64(k, n, algo, sink, st, dev); rc != kNoVariant) return rc;
    // measured fastest (profiles/r01/kbench_*): non-temporal loads
    // and stores, two tiles of prefetch in flight per wave, 3 workgroups/CU.
    // Placement with a histogram on up to 4M keys: 1024-thread workgroups, 1
    // per CU -- every workgroup ends with one device-scope atomic per bin, and
    // with few ranks those all hit one cache line: 768 flushing workgroups
    // cost ~6 us of a 24-us launch on 1M keys (cfg1), 256 cost ~1 us
    // (tools/abbench.py cfg1: 24.3 -> 18.3 us); on 16M keys the wide shape
    // streams 3-5 % slower and the 256-thread one stays.
    if constexpr (kShort) {
      if (sink_has_hist(sink) && n <= (4u << 20)) {
        g_kernel = "k_fixed_xpose64<nt,d2,1024>@1";
        k_fixed_xpose64<Algo, SinkNt, true, 2, 1024><<<grid_for((n + 1023) / 1024, 1, dev), 1024, 0, st>>>(
            k, n, algo, sink_nt);
        HIP_TRY(hipGetLastError());
        return 0;
      }
    }
    g_kernel = "k_fixed_xpose64<nt,d2>@3";
    if constexpr (kShort)
      k_fixed_xpose64<Algo, SinkNt, true, 2><<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, st>>>(
          k, n, algo, sink_nt);
  } else if (kShort && packed && (((keylen == 32 || keylen == 16) && al16) || (keylen == 8 && al8))) {
    if constexpr (kShort) launch_small(keylen, k, n, algo, sink, st, dev, blocks);
  } else if constexpr (!kShort) {
    // CRC-table algorithms (keys > 900 B: their 64-key tiles never fit a
    // window): per-lane global reads, the 6-bit tables in LDS, 8 WG/CU
    // (VGPR-bound to 3 waves per SIMD)
    const unsigned g = grid_for(blocks, 8, dev);
    if (int rc = hook_crc_long(k, stride, keylen, n, algo, sink, st, dev, blocks); rc != kNoVariant) return rc;
    if (al16 && stride % 16 == 0) {
      g_kernel = "k_global<fixed,a16,lines>@8";
      k_global<false, Algo, SinkNt, true, kLongLines><<<g, kBlock, 0, st>>>(k, nullptr, 0, stride, keylen, n,
                                                                             algo, sink_nt);
    } else {
      g_kernel = "k_global<fixed>@8";
      k_global<false, Algo, SinkNt><<<g, kBlock, 0, st>>>(k, nullptr, 0, stride, keylen, n, algo, sink_nt);
    }
  } else {
    const u64 tiles = (n + 63) / 64;
    const u64 tile_bytes = 63 * (u64)stride + keylen + 16;  // a 64-key tile + alignment slack
    if (tile_bytes > 16384) {
      // keys too long for a 64-key window: per-lane global reads (r01: an
      // LDS chunk-streaming kernel measured 0.36-0.47 of peak against this
      // kernel's 0.50-0.62 on 256 B - 8 KiB keys)
      // 2 WG/CU: the per-lane walks of 64 keys touch 64 lines per wave
      // instruction, and fewer waves keep more of those lines in L2 for the
      // next 16-B pieces (r02, tools/abbench.py long64: 0.575 at 2 WG/CU
      // against 0.535 at 8)
      constexpr int kPerCu = 2;
      if (al16 && stride % 16 == 0) {
        if (int rc = hook_long_walk(k, stride, keylen, n, algo, sink, st, dev, blocks, kPerCu); rc != kNoVariant)
          return rc;
        g_kernel = "k_global<fixed,a16,lines>@2";
        k_global<false, Algo, SinkNt, true, kLongLines><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
            k, nullptr, 0, stride, keylen, n, algo, sink_nt);
      } else {
        g_kernel = "k_global<fixed>@2";
        k_global<false, Algo, SinkNt><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
            k, nullptr, 0, stride, keylen, n, algo, sink_nt);
      }
    } else if (tile_bytes > kWinBytes) {
      g_kernel = "k_window<fixed,nt,16K>@2";
      k_window<16384, false, Algo, SinkNt, 2><<<grid_for((tiles + 3) / 4, 2, dev), kBlock, 0, st>>>(
          k, nullptr, 0, stride, keylen, n, algo, sink_nt);
    } else {  // (10224 B at 4 WG/CU measured 2-4 % slower for fixed keys: longbench r01)
      g_kernel = "k_window<fixed,nt,12K>@3";
      k_window<kWinBytes, false, Algo, SinkNt, 2><<<grid_for((tiles + 3) / 4, 3, dev), kBlock, 0, st>>>(
          k, nullptr, 0, stride, keylen, n, algo, sink_nt);
    }
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

template <class Algo, class Sink>
static int launch_var_one(const void *bytes, u64 nbytes, const u64 *offsets, u64 obase, size_t n, Algo algo,
                          Sink sink, hipStream_t st);

// Variable-length keys in launches of about launch_chunk_bytes() of key bytes
// each (split by key count at the batch's mean length; every launch keeps the
// whole batch's window choice).
template <class Algo, class Sink>
static int launch_var(const void *bytes, u64 nbytes, const u64 *offsets, u64 obase, size_t n, Algo algo,
                      Sink sink, hipStream_t st) {
  const u64 lim = launch_chunk_bytes();
  if (n == 0 || nbytes <= lim) return launch_var_one(bytes, nbytes, offsets, obase, n, algo, sink, st);
  const u64 mean = std::max<u64>(1, nbytes / n);
  const u64 step = std::max<u64>(4096, (lim / mean) & ~(u64)4095);
  const char *tag = "";
  for (u64 k0 = 0; k0 < n; k0 += step) {
    const u64 c = std::min<u64>(step, n - k0);
    if (int rc = launch_var_one(bytes, mean * c, offsets + k0, obase, c, algo, sink.shift(k0), st)) return rc;
    if (k0 == 0) tag = g_kernel;
  }
  g_kernel = tag;
  return 0;
}

// One launch over variable-length keys.  `nbytes` = key bytes the batch
// spans (offsets[n] - offsets[0]; 0 = unknown) sizes the LDS window for the
// mean key length (r01): mean <= 160 B (cfg3's 16..256 mix, mean 136) ->
// 10224 B per wave at 4 workgroups/CU; longer -> 16 KiB at 2.  (Per-lane
// global reads measured slower than the 16 KiB window even at 1-3 KiB keys:
// the window's DMA pulls the lines into L2 for the keys that overflow it.
// r02/r03 measured a double-buffered window, offsets prefetched a tile
// ahead, the next window prefetched in VGPRs, 128-B window alignment and
// length-sorted workgroup windows: none faster)
template <class Algo, class Sink>
static int launch_var_one(const void *bytes, u64 nbytes, const u64 *offsets, u64 obase, size_t n, Algo algo,
                      Sink sink, hipStream_t st) {
  if (n == 0) return 0;
  if (!bytes || !offsets) return fail("null bytes/offsets pointer%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  const uint8_t *b = static_cast<const uint8_t *>(bytes);
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt sink_nt = NtSink<Sink>::make(sink);
  const u64 wb = ((n + 63) / 64 + 3) / 4;  // blocks of 4 wave-tiles
  bool wide = nbytes / n > 160;
  if (int rc = hook_var(b, offsets, obase, n, algo, sink, st, dev, wb, wide); rc != kNoVariant) return rc;
  if (wide) {
    g_kernel = "k_window<var,nt,16K>@2";
    k_window<16384, true, Algo, SinkNt, 2><<<grid_for(wb, 2, dev), kBlock, 0, st>>>(b, offsets, obase, 0, 0, n,
                                                                                    algo, sink_nt);
  } else {
    // s_setprio 1 while a wave fetches its next tile's offsets and issues the
    // window DMA (r04, interleaved: cfg3 +1.8 %, cfg3c +0.8 %; 3 equal to 1;
    // tuning 205 = without)
    g_kernel = "k_window<var,nt,10224>@4";
    k_window<10224, true, Algo, SinkNt, 2, 16, LdsReader, 1><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
        b, offsets, obase, 0, 0, n, algo, sink_nt);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // namespace pdht
