// tuning/pdht_hooks_launch.h -- the TUNING build's alternative launch shapes
// of the hash paths: launch.h calls one hook per path, which the product
// build resolves to product/pdht_hooks_launch.h (none taken) and
// libpdht_hip_tuning.so to this header (-Ipdht_amd/csrc/tuning).  A hook
// returns kNoVariant when the process-wide variant (pdht_hip_set_variant)
// does not concern it, else the launch's status.  Every variant here was
// measured against the product shape (logs in profiles/):
//   64-B keys    7 one tile of prefetch per wave at 4 WG/CU; 26 plain digest
//                stores; 80 / 81 1024-thread transpose at 1 / 2 WG/CU; 82 the
//                256-thread shape whatever the histogram; 188 digests stored
//                16 B per lane; 206 s_setprio 1 around the prefetch issue;
//                250 / 251 the tile order scattered / in per-wave runs
//   small keys   219 / 220 8-B placement with 4 / 16 keys per lane in flight;
//                221 8-B hashing with plain loads; 222 / 223 8 keys per lane
//                (256 / 1024 threads); 224 32-B keys with plain loads and
//                stores; 225 / 226 16-B keys with 4 keys per lane
//   launches     114-118 launch size 256 MiB / 1 / 2 / 4 GiB / one launch
//   long keys    96 the 240-B / 64-B spans before the line spans; 190 / 191
//                CityHashCrc256Long's block loop as a 128-B line stream
//   var keys     12 / 13 force the 10224-B / 16-KiB window; 170-173 the
//                pipelined window kernel; 174 / 175 the r03 funnel reader;
//                180-187 the pipelined kernel's cache policies; 189 16-B
//                digest stores; 203 / 204 s_setprio 3 / 1; 205 no s_setprio;
//                252 workgroup-combined digest stores (2 KiB runs)
#pragma once
#include "pdht_hooks.h"
#include "kernels_tuning.h"

namespace pdht {

static int tuning_launched() {
  HIP_TRY(hipGetLastError());
  return 0;
}

template <class Algo, class Sink>
static int hook_small(size_t keylen, const uint8_t *k, size_t n, Algo algo, Sink sink, hipStream_t st, int dev,
                        u64 blocks) {
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt snt = NtSink<Sink>::make(sink);
  const int v = tuning_variant();
  bool hist = false;
  if constexpr (std::is_same<Sink, SinkPlace>::value) hist = sink.hist != nullptr;
  if (hist && keylen == 8 && (v == 219 || v == 220)) {
    if (v == 219) {
      g_kernel = "k_fixed_direct<8,4,nt,1024>@1";
      k_fixed_direct<8, 4, Algo, SinkNt, true, 1024>
          <<<grid_for((blocks + 15) / 16, 1, dev), 1024, 0, st>>>(k, n, algo, snt);
    } else {
      g_kernel = "k_fixed_direct<8,16,nt,1024>@1";
      k_fixed_direct<8, 16, Algo, SinkNt, true, 1024>
          <<<grid_for((blocks + 63) / 64, 1, dev), 1024, 0, st>>>(k, n, algo, snt);
    }
    return tuning_launched();
  }
  if (hist && keylen == 16 && v == 225) {
    g_kernel = "k_fixed_direct<16,4,nt,1024>@2";
    k_fixed_direct<16, 4, Algo, SinkNt, true, 1024>
        <<<grid_for((blocks + 15) / 16, 2, dev), 1024, 0, st>>>(k, n, algo, snt);
    return tuning_launched();
  }
  if (hist) return kNoVariant;
  if (keylen == 8 && v >= 221 && v <= 223) {
    if (v == 221) {
      g_kernel = "k_fixed_direct<8,4,nt-store>@8";
      k_fixed_direct<8, 4, Algo, SinkNt, false><<<grid_for((blocks + 3) / 4, 8, dev), kBlock, 0, st>>>(k, n, algo,
                                                                                                      snt);
    } else if (v == 222) {
      g_kernel = "k_fixed_direct<8,8,nt>@8";
      k_fixed_direct<8, 8, Algo, SinkNt, true><<<grid_for((blocks + 7) / 8, 8, dev), kBlock, 0, st>>>(k, n, algo,
                                                                                                     snt);
    } else {
      g_kernel = "k_fixed_direct<8,8,nt,1024>@1";
      k_fixed_direct<8, 8, Algo, SinkNt, true, 1024>
          <<<grid_for((blocks + 31) / 32, 1, dev), 1024, 0, st>>>(k, n, algo, snt);
    }
    return tuning_launched();
  }
  if (keylen == 16 && v == 226) {
    g_kernel = "k_fixed_direct<16,4,nt>@8";
    k_fixed_direct<16, 4, Algo, SinkNt, true><<<grid_for((blocks + 3) / 4, 8, dev), kBlock, 0, st>>>(k, n, algo,
                                                                                                    snt);
    return tuning_launched();
  }
  if (keylen == 32 && v == 224) {
    g_kernel = "k_fixed_direct<32,2>@8";
    k_fixed_direct<32, 2, Algo, Sink><<<grid_for((blocks + 1) / 2, 8, dev), kBlock, 0, st>>>(k, n, algo, sink);
    return tuning_launched();
  }
  return kNoVariant;
}

// launch size (bytes of keys per launch); dflt = the product's
static u64 hook_chunk_bytes(u64 dflt) {
  switch (tuning_variant()) {
    case 114: return 256ull << 20;
    case 115: return 1ull << 30;
    case 116: return 2ull << 30;
    case 117: return 4ull << 30;
    case 118: return ~0ull;
    default: return dflt;
  }
}

// packed, 16-B aligned 64-B keys
template <class Algo, class Sink>
static int hook_xpose64(const uint8_t *k, size_t n, Algo algo, Sink sink, hipStream_t st, int dev) {
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt sink_nt = NtSink<Sink>::make(sink);
  switch (tuning_variant()) {
    case 7:  // one tile of prefetch per wave, 4 WG/CU (r01: 2-5 % slower)
      g_kernel = "k_fixed_xpose64<nt,d1>@4";
      k_fixed_xpose64<Algo, SinkNt, true, 1><<<grid_for((n + 255) / 256, 4, dev), kBlock, 0, st>>>(k, n, algo,
                                                                                                  sink_nt);
      return tuning_launched();
    case 80:
    case 81:  // 1024-thread workgroups, 1 / 2 per CU
      g_kernel = tuning_variant() == 80 ? "k_fixed_xpose64<nt,d2,1024>@1" : "k_fixed_xpose64<nt,d2,1024>@2";
      k_fixed_xpose64<Algo, SinkNt, true, 2, 1024>
          <<<grid_for((n + 1023) / 1024, tuning_variant() == 80 ? 1 : 2, dev), 1024, 0, st>>>(k, n, algo, sink_nt);
      return tuning_launched();
    case 82:  // the 256-thread shape whatever the histogram
      g_kernel = "k_fixed_xpose64<nt,d2>@3";
      k_fixed_xpose64<Algo, SinkNt, true, 2><<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, st>>>(k, n, algo,
                                                                                                  sink_nt);
      return tuning_launched();
    case 206:  // s_setprio 1 around each wave's prefetch issue
      g_kernel = "k_fixed_xpose64<nt,d2,prio1>@3";
      k_fixed_xpose64<Algo, SinkNt, true, 2, kBlock, 1><<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, st>>>(
          k, n, algo, sink_nt);
      return tuning_launched();
    case 188:  // digests stored 16 B per lane (even lanes, DPP pairs)
      if constexpr (std::is_same<Sink, Sink64>::value) {
        g_kernel = "k_fixed_xpose64<nt,d2,st16>@3";
        k_fixed_xpose64<Algo, Sink64x2T<true>, true, 2><<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, st>>>(
            k, n, algo, Sink64x2T<true>{nullptr, sink.out});
        return tuning_launched();
      }
      return kNoVariant;
    case 250:
    case 251: {  // r05: scattered (power-of-two tile counts) / wave-contiguous tile order, whole tiles
      const u64 ntiles = n >> 6;
      const unsigned g = grid_for((n + 255) / 256, 3, dev);
      if (n % 64 || ntiles == 0) return kNoVariant;
      if (tuning_variant() == 250 && (ntiles & (ntiles - 1))) return kNoVariant;
      if (tuning_variant() == 250) {
        g_kernel = "k_fixed_xpose64_order<scatter>@3";
        k_fixed_xpose64_order<Algo, SinkNt, 1><<<g, kBlock, 0, st>>>(k, n, algo, sink_nt);
      } else {
        g_kernel = "k_fixed_xpose64_order<runs>@3";
        k_fixed_xpose64_order<Algo, SinkNt, 2><<<g, kBlock, 0, st>>>(k, n, algo, sink_nt);
      }
      return tuning_launched();
    }
    case 26:  // plain digest stores (r01: 2-6 % slower)
      g_kernel = "k_fixed_xpose64<nt-load,plain-store,d2>@3";
      k_fixed_xpose64<Algo, Sink, true, 2><<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, st>>>(k, n, algo, sink);
      return tuning_launched();
    default:
      return kNoVariant;
  }
}

// CRC-table algorithms on keys > 900 B (16-B aligned rows only)
template <class Algo, class Sink>
static int hook_crc_long(const uint8_t *k, size_t stride, size_t keylen, size_t n, Algo algo, Sink sink,
                         hipStream_t st, int dev, u64 blocks) {
  if (((uintptr_t)k & 15) || stride % 16) return kNoVariant;
  const int v = tuning_variant();
  if (v >= 279 && v <= 281 && stride == keylen && (keylen == 1024 || keylen == 2048 || keylen == 4096)) {
    // the LDS-DMA ring (k_long_ring): R = 4 / 2 / 3 line-rounds per wave
    typedef typename NtSink<Sink>::type SinkNt;
    const SinkNt sink_nt = NtSink<Sink>::make(sink);
    const int R = v == 279 ? 4 : v == 280 ? 2 : 3;
    const int per_cu = R == 2 ? 2 : 1;
    const size_t lds = (size_t)4 * R * 8192;
    const unsigned g = (unsigned)std::min<u64>((n + 255) / 256, (u64)std::max(1, g_dev[dev].cus) * per_cu);
    auto go = [&](auto kern, const char *tag) {
      HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
      g_kernel = tag;
      kern<<<g, 256, lds, st>>>(k, n, algo, sink_nt);
      return tuning_launched();
    };
#define PDHT_RING(LL, RR) \
  if (keylen == LL && R == RR) return go(&k_long_ring<LL, RR, Algo, SinkNt>, "k_long_ring<" #LL "," #RR ">");
    PDHT_RING(1024, 4) PDHT_RING(1024, 2) PDHT_RING(1024, 3)
    PDHT_RING(2048, 4) PDHT_RING(2048, 2) PDHT_RING(2048, 3)
    PDHT_RING(4096, 4) PDHT_RING(4096, 2) PDHT_RING(4096, 3)
#undef PDHT_RING
  }
  if (v != 190 && v != 191) return kNoVariant;
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt sink_nt = NtSink<Sink>::make(sink);
  const int pc = v == 190 ? 8 : 4;  // CityHashCrc256Long's block loop as a 128-B line stream
  g_kernel = pc == 8 ? "k_global<fixed,a16,stream>@8" : "k_global<fixed,a16,stream>@4";
  k_global<false, Algo, SinkNt, true, kLongStream><<<grid_for(blocks, pc, dev), kBlock, 0, st>>>(
      k, nullptr, 0, stride, keylen, n, algo, sink_nt);
  return tuning_launched();
}

// fixed keys too long for a 64-key window, 16-B aligned rows
template <class Algo, class Sink>
static int hook_long_walk(const uint8_t *k, size_t stride, size_t keylen, size_t n, Algo algo, Sink sink,
                            hipStream_t st, int dev, u64 blocks, int per_cu) {
  if (tuning_variant() != 96) return kNoVariant;
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt sink_nt = NtSink<Sink>::make(sink);
  g_kernel = "k_global<fixed,a16>@2";  // r02 before the line spans: spans as the algorithm reads them
  k_global<false, Algo, SinkNt, true><<<grid_for(blocks, per_cu, dev), kBlock, 0, st>>>(k, nullptr, 0, stride,
                                                                                       keylen, n, algo, sink_nt);
  return tuning_launched();
}

// variable-length keys; may also force the window width (12 / 13)
template <class Algo, class Sink>
static int hook_var(const uint8_t *b, const u64 *offsets, u64 obase, size_t n, Algo algo, Sink sink,
                      hipStream_t st, int dev, u64 wb, bool &wide) {
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt sink_nt = NtSink<Sink>::make(sink);
  const int v = tuning_variant();
  if (v == 12) wide = false;
  if (v == 13) wide = true;
  if (!wide && v == 205) {  // the product window kernel without s_setprio
    g_kernel = "k_window<var,nt,10224>@4";
    k_window<10224, true, Algo, SinkNt, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, 0, 0, n,
                                                                                    algo, sink_nt);
    return tuning_launched();
  }
  if constexpr (std::is_same<Algo, AlgoCity64>::value && std::is_same<Sink, Sink64>::value) {
    if (v >= 180 && v <= 187) {  // cache policies of the pipe kernel's DMA / digest stores
      auto go = [&](auto kern, const char *tag) {
        g_kernel = tag;
        kern<<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo, sink.out);
      };
      switch (v) {
        case 180: go(k_window_pipe<10224, 1, Algo, 2, LdsReader, 0, 0>, "k_window_pipe<dma nt,st plain>"); break;
        case 181: go(k_window_pipe<10224, 1, Algo, 2, LdsReader, 0, 1>, "k_window_pipe<dma nt,st sc0>"); break;
        case 182: go(k_window_pipe<10224, 1, Algo, 2, LdsReader, 0, 16>, "k_window_pipe<dma nt,st sc1>"); break;
        case 183: go(k_window_pipe<10224, 1, Algo, 2, LdsReader, 0, 18>, "k_window_pipe<dma nt,st sc1 nt>"); break;
        case 184: go(k_window_pipe<10224, 1, Algo, 2, LdsReader, 0, 19>, "k_window_pipe<dma nt,st sc0 sc1 nt>"); break;
        case 185: go(k_window_pipe<10224, 1, Algo, 0, LdsReader, 0, 2>, "k_window_pipe<dma plain,st nt>"); break;
        case 186: go(k_window_pipe<10224, 1, Algo, 3, LdsReader, 0, 2>, "k_window_pipe<dma sc0 nt,st nt>"); break;
        default: go(k_window_pipe<10224, 1, Algo, 16, LdsReader, 0, 2>, "k_window_pipe<dma sc1,st nt>"); break;
      }
      return tuning_launched();
    }
    if (v == 203 || v == 204) {  // the product window kernel, s_setprio 3 / 1 around the fetch phase
      g_kernel = v == 203 ? "k_window<var,nt,10224,prio3>@4" : "k_window<var,nt,10224,prio1>@4";
      if (v == 203)
        k_window<10224, true, Algo, Sink64T<true>, 2, 16, LdsReader, 3><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
            b, offsets, obase, 0, 0, n, algo, Sink64T<true>{nullptr, sink.out});
      else
        k_window<10224, true, Algo, Sink64T<true>, 2, 16, LdsReader, 1><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
            b, offsets, obase, 0, 0, n, algo, Sink64T<true>{nullptr, sink.out});
      return tuning_launched();
    }
    if (v == 252 && !wide) {  // r05: workgroup-combined digest stores (super-tiles of 4 consecutive tiles)
      g_kernel = "k_window_wc<var,10224>@4";
      k_window_wc<10224, Algo><<<grid_for(((n + 63) / 64 + 3) / 4, 4, dev), kBlock, 0, st>>>(b, offsets, obase, n,
                                                                                          algo, sink.out);
      return tuning_launched();
    }
    if (v == 189) {  // the product window kernel, digests stored 16 B per lane
      g_kernel = "k_window<var,nt,10224,st16>@4";
      k_window<10224, true, Algo, Sink64x2T<true>, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets, obase, 0, 0, n, algo, Sink64x2T<true>{nullptr, sink.out});
      return tuning_launched();
    }
    if (v == 174 || v == 175) {  // 174: pipe kernel, r03 funnel reader; 175: product kernel, r03 reader
      if (v == 174) {
        g_kernel = "k_window_pipe<var,10224,G1,funnel>@4";
        k_window_pipe<10224, 1, Algo, 2, LdsReaderFunnel><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
            b, offsets, obase, n, algo, sink.out);
      } else {
        g_kernel = "k_window<var,nt,10224,funnel>@4";
        k_window<10224, true, Algo, Sink64T<true>, 2, 16, LdsReaderFunnel>
            <<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, 0, 0, n, algo,
                                                     Sink64T<true>{nullptr, sink.out});
      }
      return tuning_launched();
    }
    if (v >= 170 && v <= 173) {  // pipelined window kernel (offsets a tile ahead, stores a tile late)
      const int pc = v == 173 ? 3 : 4;
      if (v == 170 || v == 173) {
        g_kernel = v == 170 ? "k_window_pipe<var,10224,G1>@4" : "k_window_pipe<var,10224,G1>@3";
        k_window_pipe<10224, 1, Algo, 2><<<grid_for(wb, pc, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                     sink.out);
      } else if (v == 171) {
        g_kernel = "k_window_pipe<var,10224,G4>@4";
        k_window_pipe<10224, 4, Algo, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                    sink.out);
      } else {
        g_kernel = "k_window_pipe<var,10224,G16>@4";
        k_window_pipe<10224, 16, Algo, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                     sink.out);
      }
      return tuning_launched();
    }
  }
  return kNoVariant;
}

}  // namespace pdht
