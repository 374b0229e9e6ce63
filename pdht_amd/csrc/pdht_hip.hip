// pdht_hip.hip -- C-ABI of the batch key-hashing engine (include/pdht_hip.h).
//
// Launch logic, per-device state, and the host-resident streaming pipeline.
// Kernels: kernels.h.  Algorithm: city_core.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "../../include/pdht_hip.h"
#include "bucket.h"
#include "kernels.h"

#define PDHT_API extern "C" __attribute__((visibility("default")))

namespace pdht {

// ------------------------------------------------------------- errors ---
static thread_local char g_err[512] = "";
static thread_local const char *g_kernel = "";

static int fail(const char *fmt, const char *a = "", long long b = 0) {
  snprintf(g_err, sizeof g_err, fmt, a, b);
  return PDHT_HIP_ERROR;
}
#define HIP_TRY(expr)                                                              \
  do {                                                                             \
    hipError_t e_ = (expr);                                                        \
    if (e_ != hipSuccess) return fail("%s (" #expr ")", hipGetErrorString(e_)); \
  } while (0)

// Tuning build (libpdht_hip_tuning.so, -DPDHT_HIP_TUNING; tools/ and the
// A/B tests only): a process-wide variant number selects an alternative
// kernel where one exists, and the workgroups per CU can be overridden.  The
// product library has neither: one measured-best kernel per path, no
// process-global mutable state, no environment knobs.
#ifdef PDHT_HIP_TUNING
static std::atomic<int> g_variant{0};
static std::atomic<int> g_per_cu{0};
static int tuning_variant() { return g_variant.load(std::memory_order_relaxed); }
#endif

// ------------------------------------------------------- device state ---
constexpr int kMaxDev = 64;
struct DevInfo {
  std::once_flag once;
  int cus = 0;
  hipError_t err = hipSuccess;
};
static DevInfo g_dev[kMaxDev];

static int current_device(int *dev) {
  HIP_TRY(hipGetDevice(dev));
  if (*dev < 0 || *dev >= kMaxDev) return fail("device index %s%lld out of range", "", *dev);
  DevInfo &d = g_dev[*dev];
  std::call_once(d.once, [&] {
    d.err = hipDeviceGetAttribute(&d.cus, hipDeviceAttributeMultiprocessorCount, *dev);
  });
  if (d.err != hipSuccess) return fail("%s (querying CU count)", hipGetErrorString(d.err));
  return 0;
}

// Persistent grid: enough workgroups to keep every CU at `per_cu` blocks,
// never more than the work needs.
static unsigned grid_for(u64 work_blocks, int per_cu, int dev) {
#ifdef PDHT_HIP_TUNING
  if (const int o = g_per_cu.load(std::memory_order_relaxed)) per_cu = o;
#endif
  const u64 cap = (u64)std::max(1, g_dev[dev].cus) * per_cu;
  return (unsigned)std::max<u64>(1, std::min<u64>(work_blocks, cap));
}

static FastMod make_fastmod(u64 d) {
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
constexpr int kWinBytes = 12288;  // k_window over fixed keys: LDS window per wave (12 KiB)
// Kernel tags (pdht_hip_last_kernel): the kernel and its launch shape, so a
// profile taken of one shape (profiles/traffic_*.json) is never attributed to
// another.

// Packed 8/16/32-byte keys: each lane loads its own key (lane-adjacent rows,
// so 8- and 16-byte keys are fully coalesced), U keys in flight per lane.
// tools/placebench.py (interleaved A/B, r01): 8-B keys with non-temporal
// stores (+26 % on fused placement), 16-B keys with non-temporal loads and
// stores (+6-11 %).
template <class Algo, class Sink>
static void launch_small(size_t keylen, const uint8_t *k, size_t n, Algo algo, Sink sink,
                         hipStream_t st, int dev, u64 blocks) {
  typedef typename NtSink<Sink>::type SinkNt;
  const SinkNt snt = NtSink<Sink>::make(sink);
  if constexpr (std::is_same<Sink, SinkPlace>::value) {
    // With a histogram: 1024-thread workgroups, 2 per CU.  Every workgroup
    // flushes its LDS bins with one device-scope atomic per bin, and those
    // run at the memory-side atomic rate (~1.3 TB/s of added bytes): 2048
    // workgroups x 1024 bins x 8 B took ~16 us of an 85-us launch; a quarter
    // as many workgroups measured +24 % (8-B keys) and +29 % (16-B keys) on
    // 16M keys, 1024 ranks (tools/placebench.py, r01).
    // (r02, tools/abbench.py place8_*: 8-B keys stream best at ONE such
    // workgroup per CU -- 0.80 of the roofline against 0.74 at two, half the
    // flushes again; 16-B keys stay at two)
    if (sink.hist && keylen == 8) {
      g_kernel = "k_fixed_direct<8,4,nt-store,1024>@1";
      k_fixed_direct<8, 4, Algo, SinkNt, false, 1024>
          <<<grid_for((blocks + 15) / 16, 1, dev), 1024, 0, st>>>(k, n, algo, snt);
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
    g_kernel = "k_fixed_direct<8,4,nt-store>@8";
    k_fixed_direct<8, 4, Algo, SinkNt, false><<<grid_for((blocks + 3) / 4, 8, dev), kBlock, 0, st>>>(
        k, n, algo, snt);
  } else if (keylen == 16) {
    g_kernel = "k_fixed_direct<16,2,nt>@8";
    k_fixed_direct<16, 2, Algo, SinkNt, true><<<grid_for((blocks + 1) / 2, 8, dev), kBlock, 0, st>>>(
        k, n, algo, snt);
  } else {
    g_kernel = "k_fixed_direct<32,2>@8";
    k_fixed_direct<32, 2, Algo, Sink><<<grid_for((blocks + 1) / 2, 8, dev), kBlock, 0, st>>>(k, n, algo,
                                                                                            sink);
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
template <class Algo, class Sink>
static int launch_fixed(const void *keys, size_t stride, size_t keylen, size_t n, Algo algo,
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
#ifdef PDHT_HIP_TUNING
    if constexpr (kShort) {
      if (tuning_variant() == 7) {  // one tile of prefetch per wave, 4 WG/CU (r01: 2-5 % slower)
        g_kernel = "k_fixed_xpose64<nt,d1>@4";
        k_fixed_xpose64<Algo, SinkNt, true, 1><<<grid_for((n + 255) / 256, 4, dev), kBlock, 0, st>>>(
            k, n, algo, sink_nt);
        HIP_TRY(hipGetLastError());
        return 0;
      }
      if (tuning_variant() == 80 || tuning_variant() == 81) {  // 1024-thread workgroups, 1 / 2 per CU
        g_kernel = tuning_variant() == 80 ? "k_fixed_xpose64<nt,d2,1024>@1" : "k_fixed_xpose64<nt,d2,1024>@2";
        k_fixed_xpose64<Algo, SinkNt, true, 2, 1024>
            <<<grid_for((n + 1023) / 1024, tuning_variant() == 80 ? 1 : 2, dev), 1024, 0, st>>>(k, n, algo,
                                                                                                sink_nt);
        HIP_TRY(hipGetLastError());
        return 0;
      }
      if (tuning_variant() == 82) {  // the 256-thread shape whatever the histogram
        g_kernel = "k_fixed_xpose64<nt,d2>@3";
        k_fixed_xpose64<Algo, SinkNt, true, 2><<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, st>>>(
            k, n, algo, sink_nt);
        HIP_TRY(hipGetLastError());
        return 0;
      }
      if (tuning_variant() == 26) {  // plain digest stores (r01: 2-6 % slower)
        g_kernel = "k_fixed_xpose64<nt-load,plain-store,d2>@3";
        k_fixed_xpose64<Algo, Sink, true, 2><<<grid_for((n + 255) / 256, 3, dev), kBlock, 0, st>>>(
            k, n, algo, sink);
        HIP_TRY(hipGetLastError());
        return 0;
      }
    }
#endif
    // measured fastest (tools/kbench.py): non-temporal loads
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
      // against 0.535 at 8); the CRC path (LDS tables) is indifferent and
      // keeps 8.
      constexpr int kPerCu = kShort ? 2 : 8;
      if (al16 && stride % 16 == 0) {
#ifdef PDHT_HIP_TUNING
        if (tuning_variant() == 93) {  // CRC-256 blocks as whole lines
          g_kernel = "k_global<fixed,a16,lines>";
          k_global<false, Algo, SinkNt, true, 3><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
              k, nullptr, 0, stride, keylen, n, algo, sink_nt);
          HIP_TRY(hipGetLastError());
          return 0;
        }
        if (tuning_variant() == 98) {  // + CityHash128's shifted loop on line spans
          g_kernel = "k_global<fixed,a16,lines16>";
          k_global<false, Algo, SinkNt, true, 7><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
              k, nullptr, 0, stride, keylen, n, algo, sink_nt);
          HIP_TRY(hipGetLastError());
          return 0;
        }
        if (tuning_variant() == 95 || tuning_variant() == 97) {  // 128-B spans (97: one carry array)
          g_kernel = tuning_variant() == 95 ? "k_global<fixed,a16,pairs>" : "k_global<fixed,a16,lines16,1carry>";
          if (tuning_variant() == 97)
            k_global<false, Algo, SinkNt, true, 6><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
                k, nullptr, 0, stride, keylen, n, algo, sink_nt);
          else
            k_global<false, Algo, SinkNt, true, 4><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
                k, nullptr, 0, stride, keylen, n, algo, sink_nt);
          HIP_TRY(hipGetLastError());
          return 0;
        }
        if (tuning_variant() == 96) {  // r02 before the line spans: 240-B / 64-B spans as the algorithm reads them
          g_kernel = kShort ? "k_global<fixed,a16>@2" : "k_global<fixed,a16>@8";
          k_global<false, Algo, SinkNt, true><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
              k, nullptr, 0, stride, keylen, n, algo, sink_nt);
          HIP_TRY(hipGetLastError());
          return 0;
        }
        if (tuning_variant() == 91 || tuning_variant() == 92) {  // nt span loads (all / all but the last line)
          g_kernel = tuning_variant() == 91 ? "k_global<fixed,a16,nt>" : "k_global<fixed,a16,nt-head>";
          if (tuning_variant() == 91)
            k_global<false, Algo, SinkNt, true, 1><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
                k, nullptr, 0, stride, keylen, n, algo, sink_nt);
          else
            k_global<false, Algo, SinkNt, true, 2><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
                k, nullptr, 0, stride, keylen, n, algo, sink_nt);
          HIP_TRY(hipGetLastError());
          return 0;
        }
#endif
        g_kernel = kShort ? "k_global<fixed,a16,lines>@2" : "k_global<fixed,a16,lines>@8";
        k_global<false, Algo, SinkNt, true, kLongLines><<<grid_for(blocks, kPerCu, dev), kBlock, 0, st>>>(
            k, nullptr, 0, stride, keylen, n, algo, sink_nt);
      } else {
        g_kernel = kShort ? "k_global<fixed>@2" : "k_global<fixed>@8";
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

// Variable-length keys.  `nbytes` = key bytes the batch spans
// (offsets[n] - offsets[0]; 0 = unknown) sizes the LDS window for the mean
// key length (tools/varbench.py, r01): mean <= 160 B (cfg3's 16..256 mix,
// mean 136) -> 10224 B per wave at 4 workgroups/CU; longer -> 16 KiB at 2.
// (Per-lane global reads measured slower than the 16 KiB window even at
// 1-3 KiB keys: the window's DMA pulls the lines into L2 for the keys that
// overflow it.)
template <class Algo, class Sink>
static int launch_var(const void *bytes, u64 nbytes, const u64 *offsets, u64 obase, size_t n, Algo algo,
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
#ifdef PDHT_HIP_TUNING
  if (tuning_variant() == 12) wide = false;
  if (tuning_variant() == 13) wide = true;
  if (tuning_variant() == 46) {  // windows start on a 128-B line
    g_kernel = "k_window<var,nt,10224,a128>@4";
    k_window<10224, true, Algo, SinkNt, 2, 128><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, 0, 0,
                                                                                       n, algo, sink_nt);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  if (tuning_variant() >= 23 && tuning_variant() <= 25) {  // double-buffered windows
    if (tuning_variant() == 23) {
      g_kernel = "k_window_db<10224>@2";
      k_window_db<10224, Algo, SinkNt, 2><<<grid_for(wb, 2, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                 sink_nt);
    } else if (tuning_variant() == 24) {
      g_kernel = "k_window_db<6656>@3";
      k_window_db<6656, Algo, SinkNt, 2><<<grid_for(wb, 3, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                sink_nt);
    } else {
      g_kernel = "k_window_db<8192>@2";
      k_window_db<8192, Algo, SinkNt, 2><<<grid_for(wb, 2, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                sink_nt);
    }
    HIP_TRY(hipGetLastError());
    return 0;
  }
  if (tuning_variant() == 48 || tuning_variant() == 49) {  // next window prefetched in VGPRs (48: nt loads)
    g_kernel = tuning_variant() == 48 ? "k_window_rp<10224,nt>@4" : "k_window_rp<10224>@4";
    if (tuning_variant() == 48)
      k_window_rp<10224, Algo, SinkNt, true><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                    sink_nt);
    else
      k_window_rp<10224, Algo, SinkNt, false><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                     sink_nt);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  if (tuning_variant() == 30 || tuning_variant() == 31) {  // offsets prefetched one tile ahead
    if (tuning_variant() == 31 || wide) {
      g_kernel = "k_window_var<16K>@2";
      k_window_var<16384, Algo, SinkNt, 2><<<grid_for(wb, 2, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                  sink_nt);
    } else {
      g_kernel = "k_window_var<10224>@4";
      k_window_var<10224, Algo, SinkNt, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, n, algo,
                                                                                  sink_nt);
    }
    HIP_TRY(hipGetLastError());
    return 0;
  }
#endif
  if (wide) {
    g_kernel = "k_window<var,nt,16K>@2";
    k_window<16384, true, Algo, SinkNt, 2><<<grid_for(wb, 2, dev), kBlock, 0, st>>>(b, offsets, obase, 0, 0, n,
                                                                                    algo, sink_nt);
  } else {
    g_kernel = "k_window<var,nt,10224>@4";
    k_window<10224, true, Algo, SinkNt, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(b, offsets, obase, 0, 0, n,
                                                                                    algo, sink_nt);
  }
  HIP_TRY(hipGetLastError());
  return 0;
}

static SinkPlace make_place_sink(u64 *mbits, u32 *ptindex, void *rank, size_t rank_stride,
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

static int check_place(size_t n, const u64 *mbits, u32 nptes, u32 nranks, const void *rank,
                       size_t rank_stride) {
  if (n && !mbits) return fail("mbits must not be NULL%s", "");
  if (nptes == 0) return fail("nptes must be >= 1 (hash.c:27 divides by it)%s", "");
  if (nranks == 0) return fail("nranks must be >= 1 (hash.c:29 divides by it)%s", "");
  if (nranks > 0x7fffffffu) return fail("nranks is c->size, an int: must be < 2^31%s", "");
  if (rank && rank_stride < 4) return fail("rank_stride must be >= 4%s", "");
  return 0;
}

// ------------------------------------------------- host-resident path ---
// Per-device streaming context: NS slots, each with a stream, device
// buffers and pinned staging, used round-robin so chunk c+1's H2D overlaps
// chunk c's kernel and chunk c-1's D2H.
constexpr int kSlots = 3;
constexpr size_t kChunkBytes = 32u << 20;  // key bytes per chunk

struct Slot {
  hipStream_t st = nullptr;
  hipEvent_t done = nullptr;
  uint8_t *d_in = nullptr;    // keys (and offsets after them for var)
  uint8_t *d_out = nullptr;   // digests / placement outputs
  uint8_t *h_in = nullptr;    // pinned staging (pageable inputs)
  uint8_t *h_out = nullptr;   // pinned staging (pageable outputs)
  size_t in_cap = 0, out_cap = 0;
  // pending harvest of staged outputs
  struct Copy {
    void *dst;
    size_t off, bytes;
  };
  std::vector<Copy> pending;
  bool busy = false;
};
struct HostCtx {
  std::mutex mu;
  bool ready = false;
  Slot slot[kSlots];
};
static HostCtx g_host[kMaxDev];

static bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Device-side address of pinned host memory (nullptr if p is not pinned or
// not mapped for the device).
static void *pinned_device_ptr(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  return a.devicePointer;
}

// Zero-copy host batch: run `launch()` (kernels on device addresses of pinned
// host buffers) on `device` and wait for it.
template <class Launch>
static int zero_copy_run(int device, Launch launch) {
  if (device < 0 || device >= kMaxDev) return fail("device index %s%lld out of range", "", device);
  int prev = -1;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(device));
  int rc = launch();
  if (rc == 0) {
    hipError_t e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) rc = fail("%s (zero-copy batch)", hipGetErrorString(e));
  }
  (void)hipSetDevice(prev);
  return rc;
}
#ifdef PDHT_HIP_TUNING
static bool zero_copy_allowed() { return tuning_variant() != 61; }  // 61: chunked copies (A/B)
#else
static constexpr bool zero_copy_allowed() { return true; }
#endif

static int slot_reserve(Slot &s, size_t in_bytes, size_t out_bytes) {
  if (!s.st) HIP_TRY(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
  if (!s.done) HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
  if (in_bytes > s.in_cap) {
    if (s.d_in) HIP_TRY(hipFree(s.d_in));
    if (s.h_in) HIP_TRY(hipHostFree(s.h_in));
    s.d_in = nullptr;
    s.h_in = nullptr;
    HIP_TRY(hipMalloc(&s.d_in, in_bytes));
    HIP_TRY(hipHostMalloc(&s.h_in, in_bytes, hipHostMallocDefault));
    s.in_cap = in_bytes;
  }
  if (out_bytes > s.out_cap) {
    if (s.d_out) HIP_TRY(hipFree(s.d_out));
    if (s.h_out) HIP_TRY(hipHostFree(s.h_out));
    s.d_out = nullptr;
    s.h_out = nullptr;
    HIP_TRY(hipMalloc(&s.d_out, out_bytes));
    HIP_TRY(hipHostMalloc(&s.h_out, out_bytes, hipHostMallocDefault));
    s.out_cap = out_bytes;
  }
  return 0;
}

// Wait for the slot's previous chunk and copy its staged outputs out.
static int slot_drain(Slot &s) {
  if (!s.busy) return 0;
  HIP_TRY(hipEventSynchronize(s.done));
  for (auto &c : s.pending) memcpy(c.dst, s.h_out + c.off, c.bytes);
  s.pending.clear();
  s.busy = false;
  return 0;
}

// One output array of a chunk: device region [doff, doff+bytes) of d_out goes
// to host `dst` (pinned: DMA directly; pageable: via h_out + harvest).
static int chunk_out(Slot &s, void *dst, bool pinned, size_t doff, size_t bytes) {
  if (bytes == 0) return 0;
  if (pinned) {
    HIP_TRY(hipMemcpyAsync(dst, s.d_out + doff, bytes, hipMemcpyDeviceToHost, s.st));
  } else {
    HIP_TRY(hipMemcpyAsync(s.h_out + doff, s.d_out + doff, bytes, hipMemcpyDeviceToHost, s.st));
    s.pending.push_back(Slot::Copy{dst, doff, bytes});
  }
  return 0;
}

static int chunk_in(Slot &s, const void *src, bool pinned, size_t doff, size_t bytes) {
  if (bytes == 0) return 0;
  const void *from = src;
  if (!pinned) {
    memcpy(s.h_in + doff, src, bytes);
    from = s.h_in + doff;
  }
  HIP_TRY(hipMemcpyAsync(s.d_in + doff, from, bytes, hipMemcpyHostToDevice, s.st));
  return 0;
}

// Drive a chunked host-resident batch.  `plan(c, &k0, &k1)` yields chunk c's
// key range (false when done); `run(slot, k0, k1)` stages, launches and
// queues the copies of one chunk on slot.st.
template <class Plan, class Run>
static int host_pipeline(int device, Plan plan, Run run) {
  if (device < 0 || device >= kMaxDev) return fail("device index %s%lld out of range", "", device);
  int prev = -1;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(device));
  HostCtx &H = g_host[device];
  std::lock_guard<std::mutex> lock(H.mu);
  int rc = 0;
  size_t k0, k1;
  for (size_t c = 0; rc == 0 && plan(c, &k0, &k1); ++c) {
    Slot &s = H.slot[c % kSlots];
    rc = slot_drain(s);
    if (rc == 0) {
      rc = run(s, k0, k1);
      if (rc != 0) {
        // a chunk that failed half-way may already have queued copies and
        // harvest entries: let them finish, then forget them, so the slot
        // never copies into this call's buffers after it has returned
        if (s.st) (void)hipStreamSynchronize(s.st);
        s.pending.clear();
        s.busy = false;
      }
    }
    if (rc == 0) {
      hipError_t e = hipEventRecord(s.done, s.st);
      if (e != hipSuccess) rc = fail("%s (hipEventRecord)", hipGetErrorString(e));
      s.busy = true;
    }
  }
  for (int i = 0; i < kSlots; ++i) {
    int r2 = slot_drain(H.slot[i]);
    if (rc == 0) rc = r2;
  }
  (void)hipSetDevice(prev);
  return rc;
}

// Fixed-length host batch with a per-chunk device launcher.
template <class Launch>
static int host_fixed(const void *keys, size_t keylen, size_t n, size_t out_per_key,
                      void *out, int device, Launch launch) {
  if (n == 0) return 0;
  if (!keys || !out || keylen == 0) return fail("null pointer or zero keylen%s", "");
  const size_t per = std::max<size_t>(1, kChunkBytes / keylen);
  const bool pin_in = is_pinned(keys), pin_out = is_pinned(out);
  // Pinned keys and digests: zero-copy.  The kernel itself reads the keys
  // and writes the digests over PCIe, no staging copies: 0.87 vs 0.75
  // Gkeys/s on 16M x 64 B (62 vs 54 GB/s of PCIe traffic, r01).
  void *zk = pin_in && pin_out && zero_copy_allowed() ? pinned_device_ptr(keys) : nullptr;
  void *zo = zk ? pinned_device_ptr(out) : nullptr;
  if (zk && zo)
    return zero_copy_run(device, [&] {
      return launch(static_cast<const uint8_t *>(zk), n, static_cast<uint8_t *>(zo), nullptr);
    });
  auto plan = [&](size_t c, size_t *a, size_t *b) {
    if (c * per >= n) return false;
    *a = c * per;
    *b = std::min(n, *a + per);
    return true;
  };
  auto run = [&](Slot &s, size_t a, size_t b) -> int {
    const size_t cnt = b - a;
    if (int rc = slot_reserve(s, per * keylen, per * out_per_key)) return rc;
    if (int rc = chunk_in(s, static_cast<const uint8_t *>(keys) + a * keylen, pin_in, 0, cnt * keylen))
      return rc;
    if (int rc = launch(s.d_in, cnt, s.d_out, s.st)) return rc;
    return chunk_out(s, static_cast<uint8_t *>(out) + a * out_per_key, pin_out, 0, cnt * out_per_key);
  };
  return host_pipeline(device, plan, run);
}

}  // namespace pdht

using namespace pdht;

// ===================================================================== ABI ===
static_assert(PDHT_HIP_ABI_VERSION == 3, "bump the version string with the ABI");
PDHT_API const char *pdht_hip_version(void) { return "pdht-hip 0.3 (abi 3, gfx950, CityHash v1.0.x)"; }
PDHT_API const char *pdht_hip_last_error(void) { return g_err; }
PDHT_API const char *pdht_hip_last_kernel(void) { return g_kernel; }
#ifdef PDHT_HIP_TUNING
PDHT_API int pdht_hip_set_variant(int v) { return g_variant.exchange(v); }
PDHT_API int pdht_hip_set_blocks_per_cu(int per_cu) { return g_per_cu.exchange(per_cu); }
#endif

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

#define ST(s) reinterpret_cast<hipStream_t>(s)

PDHT_API int pdht_city64_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                   uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity64{}, Sink64{nullptr, out}, ST(s));
}
PDHT_API int pdht_city64_seeds_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                         uint64_t seed0, uint64_t seed1, uint64_t *out,
                                         pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity64Seeds{seed0, seed1}, Sink64{nullptr, out},
                      ST(s));
}
PDHT_API int pdht_city64_batch_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                       size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_var(bytes, nbytes, offsets, 0, n, AlgoCity64{}, Sink64{nullptr, out}, ST(s));
}
PDHT_API int pdht_city128_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                    uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity128{}, Sink128{nullptr, out}, ST(s));
}
PDHT_API int pdht_city128_seed_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                         uint64_t lo, uint64_t hi, uint64_t *out,
                                         pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_fixed(keys, stride, keylen, n, AlgoCity128Seed{lo, hi}, Sink128{nullptr, out}, ST(s));
}
PDHT_API int pdht_city128_batch_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                        size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  return launch_var(bytes, nbytes, offsets, 0, n, AlgoCity128{}, Sink128{nullptr, out}, ST(s));
}
PDHT_API int pdht_citycrc128_batch_dev(const void *keys, size_t stride, size_t keylen, size_t n,
                                       uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  if (keylen > 900) {  // CityHashCrc256 rounds: CRC-32C tables in LDS
#ifdef PDHT_HIP_TUNING
    if (tuning_variant() == 90)  // 5-bit slices, 13 lookups per word (r02 before the 6-bit tables)
      return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128, 5>{}, Sink128{nullptr, out}, ST(s));
#endif
    return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128>{}, Sink128{nullptr, out}, ST(s));
  }
  return launch_fixed(keys, stride, keylen, n, AlgoCrc128{}, Sink128{nullptr, out}, ST(s));
}
PDHT_API int pdht_citycrc128_seed_batch_dev(const void *keys, size_t stride, size_t keylen,
                                            size_t n, uint64_t lo, uint64_t hi, uint64_t *out,
                                            pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  if (keylen > 900)
    return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128Seed>{{lo, hi}}, Sink128{nullptr, out},
                        ST(s));
  return launch_fixed(keys, stride, keylen, n, AlgoCrc128Seed{lo, hi}, Sink128{nullptr, out}, ST(s));
}
PDHT_API int pdht_citycrc128_batch_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                           size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
  // any key may exceed 900 B (CityHashCrc256 rounds): CRC-32C tables in LDS
  return launch_var(bytes, nbytes, offsets, 0, n, CrcLds<AlgoCrc128>{}, Sink128{nullptr, out}, ST(s));
}

PDHT_API int pdht_place_batch_dev(const void *keys, size_t keysize, size_t n, uint32_t nptes,
                                  uint32_t nranks, uint64_t *mbits, uint32_t *ptindex, void *rank,
                                  size_t rank_stride, uint64_t *hist, pdht_hip_stream_t s) {
  if (int rc = check_place(n, mbits, nptes, nranks, rank, rank_stride)) return rc;
  return launch_fixed(keys, keysize, keysize, n, AlgoCity64{},
                      make_place_sink(mbits, ptindex, rank, rank_stride, hist, nptes, nranks), ST(s));
}

// -------------------------------------------------------- host batches ---
PDHT_API int pdht_city64_batch_host(const void *keys, size_t keylen, size_t n, uint64_t *out,
                                    int device) {
  return host_fixed(keys, keylen, n, 8, out, device,
                    [&](const uint8_t *dk, size_t cnt, uint8_t *dout, hipStream_t st) {
                      return launch_fixed(dk, keylen, keylen, cnt, AlgoCity64{},
                                          Sink64{nullptr, reinterpret_cast<u64 *>(dout)}, st);
                    });
}

PDHT_API int pdht_citycrc128_batch_host(const void *keys, size_t keylen, size_t n, uint64_t *out,
                                        int device) {
  return host_fixed(keys, keylen, n, 16, out, device,
                    [&](const uint8_t *dk, size_t cnt, uint8_t *dout, hipStream_t st) {
                      if (keylen > 900)
                        return launch_fixed(dk, keylen, keylen, cnt, CrcLds<AlgoCrc128>{},
                                            Sink128{nullptr, reinterpret_cast<u64 *>(dout)}, st);
                      return launch_fixed(dk, keylen, keylen, cnt, AlgoCrc128{},
                                          Sink128{nullptr, reinterpret_cast<u64 *>(dout)}, st);
                    });
}

PDHT_API int pdht_place_batch_host(const void *keys, size_t keysize, size_t n, uint32_t nptes,
                                   uint32_t nranks, uint64_t *mbits, uint32_t *ptindex, void *rank,
                                   size_t rank_stride, int device) {
  if (int rc = check_place(n, mbits, nptes, nranks, rank, rank_stride)) return rc;
  if (n == 0) return 0;
  if (!keys || keysize == 0) return fail("null keys or zero keysize%s", "");
  const size_t per = std::max<size_t>(1, kChunkBytes / keysize);
  const bool pin_in = is_pinned(keys);
  const bool pin_m = is_pinned(mbits);
  const bool pin_p = ptindex && is_pinned(ptindex);
  const bool pin_r = rank && is_pinned(rank);
  if (pin_in && pin_m && (!ptindex || pin_p) && (!rank || pin_r) && zero_copy_allowed()) {
    // zero-copy: the placement kernel reads and writes the pinned buffers
    void *zk = pinned_device_ptr(keys), *zm = pinned_device_ptr(mbits);
    void *zp = ptindex ? pinned_device_ptr(ptindex) : nullptr;
    void *zr = rank ? pinned_device_ptr(rank) : nullptr;
    if (zk && zm && (!ptindex || zp) && (!rank || zr))
      return zero_copy_run(device, [&] {
        return launch_fixed(zk, keysize, keysize, n, AlgoCity64{},
                            make_place_sink(static_cast<u64 *>(zm), static_cast<u32 *>(zp), zr, rank_stride,
                                            nullptr, nptes, nranks),
                            nullptr);
      });
  }
  // device output layout per chunk: [mbits u64 x per][ptindex u32 x per][rank u32 x per]
  const size_t o_pt = per * 8, o_rk = per * 12;
  auto plan = [&](size_t c, size_t *a, size_t *b) {
    if (c * per >= n) return false;
    *a = c * per;
    *b = std::min(n, *a + per);
    return true;
  };
  auto run = [&](Slot &s, size_t a, size_t b) -> int {
    const size_t cnt = b - a;
    if (int rc = slot_reserve(s, per * keysize, per * 16)) return rc;
    if (int rc = chunk_in(s, static_cast<const uint8_t *>(keys) + a * keysize, pin_in, 0, cnt * keysize))
      return rc;
    u64 *dm = reinterpret_cast<u64 *>(s.d_out);
    u32 *dp = ptindex ? reinterpret_cast<u32 *>(s.d_out + o_pt) : nullptr;
    u32 *dr = rank ? reinterpret_cast<u32 *>(s.d_out + o_rk) : nullptr;
    if (int rc = launch_fixed(s.d_in, keysize, keysize, cnt, AlgoCity64{},
                              make_place_sink(dm, dp, dr, 4, nullptr, nptes, nranks), s.st))
      return rc;
    if (int rc = chunk_out(s, mbits + a, pin_m, 0, cnt * 8)) return rc;
    if (ptindex)
      if (int rc = chunk_out(s, ptindex + a, pin_p, o_pt, cnt * 4)) return rc;
    if (rank) {
      if (rank_stride == 4) {
        if (int rc = chunk_out(s, static_cast<uint32_t *>(rank) + a, pin_r, o_rk, cnt * 4)) return rc;
      } else {
        // strided ptl_process_t destination: 2-D copy of the 4-byte members
        HIP_TRY(hipMemcpy2DAsync(static_cast<uint8_t *>(rank) + a * rank_stride, rank_stride,
                                 s.d_out + o_rk, 4, 4, cnt, hipMemcpyDeviceToHost, s.st));
      }
    }
    return 0;
  };
  return host_pipeline(device, plan, run);
}

PDHT_API int pdht_city64_batch_var_host(const void *bytes, const uint64_t *offsets, size_t n,
                                        uint64_t *out, int device) {
  if (n == 0) return 0;
  if (!bytes || !offsets || !out) return fail("null pointer%s", "");
  const bool pin_in = is_pinned(bytes), pin_out = is_pinned(out);
  if (pin_in && pin_out && is_pinned(offsets) && zero_copy_allowed()) {
    void *zb = pinned_device_ptr(bytes), *zf = pinned_device_ptr(offsets), *zo = pinned_device_ptr(out);
    if (zb && zf && zo)
      return zero_copy_run(device, [&] {
        return launch_var(zb, offsets[n] - offsets[0], static_cast<const u64 *>(zf), 0, n, AlgoCity64{},
                          Sink64{nullptr, static_cast<u64 *>(zo)}, nullptr);
      });
  }
  const size_t max_keys = kChunkBytes / 16;
  // chunk c covers keys [a, b) with at most kChunkBytes of key bytes (a key
  // longer than that gets a chunk of its own and a larger buffer)
  size_t next = 0;
  std::vector<std::pair<size_t, size_t>> chunks;
  while (next < n) {
    size_t a = next, b = a + 1;
    const u64 lim = offsets[a] + kChunkBytes;
    size_t hi = std::min(n, a + max_keys);
    // largest b <= hi with offsets[b] <= lim (binary search; offsets sorted)
    size_t lo_b = a + 1, hi_b = hi;
    while (lo_b < hi_b) {
      size_t mid = (lo_b + hi_b + 1) / 2;
      if (offsets[mid] <= lim) lo_b = mid; else hi_b = mid - 1;
    }
    b = std::max(a + 1, lo_b);
    chunks.push_back({a, b});
    next = b;
  }
  auto plan = [&](size_t c, size_t *a, size_t *b) {
    if (c >= chunks.size()) return false;
    *a = chunks[c].first;
    *b = chunks[c].second;
    return true;
  };
  auto run = [&](Slot &s, size_t a, size_t b) -> int {
    const size_t cnt = b - a;
    const size_t nbytes = offsets[b] - offsets[a];
    const size_t off_at = (nbytes + 255) & ~(size_t)255;  // offsets after the bytes
    if (int rc = slot_reserve(s, std::max(off_at + (max_keys + 1) * 8, off_at + (cnt + 1) * 8),
                              max_keys * 8))
      return rc;
    if (int rc = chunk_in(s, static_cast<const uint8_t *>(bytes) + offsets[a], pin_in, 0, nbytes)) return rc;
    // offsets are always staged (tiny) so that they can be copied as-is
    HIP_TRY(hipMemcpyAsync(s.d_in + off_at, offsets + a, (cnt + 1) * 8, hipMemcpyHostToDevice, s.st));
    if (int rc = launch_var(s.d_in, nbytes, reinterpret_cast<const u64 *>(s.d_in + off_at), offsets[a], cnt,
                            AlgoCity64{}, Sink64{nullptr, reinterpret_cast<u64 *>(s.d_out)}, s.st))
      return rc;
    return chunk_out(s, out + a, pin_out, 0, cnt * 8);
  };
  return host_pipeline(device, plan, run);
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

// Variable-length counterpart: the default offset-indexed kernel's data
// movement (window DMA, offsets, LDS reads of every key byte, digest stores)
// with an XOR fold for the hash.
PDHT_API int pdht_hip_key_stream_var_dev(const void *bytes, size_t nbytes, const uint64_t *offsets,
                                         size_t n, uint64_t *out, pdht_hip_stream_t s) {
  if (n && !out) return fail("null out%s", "");
#ifdef PDHT_HIP_TUNING
  // data-movement calibrations of the window kernel (no LDS reads, digest =
  // key length): 40 as shipped; 41 default-policy DMA; 42 plain stores;
  // 43 as 40 at 3 WG/CU; 44 offsets prefetched (k_window_var)
  const int v = tuning_variant();
  if (v >= 40 && v <= 45) {
    if (n == 0) return 0;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    const uint8_t *b = static_cast<const uint8_t *>(bytes);
    const u64 wb = ((n + 63) / 64 + 3) / 4;
    const Sink64T<true> snt{nullptr, out};
    const Sink64 spl{nullptr, out};
    hipStream_t st = ST(s);
    g_kernel = "k_window<var,calib>";
    if (v == 40)
      k_window<10224, true, AlgoLenOnly, Sink64T<true>, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets, 0, 0, 0, n, AlgoLenOnly{}, snt);
    else if (v == 41)
      k_window<10224, true, AlgoLenOnly, Sink64T<true>, 0><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets, 0, 0, 0, n, AlgoLenOnly{}, snt);
    else if (v == 42)
      k_window<10224, true, AlgoLenOnly, Sink64, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets, 0, 0, 0, n, AlgoLenOnly{}, spl);
    else if (v == 43)
      k_window<10224, true, AlgoLenOnly, Sink64T<true>, 2><<<grid_for(wb, 3, dev), kBlock, 0, st>>>(
          b, offsets, 0, 0, 0, n, AlgoLenOnly{}, snt);
    else if (v == 45)  // windows start on a 128-B line
      k_window<10224, true, AlgoLenOnly, Sink64T<true>, 2, 128><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets, 0, 0, 0, n, AlgoLenOnly{}, snt);
    else
      k_window_var<10224, AlgoLenOnly, Sink64T<true>, 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets, 0, n, AlgoLenOnly{}, snt);
    HIP_TRY(hipGetLastError());
    return 0;
  }
#endif
  return launch_var(bytes, nbytes, offsets, 0, n, AlgoFoldVar{}, Sink64{nullptr, out}, ST(s));
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

// ------------------------------------------------- destination bucketing ---
namespace pdht {
struct BucketWs {
  u32 *counts, *chunks;
  u64 *totals, *base, *fbase;
  u32 *tickets;  // [8] per-XCD tile tickets of the dynamic scatter
  // two-pass sort (8/16/32-B keys): fine-bucket counts per tile and per
  // 32-tile chunk, fine totals, rank counts per count-chunk, and the
  // intermediate ([n][keysize] key rows + [n] original indices)
  u32 *countsF, *chunksF, *chunkcnt;
  u64 *totalsF;
  uint8_t *ikeys;
  u32 *iidx;
  size_t bytes;
};
static size_t round256(size_t x) { return (x + 255) & ~(size_t)255; }
static bool two_pass_keysize(size_t keysize) { return keysize == 8 || keysize == 16 || keysize == 32; }
// Two-pass bucketing from this many ranks up (interleaved
// A/B on 16M keys; at 1024 ranks one pass is 10 % faster for 8-B keys, equal
// for 16-B keys, 30 % faster for 32-B keys; at 2048 ranks two passes are 1.3x
// faster for 8-B keys and at 8192 ranks 2.1x).
static u32 two_pass_min_ranks(size_t keysize) { return keysize == 8 ? 1536 : keysize == 16 ? 1025 : 2049; }
// Sized for the smallest tile any scatter kernel uses, plus the two-pass
// intermediate when the batch can take that path: 8/16/32-B keys from
// two_pass_min_ranks() up (the tuning build forces two passes at any nranks
// and always reserves it).  16M x 8-B keys at 1024 ranks: 17 MB; from 1536
// ranks + 192 MB.
static BucketWs bucket_layout(void *ws, size_t n, size_t keysize, u32 nranks) {
  const u64 ntiles = (n + kBucketMinTile - 1) / kBucketMinTile;
  const u64 nchunks = (ntiles + kBucketChunk - 1) / kBucketChunk;
  BucketWs w{};
  uint8_t *p = static_cast<uint8_t *>(ws);
  size_t off = 0;
  w.counts = reinterpret_cast<u32 *>(p + off);
  off += round256((size_t)nranks * ntiles * 4);
  w.chunks = reinterpret_cast<u32 *>(p + off);
  off += round256((size_t)nranks * nchunks * 4);
  w.totals = reinterpret_cast<u64 *>(p + off);
  off += round256((size_t)nranks * 8);
  w.base = reinterpret_cast<u64 *>(p + off);
  off += round256((size_t)nranks * 8);
  w.fbase = reinterpret_cast<u64 *>(p + off);
  off += round256((size_t)kTpMaxDigits * 8);
  w.tickets = reinterpret_cast<u32 *>(p + off);
  off += 256;
#ifdef PDHT_HIP_TUNING
  const bool two_pass = two_pass_keysize(keysize);
#else
  const bool two_pass = two_pass_keysize(keysize) && nranks >= two_pass_min_ranks(keysize);
#endif
  if (two_pass) {
    const u64 tp_tiles = (n + kTpCountTile - 1) / kTpCountTile;
    const u64 tp_chunks32 = (tp_tiles + kBucketChunk - 1) / kBucketChunk;
    const u64 tp_chunks = (tp_tiles + kTpChunkTiles - 1) / kTpChunkTiles;
    w.countsF = reinterpret_cast<u32 *>(p + off);
    off += round256((size_t)tp_tiles * kTpMaxDigits * 4);
    w.chunksF = reinterpret_cast<u32 *>(p + off);
    off += round256((size_t)tp_chunks32 * kTpMaxDigits * 4);
    w.totalsF = reinterpret_cast<u64 *>(p + off);
    off += round256((size_t)kTpMaxDigits * 8);
    w.chunkcnt = reinterpret_cast<u32 *>(p + off);
    off += round256((size_t)tp_chunks * nranks * 4);
    w.ikeys = p + off;
    off += round256(n * keysize);
    w.iidx = reinterpret_cast<u32 *>(p + off);
    off += round256(n * 4);
  }
  w.bytes = off;
  return w;
}

static int set_lds(const void *fn, size_t bytes) {
  if (bytes > 65536)
    HIP_TRY(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
  return 0;
}

struct BucketArgs {
  const uint8_t *k;
  u64 n;
  FastMod rk;
  u32 nranks, nbits;
  TileStarts ts;
  u64 ntiles;
};

template <int L, class Out, bool PACK = false, int W = kStW, int KPL = kStKPL, bool DYN = false, int OB = 0>
static int launch_staged(const BucketArgs &a, const Out &out, hipStream_t st, int dev, u32 *tickets = nullptr) {
  static const char *const names[3] = {"k_bucket_scatter_staged<8B>", "k_bucket_scatter_staged<16B>",
                                       "k_bucket_scatter_staged<32B>"};
  static const char *const pnames[3] = {"k_bucket_scatter_staged<8B,u16>", "k_bucket_scatter_staged<16B,u16>",
                                        "k_bucket_scatter_staged<32B,u16>"};
  static const char *const onames[3] = {"k_bucket_scatter_staged<8B,own>", "k_bucket_scatter_staged<16B,own>",
                                        "k_bucket_scatter_staged<32B,own>"};
  static const char *const o8names[3] = {"k_bucket_scatter_staged<8B,own,8x16>",
                                         "k_bucket_scatter_staged<16B,own,8x16>",
                                         "k_bucket_scatter_staged<32B,own,8x16>"};
  g_kernel = (OB ? (W == 8 ? o8names : onames) : PACK ? pnames : names)[L == 8 ? 0 : L == 16 ? 1 : 2];
  const size_t bytes = staged_lds_bytes(a.nranks, W, KPL, PACK, OB);
  auto fn = &k_bucket_scatter_staged<L, Out, W, KPL, PACK, DYN, OB>;
  if (int rc = set_lds(reinterpret_cast<const void *>(fn), bytes)) return rc;
  const int per_cu = bytes <= 53 * 1024 ? 3 : bytes <= 80 * 1024 ? 2 : 1;
  unsigned g = (unsigned)std::min<u64>(a.ntiles, (u64)std::max(1, g_dev[dev].cus) * per_cu);
  if (g >= 8) g &= ~7u;  // a multiple of 8: XCD-contiguous tile order (TileOrder)
  // (DYN: 8 XCD groups need a grid that is a multiple of 8; small grids use
  // the static order)
  if (DYN && g % 8 == 0)
    fn<<<g, W * 64, bytes, st>>>(a.k, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out, tickets);
  else
    k_bucket_scatter_staged<L, Out, W, KPL, PACK, false, OB>
        <<<g, W * 64, bytes, st>>>(a.k, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out, nullptr);
  return 0;
}

#ifdef PDHT_HIP_TUNING
template <int W, int L, int KPL, class Out>
static int launch_reg(const BucketArgs &a, const Out &out, hipStream_t st, int dev) {
  static const char *const names[3] = {"k_bucket_scatter_reg<8B>", "k_bucket_scatter_reg<16B>",
                                       "k_bucket_scatter_reg<32B>"};
  g_kernel = names[L == 8 ? 0 : L == 16 ? 1 : 2];
  const size_t bytes = (size_t)W * a.nranks * 4;
  if (int rc = set_lds(reinterpret_cast<const void *>(&k_bucket_scatter_reg<W, L, KPL, Out>), bytes)) return rc;
  k_bucket_scatter_reg<W, L, KPL, Out><<<grid_for(a.ntiles, 2, dev), W * 64, bytes, st>>>(
      a.k, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out);
  return 0;
}

#endif

template <int W, class Out>
static int launch_wg(const BucketArgs &a, const Out &out, u32 L, hipStream_t st, int dev) {
  g_kernel = W == 8 ? "k_bucket_scatter_wg<8>" : "k_bucket_scatter_wg<4>";
  const size_t bytes = (size_t)W * a.nranks * 4;
  if (int rc = set_lds(reinterpret_cast<const void *>(&k_bucket_scatter_wg<W, Out>), bytes)) return rc;
  k_bucket_scatter_wg<W, Out><<<grid_for(a.ntiles, 4, dev), W * 64, bytes, st>>>(
      a.k, L, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out);
  return 0;
}

#ifdef PDHT_HIP_TUNING
template <int W, int KPL, class Out>
static int launch_gather(const BucketArgs &a, const Out &out, u32 L, int lk, hipStream_t st, int dev) {
  const size_t bytes = gather_lds_bytes(a.nranks, W, KPL);
  const int per_cu = bytes <= 80 * 1024 ? 2 : 1;
  auto go = [&](auto fn, const char *name) -> int {
    g_kernel = name;
    if (int rc = set_lds(reinterpret_cast<const void *>(fn), bytes)) return rc;
    unsigned g = (unsigned)std::min<u64>(a.ntiles, (u64)std::max(1, g_dev[dev].cus) * per_cu);
    if (g >= 8) g &= ~7u;  // a multiple of 8: XCD-contiguous tile order (TileOrder)
    fn<<<g, W * 64, bytes, st>>>(a.k, L, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out);
    return 0;
  };
  if (lk == 8) return go(&k_bucket_scatter_gather<8, Out, W, KPL>, "k_bucket_scatter_gather<8B>");
  if (lk == 16) return go(&k_bucket_scatter_gather<16, Out, W, KPL>, "k_bucket_scatter_gather<16B>");
  if (lk == 32) return go(&k_bucket_scatter_gather<32, Out, W, KPL>, "k_bucket_scatter_gather<32B>");
  return go(&k_bucket_scatter_gather<0, Out, W, KPL>, "k_bucket_scatter_gather<any>");
}
#endif


template <int L, class Out, int W = kTpW, int KPL = kTpKPL, int PER_CU = kTpPerCu, int DBG = 0, bool DYN = false>
static int launch_two_pass(const BucketArgs &a, const TwoPass &tp, const Out &out, hipStream_t st, int dev,
                           u32 *tickets) {
  static const char *const names[3] = {"k_bucket_pass2<8B>", "k_bucket_pass2<16B>", "k_bucket_pass2<32B>"};
  constexpr int WPE = PER_CU * W / 4 > 8 ? 8 : PER_CU * W / 4;  // waves per SIMD
  const size_t b1 = pass1_lds_bytes<W, KPL>(), b2 = pass2_lds_bytes<W, KPL>();
  auto f1 = &k_bucket_pass1<L, W, KPL, WPE, DBG, DYN>;
  auto f2 = &k_bucket_pass2<L, Out, W, KPL, WPE, DBG, DYN>;
  auto f1s = &k_bucket_pass1<L, W, KPL, WPE, DBG, false>;
  auto f2s = &k_bucket_pass2<L, Out, W, KPL, WPE, DBG, false>;
  if (int rc = set_lds(reinterpret_cast<const void *>(f1), b1)) return rc;
  if (int rc = set_lds(reinterpret_cast<const void *>(f2), b2)) return rc;
  if (int rc = set_lds(reinterpret_cast<const void *>(f1s), b1)) return rc;
  if (int rc = set_lds(reinterpret_cast<const void *>(f2s), b2)) return rc;
  const u64 cus = (u64)std::max(1, g_dev[dev].cus);
  unsigned g1 = (unsigned)std::min<u64>(a.ntiles, cus * PER_CU);
  if (g1 >= 8) g1 &= ~7u;  // XCD-contiguous tile order (TileOrder)
  // (tickets need a grid that is a multiple of 8; small grids: static order)
  if (DYN && g1 % 8 == 0)
    f1<<<g1, W * 64, b1, st>>>(a.k, a.n, a.rk, tp, tickets);
  else
    f1s<<<g1, W * 64, b1, st>>>(a.k, a.n, a.rk, tp, nullptr);
  unsigned g2 = (unsigned)std::min<u64>(tp.nseg, cus * PER_CU);
  if (g2 >= 8) g2 &= ~7u;
  if (DYN && g2 % 8 == 0)
    f2<<<g2, W * 64, b2, st>>>(a.rk, a.nranks, tp, out, tickets + 8);
  else
    f2s<<<g2, W * 64, b2, st>>>(a.rk, a.nranks, tp, out, nullptr);
  g_kernel = names[L == 8 ? 0 : L == 16 ? 1 : 2];
  return 0;
}

template <int L, class Out>
static int launch_two_pass_sel(const BucketArgs &a, const TwoPass &tp, const Out &out, hipStream_t st, int dev,
                               u32 *tickets) {
#ifdef PDHT_HIP_TUNING
  // 73-76: sub-tile shape (waves x keys per lane) and workgroups per CU;
  // 77: 73 with contiguous stores (timing-only, wrong results); 86: per-XCD
  // tile tickets
  switch (tuning_variant()) {
    case 73: return launch_two_pass<L, Out, 4, 8, 4>(a, tp, out, st, dev, tickets);
    case 74: return launch_two_pass<L, Out, 8, 4, 4>(a, tp, out, st, dev, tickets);
    case 75: return launch_two_pass<L, Out, 4, 16, 2>(a, tp, out, st, dev, tickets);
    case 76: return launch_two_pass<L, Out, 4, 4, 6>(a, tp, out, st, dev, tickets);
    case 77: return launch_two_pass<L, Out, 4, 8, 4, 1>(a, tp, out, st, dev, tickets);  // timing-only
    case 86: return launch_two_pass<L, Out, kTpW, kTpKPL, kTpPerCu, 0, true>(a, tp, out, st, dev, tickets);
    default: break;
  }
#endif
  return launch_two_pass<L, Out>(a, tp, out, st, dev, tickets);
}

enum class BucketKernel { kGather, kStaged, kReg, kGeneric, kTwoPass };

enum class StagedShape { kBallot4x16, kOwner4x16, kOwner8x16, kOwner4x24 };
template <class Out>
static StagedShape staged_shape(size_t keysize, u32 nranks) {
  if (nranks < 512) return StagedShape::kBallot4x16;
  if (!std::is_same<Out, OutSoA>::value) {
    // records: owner ranking pays for 16/32-B keys only (ab_records_*_shapes.log:
    // 16-B at 1024 ranks 0.62 -> 0.56 ms, 32-B 1.29 -> 1.20); 8-B records
    // lose 3 % with it
    if (keysize != 8 && staged_lds_bytes(nranks, kStW, kStKPL, false, 2) <= 80 * 1024)
      return StagedShape::kOwner4x16;
    return StagedShape::kBallot4x16;
  }
  if (keysize != 32 && staged_lds_bytes(nranks, 8, 16, false, 2) <= 160 * 1024) return StagedShape::kOwner8x16;
  if (staged_lds_bytes(nranks, kStW, kStKPL, false, 2) <= 80 * 1024) return StagedShape::kOwner4x16;
  return StagedShape::kBallot4x16;
}

// Shared by pdht_bucket_batch_dev (OutSoA) and pdht_bucket_records_dev
// (OutRec): counting pass, scans, bucket bases, then the scatter into `out`.
// out_al: alignment bits of the output key rows (0 when they are 8-B aligned
// 8-B pieces, as in records).
template <class Out>
static int bucket_impl(const void *keys, size_t keysize, size_t n, uint32_t nranks, void *workspace,
                       size_t workspace_bytes, const Out &out, uintptr_t out_al, uint64_t *bucket_offsets,
                       hipStream_t st) {
  if (nranks == 0) return fail("nranks must be > 0%s", "");
  if (nranks > kBucketMaxRanks) return fail("bucketing supports up to 8192 ranks%s", "");
  if (n >= (1ull << 32)) return fail("bucketing: n must be < 2^32 per call%s", "");
  if (!bucket_offsets) return fail("bucket_offsets must not be NULL%s", "");
  if (n && (!keys || keysize == 0)) return fail("null keys or zero keysize%s", "");
  const BucketWs w = bucket_layout(workspace, n, keysize, nranks);
  if (!workspace || workspace_bytes < w.bytes) return fail("workspace too small%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  // Kernel choice: packed 8/16/32-B keys (aligned) -> LDS-staged scatter up to
  // 2048 ranks, register scatter above; other lengths -> generic.
  const uintptr_t al = (uintptr_t)keys | out_al;
  const bool fixed = (keysize == 8 && (al & 7) == 0) || ((keysize == 16 || keysize == 32) && (al & 15) == 0);
  // (two_pass_min_ranks <= kStagedMaxRanks + 1: the staged scatter covers
  // every nranks below the two-pass threshold)
  BucketKernel kind = !fixed                                ? BucketKernel::kGeneric
                      : nranks >= two_pass_min_ranks(keysize) ? BucketKernel::kTwoPass
                                                              : BucketKernel::kStaged;
  int ga_w = kGaW, ga_kpl = kGaKPL;
#ifdef PDHT_HIP_TUNING
  // 21 generic, 22 register scatter; 54 the gather scatter (16384-key tiles,
  // keys gathered back from L2 and re-hashed), 52 / 53 it with 8192-key
  // tiles (4 waves x 32 / 8 waves x 16 keys per lane); 55-57 its timing-only
  // builds; 58 producer/consumer scatter; 50 staged with u16 run tables.
  // All measured slower than the staged scatter.
  // 70: one pass (staged / register scatter) at any nranks; 71: two passes
  // at any nranks >= 2.
  if (tuning_variant() == 70 && kind == BucketKernel::kTwoPass)
    kind = nranks > kStagedMaxRanks ? BucketKernel::kReg : BucketKernel::kStaged;
  if (tuning_variant() == 71 && fixed && nranks >= 2) kind = BucketKernel::kTwoPass;
  if (tuning_variant() == 21) kind = BucketKernel::kGeneric;
  if (tuning_variant() == 22 && fixed) kind = BucketKernel::kReg;
  if (tuning_variant() >= 52 && tuning_variant() <= 58 && nranks <= kStagedMaxRanks) kind = BucketKernel::kGather;
  if (tuning_variant() == 52) ga_w = 4;
  if (tuning_variant() == 53) ga_kpl = 16;
#endif
  // Staged scatter shape (tools/abbench.py): owner-table
  // ranking for array outputs from 512 ranks; with it, 8 waves x 16 keys per
  // lane (8192-key tiles, 1 WG/CU) for 8/16-B keys while the LDS holds
  // (8-B keys at 1024 ranks 0.274 -> 0.261 ms, 16-B 0.443 -> 0.405; 32-B
  // keys lose 11 % and keep 4 x 16); else 4 x 16 while two workgroups fit a
  // CU (<= 1462 ranks); ballots below 512 ranks and for records.
  StagedShape shape = staged_shape<Out>(keysize, nranks);
#ifdef PDHT_HIP_TUNING
  if (tuning_variant() == 83) shape = StagedShape::kOwner8x16;
  if (tuning_variant() == 87) shape = StagedShape::kOwner4x16;
  if (tuning_variant() == 84 && keysize == 8) shape = StagedShape::kOwner4x24;
  if (tuning_variant() == 85 || tuning_variant() == 89) shape = StagedShape::kBallot4x16;
#endif
  const u64 st_tile = shape == StagedShape::kOwner8x16 ? 8192 : shape == StagedShape::kOwner4x24 ? 6144 : kStTile;
  const int waves = nranks <= 4096 ? 8 : 4;  // reg / generic: W x nranks x 4 B of LDS <= 128 KiB
  const int reg_kpl = keysize == 32 ? 8 : 16;
  const u64 tile = kind == BucketKernel::kGather     ? (u64)ga_w * ga_kpl * 64
                   : kind == BucketKernel::kTwoPass ? kTpCountTile
                   : kind == BucketKernel::kStaged   ? st_tile
                   : kind == BucketKernel::kReg    ? (u64)waves * reg_kpl * 64
                                                   : (u64)waves * kScatKPL * 64;
  const u64 ntiles = (n + tile - 1) / tile;
  const u64 nchunks = (ntiles + kBucketChunk - 1) / kBucketChunk;
  BucketArgs a{};
  a.k = static_cast<const uint8_t *>(keys);
  a.n = n;
  a.rk = make_fastmod(nranks);
  a.nranks = nranks;
  while ((1u << a.nbits) < nranks) ++a.nbits;
  a.ts = TileStarts{w.counts, w.chunks, w.base, nranks};
  a.ntiles = ntiles;
  const size_t hist_lds = (size_t)nranks * 4;
  TwoPass tp{};
  if (kind == BucketKernel::kTwoPass) {
    tp.fbits = (a.nbits + 1) / 2;
    tp.F = 1u << tp.fbits;
    tp.C = (nranks + tp.F - 1) >> tp.fbits;
    tp.cbits = a.nbits - tp.fbits;
    tp.countsF = w.countsF;
    tp.chunksF = w.chunksF;
    tp.totalsF = w.totalsF;
    tp.chunkcnt = w.chunkcnt;
    tp.base = w.base;
    tp.fbase = w.fbase;
    tp.ikeys = w.ikeys;
    tp.iidx = w.iidx;
    tp.ntiles = ntiles;
    tp.nchunks = (ntiles + kTpChunkTiles - 1) / kTpChunkTiles;
    tp.SG = std::max<u64>(1, tp.F / kTpChunkTiles);  // ~4096 keys per segment
    tp.nsegf = (tp.nchunks + tp.SG - 1) / tp.SG;
    tp.nseg = (u64)tp.F * tp.nsegf;
  }
  if (ntiles && kind == BucketKernel::kTwoPass) {
    const u64 nchunks32 = (ntiles + kBucketChunk - 1) / kBucketChunk;
    const unsigned gc = (unsigned)std::min<u64>(tp.nchunks, (u64)std::max(1, g_dev[dev].cus) * 8);
    if (keysize == 8)
      k_bucket_count_tp<8><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, tp.F, w.countsF, w.chunkcnt,
                                                          ntiles);
    else if (keysize == 16)
      k_bucket_count_tp<16><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, tp.F, w.countsF, w.chunkcnt,
                                                           ntiles);
    else
      k_bucket_count_tp<32><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, tp.F, w.countsF, w.chunkcnt,
                                                           ntiles);
    k_bucket_colscan<<<dim3((tp.F + 63) / 64, (unsigned)nchunks32), 64, 0, st>>>(w.countsF, ntiles, tp.F,
                                                                                   w.chunksF);
    k_bucket_chunkscan<<<(tp.F + 63) / 64, 64 * kCsWaves, 0, st>>>(w.chunksF, nchunks32, tp.F, w.totalsF);
    k_bucket_chunkscan<<<(nranks + 63) / 64, 64 * kCsWaves, 0, st>>>(w.chunkcnt, tp.nchunks, nranks,
                                                                        w.totals);
  } else if (ntiles) {
    const unsigned gc = grid_for(ntiles, 8, dev);
    if (fixed && keysize == 8)
      k_bucket_count_reg<8><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, w.counts, ntiles, tile);
    else if (fixed && keysize == 16)
      k_bucket_count_reg<16><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, w.counts, ntiles, tile);
    else if (fixed && keysize == 32)
      k_bucket_count_reg<32><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, w.counts, ntiles, tile);
    else
      k_bucket_count<<<gc, kBlock, hist_lds, st>>>(a.k, (u32)keysize, n, a.rk, nranks, w.counts, ntiles,
                                                   tile);
    k_bucket_colscan<<<dim3((nranks + 63) / 64, (unsigned)nchunks), 64, 0, st>>>(w.counts, ntiles, nranks,
                                                                                 w.chunks);
    k_bucket_chunkscan<<<(nranks + 63) / 64, 64 * kCsWaves, 0, st>>>(w.chunks, nchunks, nranks,
                                                                        w.totals);
  } else {
    HIP_TRY(hipMemsetAsync(w.totals, 0, (size_t)nranks * 8, st));
  }
  k_bucket_base<<<1, kBaseThreads, 0, st>>>(w.totals, nranks, w.base, bucket_offsets, tp.fbits, w.totalsF,
                                            kind == BucketKernel::kTwoPass ? w.fbase : nullptr, w.tickets);
  g_kernel = "k_bucket_base";
  if (ntiles) {
    int rc = 0;
#ifdef PDHT_HIP_TUNING
    const int lk = fixed ? (int)keysize : 0;
    if (kind == BucketKernel::kGather && !(tuning_variant() >= 55 && tuning_variant() <= 58 && lk == 8)) {
      if (ga_w == 8 && ga_kpl == 32)
        rc = launch_gather<8, 32>(a, out, (u32)keysize, lk, st, dev);
      else if (ga_w == 4)
        rc = launch_gather<4, 32>(a, out, (u32)keysize, lk, st, dev);
      else
        rc = launch_gather<8, 16>(a, out, (u32)keysize, lk, st, dev);
    } else if (kind == BucketKernel::kGather && lk == 8 && tuning_variant() == 58) {
      // producer/consumer scatter: 8 + 8 waves, 16384-key tiles, 1 WG/CU
      const size_t bytes = (size_t)8 * a.nranks * 4 + (size_t)2 * a.nranks * 4 + (size_t)2 * 16384 * 2;
      auto fn = &k_bucket_scatter_pc<Out, 8, 32>;
      g_kernel = "k_bucket_scatter_pc<8B>";
      if (int e = set_lds(reinterpret_cast<const void *>(fn), bytes)) return e;
      unsigned g = (unsigned)std::min<u64>(a.ntiles, (u64)std::max(1, g_dev[dev].cus));
      if (g >= 8) g &= ~7u;
      fn<<<g, 1024, bytes, st>>>(a.k, (u32)keysize, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out);
    } else if (kind == BucketKernel::kGather && ga_w == 8 && ga_kpl == 32 && lk == 8 &&
               tuning_variant() >= 55 && tuning_variant() <= 57) {
      // timing-only builds (wrong results): 55 no stores, 56 no gather, 57 no phase D
      const size_t bytes = gather_lds_bytes(a.nranks, 8, 32);
      const int v = tuning_variant();
      auto fn = v == 55 ? &k_bucket_scatter_gather<8, Out, 8, 32, 32, 1>
                : v == 56 ? &k_bucket_scatter_gather<8, Out, 8, 32, 32, 2>
                          : &k_bucket_scatter_gather<8, Out, 8, 32, 32, 4>;
      g_kernel = "k_bucket_scatter_gather<8B,timing-only>";
      if (int e = set_lds(reinterpret_cast<const void *>(fn), bytes)) return e;
      unsigned g = (unsigned)std::min<u64>(a.ntiles, (u64)std::max(1, g_dev[dev].cus) * 2) & ~7u;
      fn<<<g, 512, bytes, st>>>(a.k, (u32)keysize, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out);
    } else if (kind == BucketKernel::kStaged && tuning_variant() == 85)  // static tile order (r02 default before)
      rc = keysize == 8    ? launch_staged<8, Out>(a, out, st, dev)
           : keysize == 16 ? launch_staged<16, Out>(a, out, st, dev)
                           : launch_staged<32, Out>(a, out, st, dev);
    else if (kind == BucketKernel::kStaged && tuning_variant() == 50)  // u16 run tables, 3 WG/CU
      rc = keysize == 8    ? launch_staged<8, Out, true>(a, out, st, dev)
           : keysize == 16 ? launch_staged<16, Out, true>(a, out, st, dev)
                           : launch_staged<32, Out, true>(a, out, st, dev);
    else
#endif
    if (kind == BucketKernel::kTwoPass)
      rc = keysize == 8    ? launch_two_pass_sel<8, Out>(a, tp, out, st, dev, w.tickets)
           : keysize == 16 ? launch_two_pass_sel<16, Out>(a, tp, out, st, dev, w.tickets)
                           : launch_two_pass_sel<32, Out>(a, tp, out, st, dev, w.tickets);
    else if (kind == BucketKernel::kStaged && shape == StagedShape::kOwner8x16)
      rc = keysize == 8    ? launch_staged<8, Out, false, 8, 16, true, 2>(a, out, st, dev, w.tickets)
           : keysize == 16 ? launch_staged<16, Out, false, 8, 16, true, 2>(a, out, st, dev, w.tickets)
                           : launch_staged<32, Out, false, 8, 16, true, 2>(a, out, st, dev, w.tickets);
    else if (kind == BucketKernel::kStaged && shape == StagedShape::kOwner4x16)
      rc = keysize == 8    ? launch_staged<8, Out, false, kStW, kStKPL, true, 2>(a, out, st, dev, w.tickets)
           : keysize == 16 ? launch_staged<16, Out, false, kStW, kStKPL, true, 2>(a, out, st, dev, w.tickets)
                           : launch_staged<32, Out, false, kStW, kStKPL, true, 2>(a, out, st, dev, w.tickets);
#ifdef PDHT_HIP_TUNING
    else if (kind == BucketKernel::kStaged && shape == StagedShape::kOwner4x24)  // slower (spills)
      rc = launch_staged<8, Out, false, 4, 24, true, 2>(a, out, st, dev, w.tickets);
#endif
    else if (kind == BucketKernel::kStaged)  // per-XCD tile tickets
      rc = keysize == 8    ? launch_staged<8, Out, false, kStW, kStKPL, true>(a, out, st, dev, w.tickets)
           : keysize == 16 ? launch_staged<16, Out, false, kStW, kStKPL, true>(a, out, st, dev, w.tickets)
                           : launch_staged<32, Out, false, kStW, kStKPL, true>(a, out, st, dev, w.tickets);
#ifdef PDHT_HIP_TUNING
    else if (kind == BucketKernel::kReg)
      rc = keysize == 8 ? (waves == 8 ? launch_reg<8, 8, 16>(a, out, st, dev) : launch_reg<4, 8, 16>(a, out, st, dev))
           : keysize == 16
               ? (waves == 8 ? launch_reg<8, 16, 16>(a, out, st, dev) : launch_reg<4, 16, 16>(a, out, st, dev))
               : (waves == 8 ? launch_reg<8, 32, 8>(a, out, st, dev) : launch_reg<4, 32, 8>(a, out, st, dev));
#endif
    else
      rc = waves == 8 ? launch_wg<8>(a, out, (u32)keysize, st, dev) : launch_wg<4>(a, out, (u32)keysize, st, dev);
    if (rc) return rc;
  }
  HIP_TRY(hipGetLastError());
  return 0;
}
}  // namespace pdht

PDHT_API size_t pdht_bucket_workspace_bytes(size_t n, size_t keysize, uint32_t nranks) {
  return bucket_layout(nullptr, n, keysize, nranks).bytes;
}

PDHT_API int pdht_bucket_batch_dev(const void *keys, size_t keysize, size_t n, uint32_t nptes,
                                   uint32_t nranks, void *workspace, size_t workspace_bytes,
                                   void *keys_out, uint64_t *mbits_out, uint32_t *ptindex_out,
                                   uint32_t *index_out, uint64_t *bucket_offsets,
                                   pdht_hip_stream_t s) {
  if (int rc = check_place(n, mbits_out, nptes, nranks, nullptr, 0)) return rc;
  const OutSoA out{static_cast<uint8_t *>(keys_out), mbits_out, ptindex_out, index_out, make_fastmod(nptes),
                   (u32)keysize};
  return bucket_impl(keys, keysize, n, nranks, workspace, workspace_bytes, out, (uintptr_t)keys_out,
                     bucket_offsets, ST(s));
}

PDHT_API size_t pdht_bucket_record_bytes(size_t keysize) { return 24 + ((keysize + 7) & ~(size_t)7); }

PDHT_API int pdht_bucket_records_dev(const void *keys, size_t keysize, size_t n, uint32_t nranks,
                                     uint32_t msg_type, uint32_t src_rank, uint32_t ht_index,
                                     void *workspace, size_t workspace_bytes, void *records,
                                     uint64_t *bucket_offsets, pdht_hip_stream_t s) {
  if (n && !records) return fail("records must not be NULL%s", "");
  if ((uintptr_t)records & 7) return fail("records must be 8-byte aligned%s", "");
  const OutRec out{static_cast<uint8_t *>(records), (u64)pdht_bucket_record_bytes(keysize),
                   (u64)msg_type | ((u64)src_rank << 32), ht_index, (u32)keysize};
  return bucket_impl(keys, keysize, n, nranks, workspace, workspace_bytes, out, 0, bucket_offsets, ST(s));
}
