// pdht_host.hip -- host-resident batches (include/pdht_hip.h): zero-copy
// kernels on pinned buffers, a chunked copy pipeline for pageable ones.
#include "launch.h"

namespace pdht {

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
// pinned buffers take the zero-copy path (the A/B build can force the chunked
// copy pipeline onto them instead)
static bool zero_copy_allowed() { return hook_zero_copy(true); }

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
