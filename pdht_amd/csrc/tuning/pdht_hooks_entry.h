// tuning/pdht_hooks_entry.h -- the TUNING build's alternatives behind the
// C-ABI entry points of pdht_var.hip and pdht_fixed128.hip (calibrations
// with part of the work removed -- wrong digests -- and r02's CRC tables);
// product/pdht_hooks_entry.h takes none of them.
#pragma once

namespace pdht {

// pdht_city64_batch_var_dev
static int hook_var_city64(const void *bytes, const uint64_t *offsets, size_t n, uint64_t *out,
                           pdht_hip_stream_t s) {
  // r03 write-destination calibration of the product window kernel: 140-144
  // nt digest stores wrapped into 32 KiB / 2 / 8 / 32 / 128 MiB of out
  // (wrong digests: what the HBM writes cost)
  const int v = tuning_variant();
  if (v >= 140 && v <= 144 && n) {
    int dev;
    if (int rc = current_device(&dev)) return rc;
    const uint8_t *b = static_cast<const uint8_t *>(bytes);
    hipStream_t st = ST(s);
    auto win = [&](u64 k0, u64 c, auto sink) {
      const u64 wb = ((c + 63) / 64 + 3) / 4;
      k_window<10224, true, AlgoCity64, decltype(sink), 2><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets + k0, 0, 0, 0, c, AlgoCity64{}, sink);
    };
    g_kernel = "k_window<var,nt,10224>@4";
    if (v == 140) win(0, n, SinkRing<12>{nullptr, out});
    if (v == 141) win(0, n, SinkRing<18>{nullptr, out});
    if (v == 142) win(0, n, SinkRing<20>{nullptr, out});
    if (v == 143) win(0, n, SinkRing<22>{nullptr, out});
    if (v == 144) win(0, n, SinkRing<24>{nullptr, out});
    HIP_TRY(hipGetLastError());
    return 0;
  }
  return kNoVariant;
}

// pdht_hip_key_stream_var_dev
static int hook_key_stream_var(const void *bytes, size_t nbytes, const uint64_t *offsets, size_t n,
                               uint64_t *out, pdht_hip_stream_t s) {
  // data-movement calibrations of the window kernel (no LDS reads, digest =
  // key length): 40 as shipped; 41 default-policy DMA; 42 plain stores;
  // 43 as 40 at 3 WG/CU; 45 windows on 128-B lines
  const int v = tuning_variant();
  if ((v >= 119 && v <= 121) || v == 125) {
    // the window kernel's loads without the offsets: keys read as FIXED-length
    // rows of the batch's mean length (cfg3c-like data: 136 B), 119 with nt
    // digest stores, 120 with none, 121 plain stores, 125 plain stores into
    // 32 KiB (L2-resident: the store instructions without the HBM writes)
    if (n == 0) return 0;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    const uint8_t *b = static_cast<const uint8_t *>(bytes);
    const u64 L = nbytes / n;
    const u64 wb = ((n + 63) / 64 + 3) / 4;
    g_kernel = "k_window<var,calib>";
    if (v == 119)
      k_window<10224, false, AlgoLenOnly, Sink64T<true>, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, nullptr, 0, L, L, n, AlgoLenOnly{}, Sink64T<true>{nullptr, out});
    else if (v == 121)  // plain digest stores
      k_window<10224, false, AlgoLenOnly, Sink64, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, nullptr, 0, L, L, n, AlgoLenOnly{}, Sink64{nullptr, out});
    else if (v == 125)
      k_window<10224, false, AlgoLenOnly, SinkSmall, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, nullptr, 0, L, L, n, AlgoLenOnly{}, SinkSmall{nullptr, out});
    else
      k_window<10224, false, AlgoLenOnly, SinkNone, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, nullptr, 0, L, L, n, AlgoLenOnly{}, SinkNone{nullptr, out});
    HIP_TRY(hipGetLastError());
    return 0;
  }
  if (v == 110 || v == 111) {
    // the product window kernel with CityHash64 twice per key (110) / once
    // (111): what the hash arithmetic costs over the data movement (40)
    if (n == 0) return 0;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    const uint8_t *b = static_cast<const uint8_t *>(bytes);
    const u64 wb = ((n + 63) / 64 + 3) / 4;
    const Sink64T<true> snt{nullptr, out};
    g_kernel = "k_window<var,calib>";
    if (v == 110)
      k_window<10224, true, AlgoCity64x2, Sink64T<true>, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, offsets, 0, 0, 0, n, AlgoCity64x2{}, snt);
    else
      k_window<10224, true, AlgoCity64, Sink64T<true>, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, offsets, 0, 0, 0, n, AlgoCity64{}, snt);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  if (v >= 176 && v <= 179) {
    // the pipelined window kernel's data movement (digest = key length, no
    // LDS reads): 176 with its stores, 177 stores into a 32 KiB ring (no HBM
    // writes); 178/179 the same with CityHash64 (178 = variant 170's kernel)
    if (n == 0) return 0;
    int dev;
    if (int rc = current_device(&dev)) return rc;
    const uint8_t *b = static_cast<const uint8_t *>(bytes);
    const u64 wb = ((n + 63) / 64 + 3) / 4;
    g_kernel = "k_window_pipe<var,calib>";
    if (v == 176)
      k_window_pipe<10224, 1, AlgoLenOnly, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(b, offsets, 0, n,
                                                                                          AlgoLenOnly{}, out);
    else if (v == 177)
      k_window_pipe<10224, 1, AlgoLenOnly, 2, LdsReader, 64><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, offsets, 0, n, AlgoLenOnly{}, out);
    else if (v == 178)
      k_window_pipe<10224, 1, AlgoCity64, 2><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(b, offsets, 0, n,
                                                                                         AlgoCity64{}, out);
    else
      k_window_pipe<10224, 1, AlgoCity64, 2, LdsReader, 64><<<grid_for(wb, 4, dev), kBlock, 0, ST(s)>>>(
          b, offsets, 0, n, AlgoCity64{}, out);
    HIP_TRY(hipGetLastError());
    return 0;
  }
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
    else  // 45: windows start on a 128-B line
      k_window<10224, true, AlgoLenOnly, Sink64T<true>, 2, 128><<<grid_for(wb, 4, dev), kBlock, 0, st>>>(
          b, offsets, 0, 0, 0, n, AlgoLenOnly{}, snt);
    HIP_TRY(hipGetLastError());
    return 0;
  }
  return kNoVariant;
}

// pdht_citycrc128_batch_dev, keys > 900 B
static int hook_crc128_long(const void *keys, size_t stride, size_t keylen, size_t n, uint64_t *out,
                            pdht_hip_stream_t s) {
  if (tuning_variant() == 153)  // timing only: no CRC lookups (wrong digests)
    return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128, 0>{}, Sink128{nullptr, out}, ST(s));
  if (tuning_variant() == 150)  // r02's 6-bit-slice tables
    return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128, 6>{}, Sink128{nullptr, out}, ST(s));
  if (tuning_variant() == 303)  // r06: 11-bit-slice tables (6 lookups per word)
    return launch_fixed(keys, stride, keylen, n, CrcLds<AlgoCrc128, 11>{}, Sink128{nullptr, out}, ST(s));
  return kNoVariant;
}

}  // namespace pdht
