// tuning/bucket_two_pass_r05.h -- the r02-r05 two-pass bucketing (A/B
// build only: tuning/pdht_hooks_bucket.h includes it; tuning variants 290,
// 202, 264-272).  The product sorts in the tile-local form of r06
// (bucket.h k_bucket_tl_*); this one stays as the baseline the A/B harness
// measures that form against (EXPERIMENTS.md §4.4, §R6).
#pragma once

namespace pdht {

// ----------------------------------------------------- two-pass bucketing ---
// One pass writes, per 4096-key tile, one run per bucket into every output
// array: at 1024 ranks runs of 4 keys (32 B of an 8-B array, 16 B of a 4-B
// one), and the write path runs at ~1.3-3 TB/s on such runs against ~4.5 on
// >= 128-B runs (tools/scatter_probe.hip).  Two stable passes over the two
// digits of rank = c * F + f (F = 2^fbits fine buckets, C = ceil(nranks / F)
// coarse ones, F, C ~ sqrt(nranks)) write runs of ~4096 / F and ~4096 / C
// keys, at the price of an intermediate array (key row + original index):
//   pass 1 (k_bucket_pass1): per counting tile, the tile's keys in fine-bucket
//          order into the intermediate at fbase[f] + (fine-f keys of earlier
//          tiles), stable: the intermediate is ordered by (f, original index);
//   pass 2 (k_bucket_pass2): per segment = (f, SG consecutive count-chunks
//          of kTpChunkTiles tiles), a contiguous stretch of the intermediate that
//          holds, in original order, the fine-f keys of those tiles.  Sorted
//          by c in sub-tiles of 4096 keys, each key goes to its final slot:
//          bucket r = c * F + f receives the segment's keys at base[r] +
//          chunkcnt[g0][r] onwards, in order.
// Both passes take their positions from the single pass's per-tile counts
// (count kernel + scans): no extra counting and no inter-workgroup waits.
#ifndef PDHT_TP_TILE  // compile-time experiments only (make exp EXP=-DPDHT_TP_TILE=...)
#define PDHT_TP_TILE 4096
#endif
#ifndef PDHT_TP_CHUNK_TILES
#define PDHT_TP_CHUNK_TILES 8
#endif
constexpr u32 kTpCountTile = PDHT_TP_TILE;  // counting tile = pass-1 unit
constexpr u32 kTpChunkTiles = PDHT_TP_CHUNK_TILES;  // counting tiles per count-chunk (one count workgroup)
struct TwoPass {
  u32 fbits, F, C, cbits;
  const u32 *countsF;   // [ntiles][F] fine-bucket keys of tile t before it in its fchunk-tile chunk
  const u32 *chunksF;   // [ntiles/fchunk][F] ... of the chunks before it
  u32 fchunk;           // tiles per fine-count chunk
  const u64 *totalsF;   // [F] keys per fine bucket
  const u32 *chunkcnt;  // [nchunks][nranks] keys of rank r in the count-chunks before chunk g
  const u64 *base;      // [nranks] first final slot of bucket r
  const u64 *fbase;     // [F] first intermediate row of fine bucket f
  uint8_t *ikeys;       // [n][L] intermediate key rows
  u32 *iidx;            // [n] intermediate original indices
  u64 ntiles, nchunks;  // counting tiles; count-chunks of kTpChunkTiles tiles
  u64 SG, nsegf, nseg;  // count-chunks per segment (about); segments per f; segments
  // keys of fine bucket f in the tiles before tile t (t <= ntiles)
  __device__ __forceinline__ u32 fine_before(u64 t, u32 f) const {
    return t < ntiles ? countsF[t * F + f] + chunksF[(t / fchunk) * F + f] : (u32)totalsF[f];
  }
};

// Two-pass counting.  One workgroup per count-chunk of kTpChunkTiles
// counting tiles: the fine-bucket histogram of every tile -> countsF[t][f],
// and the rank histogram of the whole chunk -> chunkcnt[g][r].  The single
// pass's per-tile rank rows are as large as the keys at high rank counts
// (4096 tiles x 8192 ranks x 4 B = 128 MB for 16M keys, written, scanned and
// read again); these are nranks/F and kTpChunkTiles times smaller.
// With chunksF (fchunk = kTpChunkTiles), countsF[t][f] is already the
// exclusive scan down the chunk and chunksF[g][f] the chunk's sum, so no
// column scan of countsF follows.
template <int L>
__global__ __launch_bounds__(kBlock) void k_bucket_count_tp(const uint8_t *__restrict__ keys, u64 n, FastMod rk,
                                                            u32 nranks, u32 F, u32 *__restrict__ countsF,
                                                            u32 *__restrict__ chunkcnt, u64 ntiles,
                                                            u32 *__restrict__ chunksF) {
  constexpr int U = 128 / L;
  extern __shared__ u32 hist[];  // [nranks]
  __shared__ u32 fh[kTpMaxDigits];
  const u32 fmask = F - 1;
  const u64 nchunks = (ntiles + kTpChunkTiles - 1) / kTpChunkTiles;
  for (u64 g = blockIdx.x; g < nchunks; g += gridDim.x) {
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) hist[r] = 0;
    u32 facc = 0;  // thread f < F: fine-f keys of the chunk's tiles so far
    const u64 t1 = min((g + 1) * kTpChunkTiles, ntiles);
    for (u64 t = g * kTpChunkTiles; t < t1; ++t) {
      if (threadIdx.x < F) fh[threadIdx.x] = 0;
      __syncthreads();
      const u64 k0 = t * kTpCountTile;
      const u64 kend = min(k0 + kTpCountTile, n);
      for (u64 i = k0 + threadIdx.x; i < kend; i += (u64)kBlock * U) {
        RegReader<L / 4> kr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) load_key_regs<L, true>(keys, min(i + u * kBlock, n - 1), kr[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (i + u * kBlock < kend) {
            const u32 r = (u32)rk.mod(city64(kr[u], (u64)L));
            atomicAdd(&hist[r], 1u);
            atomicAdd(&fh[r & fmask], 1u);
          }
      }
      __syncthreads();
      if (threadIdx.x < F) {
        const u32 c = fh[threadIdx.x];
        countsF[t * F + threadIdx.x] = chunksF ? facc : c;
        facc += c;
      }
    }
    if (chunksF && threadIdx.x < F) chunksF[g * F + threadIdx.x] = facc;
    __syncthreads();
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) chunkcnt[g * nranks + r] = hist[r];
    __syncthreads();
  }
}

// Two independent chunk scans in one launch (two-pass bucketing: the fine
// buckets' count-chunk sums and the ranks' count-chunk histograms): blocks
// [0, nb1) scan the first, the rest the second.
__global__ __launch_bounds__(64 * kCsWaves) void k_bucket_chunkscan2(u32 *__restrict__ c1, u64 n1, u32 w1,
                                                                     u64 *__restrict__ t1, u32 nb1,
                                                                     u32 *__restrict__ c2, u64 n2, u32 w2,
                                                                     u64 *__restrict__ t2) {
  if (blockIdx.x < nb1)
    chunkscan_block(blockIdx.x, c1, n1, w1, t1);
  else
    chunkscan_block(blockIdx.x - nb1, c2, n2, w2, t2);
}


// Pass-1 units are the counting tiles (kTpCountTile keys); both passes work
// through their units in sub-tiles of W x KPL x 64 keys, carrying each
// digit's next slot across sub-tiles.  Runs stay long with small sub-tiles
// (1024 keys over 32 digits: 32-key runs), and small sub-tiles keep LDS and
// VGPRs per workgroup low, so that several workgroups per CU overlap one
// another's load / rank / store phases.
// r02-r03 shape of both passes (4 waves x 8 keys per lane, 4 WG/CU); since r04
// pass 1 runs 8 x 8 @ 2 and 16-B keys' pass 2 too (launch_two_pass_sel).
constexpr int kTpW = 4, kTpKPL = 8, kTpPerCu = 4;
template <int W, int KPL>
constexpr size_t pass1_lds_bytes() { return (size_t)W * KPL * 64 * (8 + 2 + 1); }
template <int W, int KPL>
constexpr size_t pass2_lds_bytes() { return (size_t)W * KPL * 64 * (8 + 4); }

template <int L, int W = kTpW, int KPL = kTpKPL, int WPE = 8>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_bucket_pass1(const uint8_t *__restrict__ keys, u64 n, FastMod rk, TwoPass tp) {
  constexpr u32 kTile = W * KPL * 64, kB = W * 64, kSub = KPL * 64;
  static_assert(kTpCountTile % kTile == 0, "sub-tiles of a counting tile");
  extern __shared__ u64 lds64[];
  u64 *stage = lds64;                                            // [kTile] key pieces
  uint16_t *sidx = reinterpret_cast<uint16_t *>(stage + kTile);  // [kTile] sub-tile-local index
  uint8_t *sdig = reinterpret_cast<uint8_t *>(sidx + kTile);     // [kTile] fine digit
  __shared__ u32 runt[W * kTpMaxDigits];
  __shared__ u32 running[kTpMaxDigits];  // next intermediate row of fine bucket f
  __shared__ u32 delta[kTpMaxDigits];
  __shared__ u32 tcount[kTpMaxDigits];
  __shared__ u32 scan_scratch[W];
  const RunTab<false> run{runt, tp.F};
  const u32 fmask = tp.F - 1;
  const u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32 q0 = wave * kSub + lane;
  for (TileOrder o(tp.ntiles); o.t < o.end; o.t += o.step) {
    const u64 t = o.t;
    const u64 tbase = t * kTpCountTile;
    const u32 ttn = (u32)min((u64)kTpCountTile, n - tbase);
    // the tile's rows in fine bucket f follow those of the earlier tiles
    if (threadIdx.x < tp.F) running[threadIdx.x] = (u32)tp.fbase[threadIdx.x] + tp.fine_before(t, threadIdx.x);
    for (u32 s0 = 0; s0 < ttn; s0 += kTile) {
      const u32 tn = min(kTile, ttn - s0);
      const u64 sbase = tbase + s0;
      for (u32 j = threadIdx.x; j < W * tp.F; j += kB) runt[j] = 0;
      RegReader<L / 4> kr[KPL];
#pragma unroll
      for (int g = 0; g < KPL; ++g) load_key_regs<L, true>(keys, min(sbase + q0 + g * 64, n - 1), kr[g]);
      u32 ff[KPL];
#pragma unroll
      for (int g = 0; g < KPL; ++g) ff[g] = (u32)rk.mod(city64(kr[g], (u64)L)) & fmask;
      __syncthreads();
#pragma unroll
      for (int g = 0; g < KPL; ++g)
        if (q0 + g * 64 < tn) run.add(wave, ff[g], 1u);
      __syncthreads();
      digit_starts<W>(run, tp.F, delta, tcount, scan_scratch, [&](u32 f) { return running[f]; });
      __syncthreads();
      u32 lp[KPL];
      rank_groups<KPL>(run, wave, ff, q0, tn, tp.fbits, lp);
#pragma unroll
      for (int g = 0; g < KPL; ++g)
        if (q0 + g * 64 < tn) {
          stage[lp[g]] = (u64)kr[g].d[0] | ((u64)kr[g].d[1] << 32);
          sidx[lp[g]] = (uint16_t)(q0 + g * 64);
          sdig[lp[g]] = (uint8_t)ff[g];
        }
      __syncthreads();
      u32 gp[KPL];
#pragma unroll
      for (int jj = 0; jj < KPL; ++jj) {
        const u32 j = jj * kB + threadIdx.x;
        if (j < tn) {
          gp[jj] = delta[sdig[j]] + j;
          tp.iidx[gp[jj]] = (u32)(sbase + sidx[j]);
          *reinterpret_cast<u64 *>(tp.ikeys + (u64)gp[jj] * L) = stage[j];
        }
      }
#pragma unroll
      for (int c = 1; c < L / 8; ++c) {
        __syncthreads();
#pragma unroll
        for (int g = 0; g < KPL; ++g)
          if (q0 + g * 64 < tn) stage[lp[g]] = (u64)kr[g].d[2 * c] | ((u64)kr[g].d[2 * c + 1] << 32);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < KPL; ++jj) {
          const u32 j = jj * kB + threadIdx.x;
          if (j < tn) *reinterpret_cast<u64 *>(tp.ikeys + (u64)gp[jj] * L + 8 * c) = stage[j];
        }
      }
      __syncthreads();
      if (threadIdx.x < tp.F) running[threadIdx.x] += tcount[threadIdx.x];
    }
    __syncthreads();
  }
}

// ONE (8-B keys into arrays, the default there since late r05): the sub-tile
// stages {key, index} instead of {digest, index} and hashes each key a
// second time in the store phase, so all four outputs of a key leave in one
// phase -- two barriers and one LDS round per sub-tile fewer than staging the
// digest first and the key bytes after it (staged_store).  Interleaved, 16M
// keys at 8192 ranks: -1.0 to -1.3 % (profiles/r05/ab/bucket8k_pass2_one_store_phase.log).
template <int L, class Out, int W = kTpW, int KPL = kTpKPL, int WPE = 8, bool ONE = (L == 8 && !Out::kPair8)>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_bucket_pass2(FastMod rk, u32 nranks, TwoPass tp, Out out) {
  static_assert(!ONE || (L == 8 && !Out::kPair8), "one store phase: 8-B keys into arrays");
  constexpr u32 kTile = W * KPL * 64, kB = W * 64, kSub = KPL * 64;
  extern __shared__ u64 lds64[];
  u64 *stage = lds64;                                    // [kTile] digests, then key pieces (ONE: keys)
  u32 *sidx = reinterpret_cast<u32 *>(stage + kTile);  // [kTile] original index
  __shared__ u32 runt[W * kTpMaxDigits];
  __shared__ u32 running[kTpMaxDigits];  // next final slot of bucket c*F + f
  __shared__ u32 delta[kTpMaxDigits];
  __shared__ u32 tcount[kTpMaxDigits];
  __shared__ u32 seg[2];  // rows of the segment before it in fine bucket f; its length
  __shared__ u32 scan_scratch[W];
  const RunTab<false> run{runt, tp.C};
  const u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32 q0 = wave * kSub + lane;
  const u32 fbits = tp.fbits;
  auto coarse = [&](u64 h, u32) { return (u32)rk.mod(h) >> fbits; };
  for (TileOrder o(tp.nseg); o.t < o.end; o.t += o.step) {
    const u32 f = (u32)(o.t / tp.nsegf);
    const u64 sg = o.t % tp.nsegf;  // the f-bucket's count-chunks split evenly over nsegf segments
    const u64 g0 = sg * tp.nchunks / tp.nsegf, g1 = (sg + 1) * tp.nchunks / tp.nsegf;
    if (threadIdx.x == 0) {
      const u32 lo = tp.fine_before(g0 * kTpChunkTiles, f);
      seg[0] = lo;
      seg[1] = tp.fine_before(min(g1 * kTpChunkTiles, tp.ntiles), f) - lo;
    }
    if (threadIdx.x < tp.C) {
      const u32 r = threadIdx.x * tp.F + f;
      if (r < nranks) running[threadIdx.x] = (u32)tp.base[r] + tp.chunkcnt[g0 * nranks + r];
    }
    __syncthreads();
    const u32 sstart = (u32)tp.fbase[f] + seg[0], slen = seg[1];
    for (u32 k0 = 0; k0 < slen; k0 += kTile) {
      const u32 tn = min(kTile, slen - k0);
      const u64 p0 = (u64)sstart + k0;
      for (u32 j = threadIdx.x; j < W * tp.C; j += kB) runt[j] = 0;
      RegReader<L / 4> kr[KPL];
      u32 ix[KPL];
#pragma unroll
      for (int g = 0; g < KPL; ++g) {
        const u64 p = p0 + min(q0 + g * 64, tn - 1);
        load_key_regs<L, true>(tp.ikeys, p, kr[g]);
        ix[g] = __builtin_nontemporal_load(tp.iidx + p);
      }
      u64 h[ONE ? 1 : KPL];
      u32 cc[KPL];
#pragma unroll
      for (int g = 0; g < KPL; ++g) {
        const u64 hh = city64(kr[g], (u64)L);
        if constexpr (!ONE) h[g] = hh;
        cc[g] = coarse(hh, 0u);
      }
      __syncthreads();
#pragma unroll
      for (int g = 0; g < KPL; ++g)
        if (q0 + g * 64 < tn) run.add(wave, cc[g], 1u);
      __syncthreads();
      digit_starts<W>(run, tp.C, delta, tcount, scan_scratch, [&](u32 c) { return running[c]; });
      __syncthreads();
      u32 lp[KPL];
      rank_groups<KPL>(run, wave, cc, q0, tn, tp.cbits, lp);
#pragma unroll
      for (int g = 0; g < KPL; ++g)
        if (q0 + g * 64 < tn) {
          if constexpr (ONE)
            stage[lp[g]] = (u64)kr[g].d[0] | ((u64)kr[g].d[1] << 32);
          else
            stage[lp[g]] = h[g];
          sidx[lp[g]] = ix[g];
        }
      __syncthreads();
      if constexpr (ONE) {
        // thread j: staged key j -> hash again -> its slot; every output at once
#pragma unroll
        for (int jj = 0; jj < KPL; ++jj) {
          const u32 j = jj * kB + threadIdx.x;
          if (j < tn) {
            RegReader<2> r;
            const u64 key = stage[j];
            r.d[0] = (u32)key;
            r.d[1] = (u32)(key >> 32);
            const u64 hv = city64(r, (u64)L);
            const u32 slot = delta[coarse(hv, 0u)] + j;
            out.meta(slot, hv, sidx[j]);
            if (out.has_keys()) out.key8(slot, 0, key);
          }
        }
      } else {
        staged_store<L, KPL, kB>(stage, delta, tn, kr, lp, q0, coarse, [&](u32 j) { return (u64)sidx[j]; }, out);
      }
      __syncthreads();
      if (threadIdx.x < tp.C) running[threadIdx.x] += tcount[threadIdx.x];
    }
    __syncthreads();
  }
}


// Pass 1 and pass 2 each take a shape: W waves x KPL keys per lane per
// sub-tile, PER_CU workgroups per CU (pass 1: W1, KPL1, PER_CU1).  Both run
// their units in the static XCD-contiguous order (TileOrder; per-XCD tickets
// gained nothing here, r02 tuning variant 86).
template <int L, class Out, int W = kTpW, int KPL = kTpKPL, int PER_CU = kTpPerCu, int W1 = W, int KPL1 = KPL,
          int PER_CU1 = PER_CU, bool ONE = (L == 8 && !Out::kPair8)>
static int launch_two_pass(const BucketArgs &a, const TwoPass &tp, const Out &out, hipStream_t st, int dev) {
  static const char *const names[3] = {"k_bucket_pass2<8B>", "k_bucket_pass2<16B>", "k_bucket_pass2<32B>"};
  constexpr int WPE = PER_CU * W / 4 > 8 ? 8 : PER_CU * W / 4;      // waves per SIMD, pass 2
  constexpr int WPE1 = PER_CU1 * W1 / 4 > 8 ? 8 : PER_CU1 * W1 / 4;  // pass 1
  const size_t b1 = pass1_lds_bytes<W1, KPL1>(), b2 = pass2_lds_bytes<W, KPL>();
  auto f1 = &k_bucket_pass1<L, W1, KPL1, WPE1>;
  auto f2 = &k_bucket_pass2<L, Out, W, KPL, WPE, ONE>;
  if (int rc = set_lds(reinterpret_cast<const void *>(f1), b1)) return rc;
  if (int rc = set_lds(reinterpret_cast<const void *>(f2), b2)) return rc;
  const u64 cus = (u64)std::max(1, g_dev[dev].cus);
  unsigned g1 = (unsigned)std::min<u64>(a.ntiles, cus * PER_CU1);
  if (g1 >= 8) g1 &= ~7u;  // XCD-contiguous tile order (TileOrder)
  f1<<<g1, W1 * 64, b1, st>>>(a.k, a.n, a.rk, tp);
  unsigned g2 = (unsigned)std::min<u64>(tp.nseg, cus * PER_CU);
  if (g2 >= 8) g2 &= ~7u;
  f2<<<g2, W * 64, b2, st>>>(a.rk, a.nranks, tp, out);
  g_kernel = names[L == 8 ? 0 : L == 16 ? 1 : 2];
  return 0;
}


// Shapes of the r02-r05 two passes other than r05's own (variants).
template <int L, class Out>
static int r05_shape(const BucketArgs &a, const TwoPass &tp, const Out &out, hipStream_t st, int dev) {
  // (r04's shape search, tuning 192-201, removed in r05)
  constexpr int kW = L == 8 && !Out::kPair8 ? 1 : 0;  // (ONE exists for 8-B arrays only)
  const int v = tuning_variant();
  if (v == 202)  // r02-r03: 4 x 8 @ 4 both, pass 2 storing in two phases
    return launch_two_pass<L, Out, kTpW, kTpKPL, kTpPerCu, kTpW, kTpKPL, kTpPerCu, false>(a, tp, out, st, dev);
  if (kW && v == 265)  // r04-r05 product for 8-B arrays: pass 2 two-phase 4 x 8 @ 4
    return launch_two_pass<L, Out, kTpW, kTpKPL, kTpPerCu, 8, 8, 2, false>(a, tp, out, st, dev);
  if (kW && v == 266)  // ONE in 4 x 8 @ 4
    return launch_two_pass<L, Out, kTpW, kTpKPL, kTpPerCu, 8, 8, 2>(a, tp, out, st, dev);
  if constexpr (L >= 16) {  // r05 spill probe (16/32-B keys in 4 keys per lane) and the r04-r05 shapes
    switch (v) {
      case 267: return launch_two_pass<L, Out, 8, 4, 2, 8, 4, 2>(a, tp, out, st, dev);
      case 268: return launch_two_pass<L, Out, 4, 4, 4, 8, 4, 2>(a, tp, out, st, dev);
      case 269: return launch_two_pass<L, Out, 8, 4, 2, 4, 8, 4>(a, tp, out, st, dev);
      case 270:
        if constexpr (L == 16) return launch_two_pass<L, Out, 8, 8, 2, 8, 8, 2>(a, tp, out, st, dev);
        else return launch_two_pass<L, Out, kTpW, kTpKPL, kTpPerCu, 8, 8, 2>(a, tp, out, st, dev);
      default: break;
    }
  }
  if constexpr (L == 8 && Out::kPair8) {  // 8-B records' pass 2: 4 x 4 @ 4 / r04-r05's 4 x 8 @ 4
    if (v == 271) return launch_two_pass<L, Out, 4, 4, 4, 8, 8, 2>(a, tp, out, st, dev);
    if (v == 272) return launch_two_pass<L, Out, kTpW, kTpKPL, kTpPerCu, 8, 8, 2>(a, tp, out, st, dev);
  }
  return kNoVariant;
}

template <int L, class Out>
static int launch_two_pass_sel(const BucketArgs &a, const TwoPass &tp, const Out &out, hipStream_t st, int dev) {
  // Shapes (waves x keys per lane per sub-tile @ workgroups per CU).  r02's
  // A/B (8 x 4 / 4 x 16 / 4 x 4 keys, 2-6 WG/CU, per-XCD tile tickets) kept
  // 4 x 8 @ 4 for both passes.  r04, interleaved, after the fine-plus digit
  // split had moved work into pass 1 (profiles/r04/ab/bucket_*_tp_shapes*.log):
  // pass 1 in 8 x 8 @ 2 (4096-key sub-tiles = one counting tile, runs twice as
  // long, half the barriers per key): 8-B keys at 8192 / 2048 ranks -11 /
  // -10.5 %, 32-B at 4096 -4 %; 16-B keys gain most with pass 2 in 8 x 8 @ 2
  // as well (-9 % at 4096 ranks; 8-B keys +4 % with it).  Pass 2 in 8 x 8 @ 3
  // or 16 x 4 @ 2, pass 1 in 4 x 16 / 16 x 4 / 8 x 4: slower.  Late r05:
  // 8-B keys into arrays store from one phase (k_bucket_pass2 ONE) and take
  // pass 2 in 8 x 8 @ 2 as well (4 x 8 @ 4 with ONE: equal to the two-phase
  // product; 8 x 8 @ 2: -1.0 to -1.3 %, profiles/r05/ab/bucket8k_*.log).
  if (int rc = r05_shape<L, Out>(a, tp, out, st, dev); rc != kNoVariant) return rc;
  // Late r05: at 8 keys per lane the 16/32-B kernels spilled VGPRs (pass 1
  // of 32-B keys 78 registers, pass 2 58); in 4 keys per lane none spill
  // (profiles/r05/ab/bucket_16_32_two_pass_shapes.log, 16M keys): 32-B arrays
  // at 4096 / 8192 ranks 1.293 -> 0.936 / 1.327 -> 0.978 ms (both passes 8 x 4
  // @ 2), 32-B records at 8192 ranks 1.728 -> 1.165 and 16-B records at 4096
  // 0.751 -> 0.656 (pass 2 in 4 x 4 @ 4); 16-B arrays keep 8 x 8 @ 2 (4 keys
  // per lane +5 %).  8-B records' pass 2 (5 VGPRs spilled at 4 x 8 @ 4) in 8 x
  // 4 @ 2: 8192 / 2048 ranks 0.389 -> 0.369 / 0.363 -> 0.346 ms.
  if constexpr (L == 32 && !Out::kPair8)
    return launch_two_pass<L, Out, 8, 4, 2, 8, 4, 2>(a, tp, out, st, dev);
  else if constexpr (L >= 16 && Out::kPair8)
    return launch_two_pass<L, Out, 4, 4, 4, 8, 4, 2>(a, tp, out, st, dev);
  else if constexpr (L == 16 || (L == 8 && !Out::kPair8))
    return launch_two_pass<L, Out, 8, 8, 2, 8, 8, 2>(a, tp, out, st, dev);
  else
    return launch_two_pass<L, Out, 8, 4, 2, 8, 8, 2>(a, tp, out, st, dev);
}


// First intermediate row of every fine bucket: the exclusive scan of the
// fine totals (r05 did this inside k_bucket_base; one more small launch here).
__global__ __launch_bounds__(kTpMaxDigits) void k_bucket_fbase(const u64 *__restrict__ ftot, u32 F,
                                                               u64 *__restrict__ fbase) {
  __shared__ u64 scratch[kTpMaxDigits / 64];
  const u64 v = threadIdx.x < F ? ftot[threadIdx.x] : 0;
  const u64 e = block_exclusive_scan<kTpMaxDigits / 64, u64>(v, scratch);
  if (threadIdx.x < F) fbase[threadIdx.x] = e;
}

// The r02-r05 workspace inside the two-pass region (BucketWs::region):
// fine-bucket counts per tile (scanned down each count-chunk) and per
// count-chunk, fine totals and bases, rank counts per count-chunk, and the
// intermediate ([n][keysize] key rows + [n] original indices).
struct R05Ws {
  u32 *countsF, *chunksF, *chunkcnt;
  u64 *totalsF, *fbase;
  uint8_t *ikeys;
  u32 *iidx;
  size_t bytes;
};
static R05Ws r05_layout(uint8_t *p, size_t n, size_t keysize, u32 nranks) {
  const u64 tiles = (n + kTpCountTile - 1) / kTpCountTile;
  const u64 chunks = (tiles + kTpChunkTiles - 1) / kTpChunkTiles;
  R05Ws r{};
  size_t o = 0;
  auto take = [&](size_t bytes) {
    uint8_t *q = p ? p + o : nullptr;
    o += round256(bytes);
    return q;
  };
  r.countsF = reinterpret_cast<u32 *>(take((size_t)tiles * kTpMaxDigits * 4));
  r.chunksF = reinterpret_cast<u32 *>(take((size_t)chunks * kTpMaxDigits * 4));  // rows of kTpChunkTiles (or kBucketChunk) tiles
  r.totalsF = reinterpret_cast<u64 *>(take((size_t)kTpMaxDigits * 8));
  r.fbase = reinterpret_cast<u64 *>(take((size_t)kTpMaxDigits * 8));
  r.chunkcnt = reinterpret_cast<u32 *>(take((size_t)chunks * nranks * 4));
  r.ikeys = take(n * keysize);
  r.iidx = reinterpret_cast<u32 *>(take(n * 4));
  r.bytes = o;
  return r;
}

static inline bool tuning_two_pass_r05() {
  const int v = tuning_variant();
  return v == 290 || v == 202 || v == 264 || (v >= 265 && v <= 272);
}

// The r02-r05 two passes of one batch (n >= 0): count kernel (fine counts
// per tile, rank counts per count-chunk), the chunk scans, bucket and fine
// bases, pass 1 (fine-bucket runs to global positions), pass 2.
template <class Out>
static int bucket_r05(const BucketArgs &a0, const BucketWs &w, size_t keysize, const Out &out,
                      uint64_t *bucket_offsets, hipStream_t st, int dev) {
  const u64 n = a0.n;
  const u32 nranks = a0.nranks;
  const R05Ws r = r05_layout(w.region, n, keysize, nranks);
  BucketArgs a = a0;
  const u64 ntiles = (n + kTpCountTile - 1) / kTpCountTile;
  a.ntiles = ntiles;
  const Digits d = digit_split<Out>(a.nbits, nranks, keysize);
  if (d.F > kTpMaxDigits || d.C > kTpMaxDigits)
    return fail("two-pass digit split: a digit of %s%lld buckets exceeds the LDS tables", "",
                (long long)(d.F > kTpMaxDigits ? d.F : d.C));
  TwoPass tp{};
  tp.fbits = d.fbits;
  tp.F = d.F;
  tp.C = d.C;
  tp.cbits = d.cbits;
  tp.countsF = r.countsF;
  tp.chunksF = r.chunksF;
  tp.totalsF = r.totalsF;
  tp.chunkcnt = r.chunkcnt;
  tp.base = w.base;
  tp.fbase = r.fbase;
  tp.ikeys = r.ikeys;
  tp.iidx = r.iidx;
  tp.ntiles = ntiles;
  tp.nchunks = (ntiles + kTpChunkTiles - 1) / kTpChunkTiles;
  split_segments(tp.nchunks, (u64)kTpChunkTiles * kTpCountTile, tp.F, &tp.SG, &tp.nsegf);
  tp.nseg = (u64)tp.F * tp.nsegf;
  const size_t hist_lds = (size_t)nranks * 4;
  if (ntiles) {
    // the count kernel scans the fine counts down each count-chunk itself
    // (no column-scan launch); 264: the r02-r05 colscan over 32-tile chunks
    const bool fscan = tuning_variant() != 264;
    tp.fchunk = fscan ? kTpChunkTiles : kBucketChunk;
    const u64 nfchunks = (ntiles + tp.fchunk - 1) / tp.fchunk;
    u32 *cF = fscan ? r.chunksF : nullptr;
    const unsigned gc = (unsigned)std::min<u64>(tp.nchunks, (u64)std::max(1, g_dev[dev].cus) * 8);
    if (keysize == 8)
      k_bucket_count_tp<8><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, tp.F, r.countsF, r.chunkcnt,
                                                          ntiles, cF);
    else if (keysize == 16)
      k_bucket_count_tp<16><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, tp.F, r.countsF, r.chunkcnt,
                                                           ntiles, cF);
    else
      k_bucket_count_tp<32><<<gc, kBlock, hist_lds, st>>>(a.k, n, a.rk, nranks, tp.F, r.countsF, r.chunkcnt,
                                                           ntiles, cF);
    if (!fscan)
      k_bucket_colscan<<<dim3((tp.F + 63) / 64, (unsigned)nfchunks), 64, 0, st>>>(r.countsF, ntiles, tp.F,
                                                                                   r.chunksF);
    const u32 nbF = (tp.F + 63) / 64;  // both chunk scans in one launch
    k_bucket_chunkscan2<<<nbF + (nranks + 63) / 64, 64 * kCsWaves, 0, st>>>(
        r.chunksF, nfchunks, tp.F, r.totalsF, nbF, r.chunkcnt, tp.nchunks, nranks, w.totals);
  } else {
    HIP_TRY(hipMemsetAsync(w.totals, 0, (size_t)nranks * 8, st));
  }
  k_bucket_base<<<1, kBaseThreads, 0, st>>>(w.totals, nranks, w.base, bucket_offsets, nullptr);
  g_kernel = "k_bucket_base";
  if (!ntiles) return 0;
  k_bucket_fbase<<<1, kTpMaxDigits, 0, st>>>(r.totalsF, tp.F, r.fbase);
  return keysize == 8    ? launch_two_pass_sel<8, Out>(a, tp, out, st, dev)
         : keysize == 16 ? launch_two_pass_sel<16, Out>(a, tp, out, st, dev)
                         : launch_two_pass_sel<32, Out>(a, tp, out, st, dev);
}

// The hooks pdht_bucket.hip calls: the r02-r05 form under its variants, and
// a two-pass region large enough for either form.
template <class Out>
static int hook_two_pass_r05(const BucketArgs &a, const BucketWs &w, size_t keysize, const Out &out,
                             uint64_t *bucket_offsets, hipStream_t st, int dev) {
  if (!tuning_two_pass_r05()) return kNoVariant;
  return bucket_r05<Out>(a, w, keysize, out, bucket_offsets, st, dev);
}
static inline size_t hook_two_pass_region(size_t dflt, size_t n, size_t keysize, u32 nranks) {
  return std::max(dflt, r05_layout(nullptr, n, keysize, nranks).bytes);
}

}  // namespace pdht
