// pdht_bucket.hip -- destination bucketing (include/pdht_hip.h
// pdht_bucket_batch_dev / pdht_bucket_records_dev; kernels in bucket.h).
#include "bucket.h"
#include "runtime.h"

// ------------------------------------------------- destination bucketing ---
#ifndef PDHT_TP_EVEN_SEG  // compile-time A/B only
#define PDHT_TP_EVEN_SEG 1
#endif
namespace pdht {
struct BucketWs {
  u32 *counts, *chunks;
  u64 *totals, *base;
  u32 *tickets;  // [8] per-XCD tile tickets of the dynamic scatter
  // the two-pass region (8/16/32-B keys from two_pass_min_ranks()): the
  // tile-local sort's per-tile f-run starts, per-chunk rank histograms, key
  // rows and their u16 indices inside the tile
  uint8_t *region;
  uint16_t *tl_starts, *tl_lidx;
  u32 *tl_chunkcnt;
  uint8_t *tl_keys;
  size_t bytes;
};
static size_t round256(size_t x) { return (x + 255) & ~(size_t)255; }
static bool two_pass_keysize(size_t keysize) { return keysize == 8 || keysize == 16 || keysize == 32; }
// Two-pass bucketing from this many ranks up.  The one-pass staged scatter
// wins while its owner-table shapes fit (staged_shape): arrays of 8/16-B keys
// on 8 x 16 tiles up to 1574 ranks, 16-B records on 4 x 16 tiles up to 1462,
// 8-B records (ballots at two workgroups per CU) up to 2047; past those the
// tile-local two passes win (r06, both forms re-measured after their r06
// load-policy changes, profiles/r06/ab/bucket_two_pass_thresholds.log: 8-B
// arrays at 1536 ranks 0.269 one pass / 0.309 two, at 2048 0.463 / 0.294;
// 16-B arrays at 1025 / 1536 0.385 / 0.411 against 0.426 / 0.430, at 1576
// 0.540 / 0.441; 8-B records at 1536-1792 0.308-0.313 / 0.332-0.335, at
// 2048 0.472 / 0.325; 16-B records at 1462 0.547 / 0.575, at 1536 0.592 /
// 0.582).  32-B arrays stay one pass to 2048 (0.838 / 0.906 at 2048); 32-B
// records take two passes from 256 ranks (256 / 512 / 1024: 1.071 / 1.067 /
// 1.093 against 1.111 / 1.130 / 1.166; below 256 not measured).
static u32 two_pass_min_ranks(size_t keysize, bool records) {
  if (records) return keysize == 8 ? 2048 : keysize == 16 ? 1463 : 256;
  return keysize == 32 ? 2049 : 1575;
}
// Tile-local two-pass sort (r06, bucket.h k_bucket_tl_*): pass-1 tiles of
// 4096 keys for 8-B keys, 2048 for 16/32-B keys (8 waves x 4 keys per lane,
// spill-free; 16-B keys in 4096-key tiles spilled 23 VGPRs and ran 0.4-1.9 %
// slower, profiles/r06/ab/bucket_16_tl_pass1_tiles.log), one
// sub-tile each; count-chunks of ct tiles, ct the largest power of two <= 8
// that still leaves >= 512 chunks (two pass-1 workgroups on each of 256
// CUs), so that a chunk's histogram never counts past 32768 keys (u16 halves
// in LDS).  Both depend on n only, so the workspace size does too.
static u32 tl_tile_shift(size_t keysize) { return hook_tl_tile_shift(keysize == 8 ? 12 : 11, keysize); }
static u32 tl_chunk_tiles(u64 ntiles, u32 tshift) {
  u32 ct = std::min<u32>(8, 32768u >> tshift);
  while (ct > 1 && ntiles / ct < 512) ct >>= 1;
  return ct;
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

template <int L, class Out, bool PACK = false, int W = kStW, int KPL = kStKPL, bool DYN = false, int OB = 0,
          bool NTK = false>
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
  auto fn = &k_bucket_scatter_staged<L, Out, W, KPL, PACK, DYN, OB, NTK>;
  if (int rc = set_lds(reinterpret_cast<const void *>(fn), bytes)) return rc;
  const int per_cu = bytes <= 53 * 1024 ? 3 : bytes <= 80 * 1024 ? 2 : 1;
  unsigned g = (unsigned)std::min<u64>(a.ntiles, (u64)std::max(1, g_dev[dev].cus) * per_cu);
  if (g >= 8) g &= ~7u;  // a multiple of 8: XCD-contiguous tile order (TileOrder)
  // (DYN: 8 XCD groups need a grid that is a multiple of 8; small grids use
  // the static order)
  if (DYN && g % 8 == 0)
    fn<<<g, W * 64, bytes, st>>>(a.k, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out, tickets);
  else
    k_bucket_scatter_staged<L, Out, W, KPL, PACK, false, OB, NTK>
        <<<g, W * 64, bytes, st>>>(a.k, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out, nullptr);
  return 0;
}



template <int W, class Out>
static int launch_wg(const BucketArgs &a, const Out &out, u32 L, hipStream_t st, int dev) {
  g_kernel = W == 8 ? "k_bucket_scatter_wg<8>" : "k_bucket_scatter_wg<4>";
  const size_t bytes = (size_t)W * a.nranks * 4;
  if (int rc = set_lds(reinterpret_cast<const void *>(&k_bucket_scatter_wg<W, Out>), bytes)) return rc;
  k_bucket_scatter_wg<W, Out><<<grid_for(a.ntiles, 4, dev), W * 64, bytes, st>>>(
      a.k, L, a.n, a.rk, a.nranks, a.nbits, a.ts, a.ntiles, out);
  return 0;
}




// The tile-local two-pass sort (bucket.h k_bucket_tl_*): pass 1 (sorts
// each tile by f in place, counts ranks per chunk), the rank scan down the
// chunks (and in-block prefixes of the rank totals), pass 2 (forms the bucket
// bases and writes bucket_offsets, gathers the f-runs of each segment, sorts
// by c, stores at the final slots).  Pass 1 in W1 x KPL1 (one tile) @ PER_CU1,
// pass 2 in W x KPL @ PER_CU.
template <int L, class Out, int W, int KPL, int PER_CU, int W1, int KPL1, int PER_CU1, int PROBE = 0,
          bool NTG = (L == 32 && Out::kPair8), bool NTK1 = true, bool ONE = (L == 8 && !Out::kPair8)>
static int launch_tl(const BucketArgs &a, const TwoPassTL &tl, const Out &out, const BucketWs &w,
                     uint64_t *bucket_offsets, hipStream_t st, int dev) {
  static const char *const names[3] = {"k_bucket_tl_pass2<8B>", "k_bucket_tl_pass2<16B>",
                                       "k_bucket_tl_pass2<32B>"};
  if ((1u << tl.tshift) != (u32)(W1 * KPL1 * 64)) return fail("tile-local pass 1: tile/shape mismatch%s", "");
  constexpr int WPE = PER_CU * W / 4 > 8 ? 8 : PER_CU * W / 4;
  constexpr int WPE1 = PER_CU1 * W1 / 4 > 8 ? 8 : PER_CU1 * W1 / 4;
  const size_t b1 = tl_pass1_lds_bytes<W1, KPL1>(a.nranks), b2 = tl_pass2_lds_bytes<W, KPL>();
  auto f1 = &k_bucket_tl_pass1<L, W1, KPL1, WPE1, NTK1>;
  auto f2 = &k_bucket_tl_pass2<L, Out, W, KPL, WPE, ONE, PROBE, NTG>;
  if (int rc = set_lds(reinterpret_cast<const void *>(f1), b1)) return rc;
  if (int rc = set_lds(reinterpret_cast<const void *>(f2), b2)) return rc;
  const u64 cus = (u64)std::max(1, g_dev[dev].cus);
  unsigned g1 = (unsigned)std::min<u64>(tl.nchunks, cus * PER_CU1);
  if (g1 >= 8) g1 &= ~7u;  // XCD-contiguous chunk order (TileOrder)
  f1<<<g1, W1 * 64, b1, st>>>(a.k, a.rk, a.nranks, tl);
  k_bucket_chunkscan_tl<<<(a.nranks + 63) / 64, 64 * kCsWaves, 0, st>>>(tl.chunkcnt, tl.nchunks, a.nranks,
                                                                       w.totals, tl.inpre, tl.bsum);
  unsigned g2 = (unsigned)std::min<u64>(tl.nseg, cus * PER_CU);
  if (g2 >= 8) g2 &= ~7u;
  f2<<<g2, W * 64, b2, st>>>(a.rk, a.nranks, tl, out);
  g_kernel = names[L == 8 ? 0 : L == 16 ? 1 : 2];
  return 0;
}

// The two digits of rank = c * F + f.  Array outputs of 8/16-B keys take one
// fine bit more than the balanced split (8192 ranks: F = 256, C = 32): pass 2
// writes 24 / 32 B per key in runs of ~4096 / C keys against pass 1's 12 / 20 B
// in runs of ~4096 / F, so longer pass-2 runs pay.  Three boxes, 16M keys
// (profiles/r03/ab/bucket_two_pass_digits.log, the r02-r05 form): 8 B at
// 8192 ranks -5.5 / 0 / -3.6 %, 16 B at 4096 ranks -4.3 / -4.0 %, 2048
// ranks within +-2 %.  32-B keys (pass 1 writes 36 B/key) lost 3 % with it,
// and records (AoS rows, pass-2 runs already >= 1 KiB) 1 %: both keep the
// balanced split (the tile-local form on the balanced split, tuning 164:
// +2.3 % at 8192 ranks, EXPERIMENTS.md §R6).
struct Digits {
  u32 fbits, F, C, cbits;
};
template <class Out>
static Digits digit_split(u32 nbits, u32 nranks, size_t keysize) {
  Digits d{};
  d.fbits = (nbits + 1) / 2;
  const bool fine_plus = hook_fine_plus(std::is_same<Out, OutSoA>::value && keysize <= 16);
  if (fine_plus && d.fbits + 1 <= std::min<u32>(8, nbits)) ++d.fbits;
  d.F = 1u << d.fbits;
  d.C = (nranks + d.F - 1) >> d.fbits;
  d.cbits = nbits - d.fbits;
  return d;
}

// Pass-2 segments: nsegf per fine bucket, each a run of whole count-chunks
// (chunk = `chunk_keys` keys, ~chunk_keys / F of them in bucket f), split
// evenly.  SG chunks make ~kTpSegKeys keys; when the remainder of
// nchunks / SG leaves at most one extra chunk per segment, take the floor
// (segments of SG or SG + 1 chunks: ~3968 keys at most) rather than the
// ceiling, whose segments are ~6 % shorter in the mean but one more per fine
// bucket -- one more pass through the sub-tile's phase chain (16M keys at
// 8192 ranks: 17 segments of 30-31 chunks instead of 18).  The even split
// measured equal to a short tail segment for arrays (+-0.5 %,
// profiles/r05/ab/bucket_pass2_even_segments.log; the -1.8 % that log shows
// for 8-B records came from their even split alone: records use the balanced
// digits, F = 128 at 8192 ranks, so they always take the ceiling).  The
// floor applies only where SG + 1 chunks stay ~2 sigma under 4096 keys: F =
// 256 (one chunk more at F <= 128 is 256+ keys and would spill a segment into
// a second sub-tile half the time).  PDHT_TP_EVEN_SEG=0 (experiment builds):
// the ceiling.
static void split_segments(u64 nchunks, u64 chunk_keys, u32 F, u64 *SG, u64 *nsegf) {
  *SG = std::max<u64>(1, (u64)F * kTpSegKeys / chunk_keys);
  const u64 nfl = std::max<u64>(1, nchunks / *SG);
  const u64 step = chunk_keys / F;  // keys of one fine bucket per chunk
  const bool floor_ok = PDHT_TP_EVEN_SEG && (*SG + 1) * step <= 3968 && nchunks - nfl * *SG <= nfl;
  *nsegf = floor_ok ? nfl : (nchunks + *SG - 1) / *SG;
}

enum class BucketKernel { kStaged, kGeneric, kTwoPass };
enum class StagedShape { kBallot4x16, kOwner4x16, kOwner8x16 };
}  // namespace pdht

// A/B hook points of the choices below (product/pdht_hooks_bucket.h: none
// taken)
#include "pdht_hooks_bucket.h"

namespace pdht {
// Sized for the smallest tile any scatter kernel uses, plus the two-pass
// region when the batch can take that path: 8/16/32-B keys from
// two_pass_min_ranks() up for the output kind (records: `records`; the tuning
// build forces two passes at any nranks and always reserves it, at least as
// large as the r02-r05 form needs: hook_two_pass_region).  16M x 8-B keys at
// 1024 ranks: 17 MB; from 1536 ranks + 176 MB.
static BucketWs bucket_layout(void *ws, size_t n, size_t keysize, u32 nranks, bool records) {
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
  w.tickets = reinterpret_cast<u32 *>(p + off);
  off += 256;
  const bool two_pass = hook_bucket_reserve(
      two_pass_keysize(keysize) && nranks >= two_pass_min_ranks(keysize, records), keysize);
  if (two_pass) {
    w.region = p + off;
    size_t q = off;
    const u32 sh = tl_tile_shift(keysize);
    const u64 tl_tiles = (n + (1ull << sh) - 1) >> sh;
    const u64 tl_chunks = (tl_tiles + tl_chunk_tiles(tl_tiles, sh) - 1) / tl_chunk_tiles(tl_tiles, sh);
    w.tl_starts = reinterpret_cast<uint16_t *>(p + q);
    q += round256((size_t)tl_tiles * kTpMaxDigits * 2);
    w.tl_chunkcnt = reinterpret_cast<u32 *>(p + q);
    q += round256((size_t)tl_chunks * nranks * 4);
    w.tl_keys = p + q;
    q += round256(n * keysize);
    w.tl_lidx = reinterpret_cast<uint16_t *>(p + q);
    q += round256(n * 2);
    off = std::max(q, off + hook_two_pass_region((size_t)0, n, keysize, nranks));
  }
  w.bytes = off;
  return w;
}

// Tile-local shapes: pass 1 one tile per sub-tile (8 waves x 8 keys per
// lane = 4096 keys; 16/32-B keys 8 x 4 = 2048, spill-free) at 2 WG/CU; pass 2
// the shapes the r02-r05 pass 2 measured best per key size and output kind
// (tuning/bucket_two_pass_r05.h launch_two_pass_sel), re-measured in r06.
template <int L, class Out>
static int launch_tl_sel(const BucketArgs &a, const TwoPassTL &tl, const Out &out, const BucketWs &w,
                         uint64_t *bucket_offsets, hipStream_t st, int dev) {
  if (int rc = hook_tl_shape<L, Out>(a, tl, out, w, bucket_offsets, st, dev); rc != kNoVariant) return rc;
  // 16-B keys' pass 2 in 8 x 4 @ 2 (8 x 8 spilled 22 VGPRs: arrays -0.5 /
  // -3.1 % at 4096 / 2048 ranks, records from 4 x 4 @ 4 -4.9 %,
  // profiles/r06/ab/bucket_16_tl_pass2_shapes.log)
  if constexpr ((L == 32 && !Out::kPair8) || L == 16)
    return launch_tl<L, Out, 8, 4, 2, 8, 4, 2>(a, tl, out, w, bucket_offsets, st, dev);
  else if constexpr (L == 32)
    return launch_tl<L, Out, 4, 4, 4, 8, 4, 2>(a, tl, out, w, bucket_offsets, st, dev);
  else if constexpr (L == 8 && !Out::kPair8)
    return launch_tl<L, Out, 8, 8, 2, 8, 8, 2>(a, tl, out, w, bucket_offsets, st, dev);
  else
    return launch_tl<L, Out, 8, 4, 2, 8, 8, 2>(a, tl, out, w, bucket_offsets, st, dev);
}

// The tile-local two-pass bucketing (k_bucket_tl_*), n >= 1.
template <class Out>
static int bucket_tl(const BucketArgs &a, const BucketWs &w, size_t keysize, const Out &out,
                     uint64_t *bucket_offsets, hipStream_t st, int dev) {
  const Digits d = digit_split<Out>(a.nbits, a.nranks, keysize);
  if (d.F > kTpMaxDigits || d.C > kTpMaxDigits)  // the kernels' LDS digit tables
    return fail("two-pass digit split: a digit of %s%lld buckets exceeds the LDS tables", "",
                (long long)(d.F > kTpMaxDigits ? d.F : d.C));
  TwoPassTL tl{};
  tl.fbits = d.fbits;
  tl.F = d.F;
  tl.C = d.C;
  tl.cbits = d.cbits;
  tl.tshift = tl_tile_shift(keysize);
  tl.n = a.n;
  tl.ntiles = (a.n + (1ull << tl.tshift) - 1) >> tl.tshift;
  tl.ct = tl_chunk_tiles(tl.ntiles, tl.tshift);
  tl.nchunks = (tl.ntiles + tl.ct - 1) / tl.ct;
  u64 SG = 0;
  split_segments(tl.nchunks, (u64)tl.ct << tl.tshift, tl.F, &SG, &tl.nsegf);
  // a segment's f-runs (one per tile) must fit pass 2's run table
  const u64 seg_tiles = (tl.nchunks + tl.nsegf - 1) / tl.nsegf * tl.ct;
  if (seg_tiles > kTlMaxRuns)
    return fail("tile-local two-pass: %s%lld tiles per segment exceed the run table", "", (long long)seg_tiles);
  tl.og = 1;
  tl.os = (u32)tl.nsegf;
  hook_tl_order(tl.F, tl.nsegf, &tl.og, &tl.os);
  tl.og = std::min(tl.og, tl.F);  // (powers of two: og divides F)
  tl.os = std::max(tl.os, 1u);
  tl.nsgg = (u32)((tl.nsegf + tl.os - 1) / tl.os);
  tl.nseg = (u64)tl.F * tl.nsgg * tl.os;
  tl.startsF = w.tl_starts;
  tl.chunkcnt = w.tl_chunkcnt;
  tl.inpre = reinterpret_cast<u32 *>(w.base);  // (nranks x u64 of space, unused here: 2 x nranks u32)
  tl.bsum = reinterpret_cast<u32 *>(w.base) + a.nranks;
  tl.offsets = bucket_offsets;
  tl.ikeys = w.tl_keys;
  tl.ilidx = w.tl_lidx;
  return keysize == 8    ? launch_tl_sel<8, Out>(a, tl, out, w, bucket_offsets, st, dev)
         : keysize == 16 ? launch_tl_sel<16, Out>(a, tl, out, w, bucket_offsets, st, dev)
                         : launch_tl_sel<32, Out>(a, tl, out, w, bucket_offsets, st, dev);
}

template <class Out>
static StagedShape staged_shape(size_t keysize, u32 nranks) {
  if (nranks < 512) return StagedShape::kBallot4x16;
  if (!std::is_same<Out, OutSoA>::value) {
    // records: owner ranking on 4 x 16 tiles (ab_records_*_shapes.log: 16-B
    // at 1024 ranks 0.62 -> 0.56 ms, 32-B 1.29 -> 1.20); 8-B records lost 3 %
    // with it in r02, and gain 6 % since both halves of a record leave
    // together (r03, profiles/r03/ab/records_shapes.log: 1024 ranks 0.296 ->
    // 0.277 ms, 512 ranks 0.273 -> 0.258); 8 x 16 tiles lose for every size
    if (staged_lds_bytes(nranks, kStW, kStKPL, false, 2) <= 80 * 1024) return StagedShape::kOwner4x16;
    return StagedShape::kBallot4x16;
  }
  // (kStagedStaticLds: the kernels' own __shared__ words, 40 B, on top)
  if (keysize != 32 && staged_lds_bytes(nranks, 8, 16, false, 2) + kStagedStaticLds <= 160 * 1024)
    return StagedShape::kOwner8x16;
  if (staged_lds_bytes(nranks, kStW, kStKPL, false, 2) <= 80 * 1024) return StagedShape::kOwner4x16;
  return StagedShape::kBallot4x16;
}

// Shared by pdht_bucket_batch_dev (OutSoA) and pdht_bucket_records_dev
// (OutRec): the two passes (bucket_tl), or the counting pass, scans, bucket
// bases and the scatter into `out`.  out_al: alignment bits of the output key rows (0
// when they are 8-B aligned 8-B pieces, as in records).
template <class Out>
static int bucket_impl(const void *keys, size_t keysize, size_t n, uint32_t nranks, void *workspace,
                       size_t workspace_bytes, const Out &out, uintptr_t out_al, uint64_t *bucket_offsets,
                       hipStream_t st) {
  if (nranks == 0) return fail("nranks must be > 0%s", "");
  if (nranks > kBucketMaxRanks) return fail("bucketing supports up to 8192 ranks%s", "");
  if (n >= (1ull << 32)) return fail("bucketing: n must be < 2^32 per call%s", "");
  if (!bucket_offsets) return fail("bucket_offsets must not be NULL%s", "");
  if (n && (!keys || keysize == 0)) return fail("null keys or zero keysize%s", "");
  const BucketWs w = bucket_layout(workspace, n, keysize, nranks, Out::kPair8);
  if (!workspace || workspace_bytes < w.bytes) return fail("workspace too small%s", "");
  int dev;
  if (int rc = current_device(&dev)) return rc;
  // Kernel choice: packed 8/16/32-B keys (aligned) -> LDS-staged scatter below
  // the two-pass threshold, two passes from it; other lengths -> generic.
  const uintptr_t al = (uintptr_t)keys | out_al;
  const bool fixed = (keysize == 8 && (al & 7) == 0) || ((keysize == 16 || keysize == 32) && (al & 15) == 0);
  // (two_pass_min_ranks <= kStagedMaxRanks + 1: the staged scatter covers
  // every nranks below the two-pass threshold)
  const BucketKernel kind = hook_bucket_kind(
      !fixed                                                 ? BucketKernel::kGeneric
      : nranks >= two_pass_min_ranks(keysize, Out::kPair8) ? BucketKernel::kTwoPass
                                                             : BucketKernel::kStaged,
      fixed, nranks);
  BucketArgs a{};
  a.k = static_cast<const uint8_t *>(keys);
  a.n = n;
  a.rk = make_fastmod(nranks);
  a.nranks = nranks;
  while ((1u << a.nbits) < nranks) ++a.nbits;
  const size_t hist_lds = (size_t)nranks * 4;
  // Two passes: the tile-local form (r06); no counting pass ahead of pass 1
  // (A/B build: the r02-r05 form under tuning variants 290, 202, 264-272)
  if (kind == BucketKernel::kTwoPass) {
    if (int rc = hook_two_pass_r05(a, w, keysize, out, bucket_offsets, st, dev); rc != kNoVariant) {
      if (rc) return rc;
    } else if (n == 0) {
      HIP_TRY(hipMemsetAsync(w.totals, 0, (size_t)nranks * 8, st));
      k_bucket_base<<<1, kBaseThreads, 0, st>>>(w.totals, nranks, w.base, bucket_offsets, nullptr);
      g_kernel = "k_bucket_base";
    } else if (int rc = bucket_tl(a, w, keysize, out, bucket_offsets, st, dev)) {
      return rc;
    }
    HIP_TRY(hipGetLastError());
    return 0;
  }
  // Staged scatter shape (tools/abbench.py): owner-table
  // ranking for array outputs from 512 ranks; with it, 8 waves x 16 keys per
  // lane (8192-key tiles, 1 WG/CU) for 8/16-B keys while the LDS holds
  // (8-B keys at 1024 ranks 0.274 -> 0.261 ms, 16-B 0.443 -> 0.405; 32-B
  // keys lose 11 % and keep 4 x 16); else 4 x 16 while two workgroups fit a
  // CU (<= 1462 ranks); ballots below 512 ranks and for records.
  const StagedShape shape = hook_staged_shape(staged_shape<Out>(keysize, nranks));
  const u64 st_tile = shape == StagedShape::kOwner8x16 ? 8192 : kStTile;
  const int waves = nranks <= 4096 ? 8 : 4;  // generic: W x nranks x 4 B of LDS <= 128 KiB
  const u64 tile = kind == BucketKernel::kStaged ? st_tile : (u64)waves * kScatKPL * 64;
  const u64 ntiles = (n + tile - 1) / tile;
  const u64 nchunks = (ntiles + kBucketChunk - 1) / kBucketChunk;
  a.ts = TileStarts{w.counts, w.chunks, w.base, nranks};
  a.ntiles = ntiles;
  if (ntiles) {
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
  k_bucket_base<<<1, kBaseThreads, 0, st>>>(w.totals, nranks, w.base, bucket_offsets, w.tickets);
  g_kernel = "k_bucket_base";
  if (ntiles) {
    int rc = hook_staged_launch(kind == BucketKernel::kStaged, keysize, a, out, st, dev, shape, w.tickets);
    if (rc != kNoVariant) {
      // an A/B alternative ran
    } else if (kind == BucketKernel::kStaged && shape == StagedShape::kOwner8x16)
      rc = keysize == 8    ? launch_staged<8, Out, false, 8, 16, true, 2>(a, out, st, dev, w.tickets)
           : keysize == 16 ? launch_staged<16, Out, false, 8, 16, true, 2>(a, out, st, dev, w.tickets)
                           : launch_staged<32, Out, false, 8, 16, true, 2>(a, out, st, dev, w.tickets);
    else if (kind == BucketKernel::kStaged && shape == StagedShape::kOwner4x16)
      rc = keysize == 8    ? launch_staged<8, Out, false, kStW, kStKPL, true, 2>(a, out, st, dev, w.tickets)
           : keysize == 16 ? launch_staged<16, Out, false, kStW, kStKPL, true, 2>(a, out, st, dev, w.tickets)
                           : launch_staged<32, Out, false, kStW, kStKPL, true, 2>(a, out, st, dev, w.tickets);
    else if (kind == BucketKernel::kStaged)  // per-XCD tile tickets
      rc = keysize == 8    ? launch_staged<8, Out, false, kStW, kStKPL, true>(a, out, st, dev, w.tickets)
           : keysize == 16 ? launch_staged<16, Out, false, kStW, kStKPL, true>(a, out, st, dev, w.tickets)
                           : launch_staged<32, Out, false, kStW, kStKPL, true>(a, out, st, dev, w.tickets);
    else
      rc = waves == 8 ? launch_wg<8>(a, out, (u32)keysize, st, dev) : launch_wg<4>(a, out, (u32)keysize, st, dev);
    if (rc) return rc;
  }
  HIP_TRY(hipGetLastError());
  return 0;
}
}  // namespace pdht

using namespace pdht;

// Workspace sizes: array outputs (pdht_bucket_batch_dev) and wire records
// (pdht_bucket_records_dev) switch to the two-pass sort at different rank
// counts (32-B records from 1025 ranks, 32-B arrays from 2049), so each has
// its own query; the records one is never smaller.
PDHT_API size_t pdht_bucket_workspace_bytes(size_t n, size_t keysize, uint32_t nranks) {
  return bucket_layout(nullptr, n, keysize, nranks, false).bytes;
}
PDHT_API size_t pdht_bucket_records_workspace_bytes(size_t n, size_t keysize, uint32_t nranks) {
  return bucket_layout(nullptr, n, keysize, nranks, true).bytes;
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
  if (int rc = hook_records(out, [&](const auto &o2) {
        return bucket_impl(keys, keysize, n, nranks, workspace, workspace_bytes, o2, 0, bucket_offsets, ST(s));
      });
      rc != kNoVariant)
    return rc;
  return bucket_impl(keys, keysize, n, nranks, workspace, workspace_bytes, out, 0, bucket_offsets, ST(s));
}
