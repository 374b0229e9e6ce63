// tuning/pdht_hooks_bucket.h -- the TUNING build's alternatives of the
// bucketing choices (pdht_bucket.hip includes "pdht_hooks_bucket.h" after its
// launch templates; product/pdht_hooks_bucket.h takes none of these).  Every
// variant was measured against the product form (EXPERIMENTS.md).
#pragma once

#include "bucket_two_pass_r05.h"

namespace pdht {

// Tile-local pass-2 segment order, blocks of og fine buckets x os segments
// (the 64 workgroups of an XCD run one block at a time): 296 / 297
// chunk-range-major (og = F, os = 1; 297 on 8192-key tiles, 294); 316-319
// og x os = 8 x 8, 16 x 4, 32 x 2, 4 x 16 (neighbouring f-runs of the same
// tiles gathered together, each bucket's neighbouring runs stored together).
static inline void hook_tl_order(u32 F, u64, u32 *og, u32 *os) {
  const int v = tuning_variant();
  if (v == 296 || v == 297) *og = F, *os = 1;
  if (v == 316) *og = 8, *os = 8;
  if (v == 317) *og = 16, *os = 4;
  if (v == 318) *og = 32, *os = 2;
  if (v == 319) *og = 4, *os = 16;
}

// 21: the generic-length kernel for 8/16/32-B keys too; 70: one pass (the
// staged scatter) up to 2048 ranks whatever the two-pass threshold; 71: two
// passes at any nranks >= 2.  (r02's gather, producer/consumer and register
// scatters measured slower than the staged one and were removed in r03.)
template <class K>
static inline K hook_bucket_kind(K kind, bool fixed, u32 nranks) {
  const int v = tuning_variant();
  if (v == 70 && kind == K::kTwoPass && nranks <= kStagedMaxRanks) kind = K::kStaged;
  if (v == 71 && fixed && nranks >= 2) kind = K::kTwoPass;
  if (v == 21) kind = K::kGeneric;
  return kind;
}

// 83 / 87: owner ranking on 8 x 16 / 4 x 16 tiles, 85 / 89: ballots, at any
// nranks (85 also in the static tile order: hook_staged_launch)
template <class S>
static inline S hook_staged_shape(S shape) {
  const int v = tuning_variant();
  if (v == 83) shape = S::kOwner8x16;
  if (v == 87) shape = S::kOwner4x16;
  if (v == 85 || v == 89) shape = S::kBallot4x16;
  return shape;
}

// The r02-r05 two-pass form (290, 202, 264-272): tuning/bucket_two_pass_r05.h

// Shapes of the tile-local two passes (r06).  291: pass 2 in 4 x 8 @ 4;
// 292: pass 2 in 8 x 4 @ 2; 293: pass 1 in 16 waves (1024 threads) @ 1 on
// the product's tiles; 294: pass 1 on 8192-key tiles (16 x 8 @ 1;
// hook_tl_tile_shift), pass-2 runs twice as long; 295: 294 on the balanced
// digit split.  Pass 1 otherwise as the product's (8 x 8 @ 2 on 4096-key
// tiles for 8-B keys, 8 x 4 @ 2 on 2048-key tiles for 16-B keys).
template <int L, class Out>
static int hook_tl_shape(const BucketArgs &a, const TwoPassTL &tl, const Out &out, const BucketWs &w,
                         uint64_t *bucket_offsets, hipStream_t st, int dev) {
  const int v = tuning_variant();
  if constexpr (L <= 16) {
    constexpr int K1 = L == 8 ? 8 : 4;  // pass-1 keys per lane at the product's tile
    if constexpr (L == 16)
      if (v == 302) {  // pass 1 in 8 x 8 (4096-key tiles, hook_tl_tile_shift), pass 2 as 304
        if constexpr (Out::kPair8)
          return launch_tl<L, Out, 4, 4, 4, 8, 8, 2>(a, tl, out, w, bucket_offsets, st, dev);
        else
          return launch_tl<L, Out, 8, 8, 2, 8, 8, 2>(a, tl, out, w, bucket_offsets, st, dev);
      }
    if constexpr (L == 16)
      if (v == 304) {  // 16-B keys' pass 2 before r06's last shape change: arrays 8 x 8 @ 2, records 4 x 4 @ 4
        if constexpr (Out::kPair8)
          return launch_tl<L, Out, 4, 4, 4, 8, 4, 2>(a, tl, out, w, bucket_offsets, st, dev);
        else
          return launch_tl<L, Out, 8, 8, 2, 8, 4, 2>(a, tl, out, w, bucket_offsets, st, dev);
      }
    if (v == 298)  // timing probe: pass 2 reading contiguous rows (wrong outputs)
      return launch_tl<L, Out, 8, 8, 2, 8, K1, 2, 1>(a, tl, out, w, bucket_offsets, st, dev);
    if (v == 291) return launch_tl<L, Out, 4, 8, 4, 8, K1, 2>(a, tl, out, w, bucket_offsets, st, dev);
    if (v == 292) return launch_tl<L, Out, 8, 4, 2, 8, K1, 2>(a, tl, out, w, bucket_offsets, st, dev);
    if (v == 293) return launch_tl<L, Out, 8, 8, 2, 16, K1 / 2, 1>(a, tl, out, w, bucket_offsets, st, dev);
    if (v == 294 || v == 295 || v == 297)
      return launch_tl<L, Out, 8, 8, 2, 16, 8, 1>(a, tl, out, w, bucket_offsets, st, dev);
  }
  if (v == 320) {  // the product's shapes, pass 2 gathering with non-temporal loads (r06 before the switch)
    if constexpr (L == 8 && !Out::kPair8)
      return launch_tl<L, Out, 8, 8, 2, 8, 8, 2, 0, true>(a, tl, out, w, bucket_offsets, st, dev);
    else if constexpr (L == 8)
      return launch_tl<L, Out, 8, 4, 2, 8, 8, 2, 0, true>(a, tl, out, w, bucket_offsets, st, dev);
    else if constexpr (L == 32 && Out::kPair8)
      return launch_tl<L, Out, 4, 4, 4, 8, 4, 2, 0, false>(a, tl, out, w, bucket_offsets, st, dev);
    else
      return launch_tl<L, Out, 8, 4, 2, 8, 4, 2, 0, true>(a, tl, out, w, bucket_offsets, st, dev);
  }
  if (v == 322) {  // the product's shapes, pass 1 loading its keys with plain (temporal) loads
    constexpr bool NG = L == 32 && Out::kPair8;
    if constexpr (L == 8 && !Out::kPair8)
      return launch_tl<L, Out, 8, 8, 2, 8, 8, 2, 0, NG, false>(a, tl, out, w, bucket_offsets, st, dev);
    else if constexpr (L == 8)
      return launch_tl<L, Out, 8, 4, 2, 8, 8, 2, 0, NG, false>(a, tl, out, w, bucket_offsets, st, dev);
    else if constexpr (L == 32 && Out::kPair8)
      return launch_tl<L, Out, 4, 4, 4, 8, 4, 2, 0, NG, false>(a, tl, out, w, bucket_offsets, st, dev);
    else
      return launch_tl<L, Out, 8, 4, 2, 8, 4, 2, 0, NG, false>(a, tl, out, w, bucket_offsets, st, dev);
  }
  if constexpr (L == 8 && !Out::kPair8)
    if (v == 323)  // 8-B arrays' pass 2 storing in two phases (metadata, then the keys)
      return launch_tl<L, Out, 8, 8, 2, 8, 8, 2, 0, false, true, false>(a, tl, out, w, bucket_offsets, st, dev);
  if constexpr (L == 32 && Out::kPair8)
    if (v == 305)  // 32-B records' pass 2 in 8 x 4 @ 2 (the arrays' shape)
      return launch_tl<L, Out, 8, 4, 2, 8, 4, 2>(a, tl, out, w, bucket_offsets, st, dev);
  return kNoVariant;
}

// 85: the staged scatter in the static tile order (the r02 default before the
// per-XCD tickets)
template <class Out, class S>
static int hook_staged_launch(bool staged, size_t keysize, const BucketArgs &a, const Out &out, hipStream_t st,
                              int dev, S shape, u32 *tickets) {
  if (!staged) return kNoVariant;
  const int v = tuning_variant();
  if (v == 85)
    return keysize == 8    ? launch_staged<8, Out>(a, out, st, dev)
           : keysize == 16 ? launch_staged<16, Out>(a, out, st, dev)
                           : launch_staged<32, Out>(a, out, st, dev);
  if (v == 321) {  // the product's shapes, keys loaded non-temporally (r02-r06 before the switch)
    if (shape == S::kOwner8x16)
      return keysize == 8    ? launch_staged<8, Out, false, 8, 16, true, 2, true>(a, out, st, dev, tickets)
             : keysize == 16 ? launch_staged<16, Out, false, 8, 16, true, 2, true>(a, out, st, dev, tickets)
                             : launch_staged<32, Out, false, 8, 16, true, 2, true>(a, out, st, dev, tickets);
    if (shape == S::kOwner4x16)
      return keysize == 8    ? launch_staged<8, Out, false, kStW, kStKPL, true, 2, true>(a, out, st, dev, tickets)
             : keysize == 16 ? launch_staged<16, Out, false, kStW, kStKPL, true, 2, true>(a, out, st, dev, tickets)
                             : launch_staged<32, Out, false, kStW, kStKPL, true, 2, true>(a, out, st, dev, tickets);
    return keysize == 8    ? launch_staged<8, Out, false, kStW, kStKPL, true, 0, true>(a, out, st, dev, tickets)
           : keysize == 16 ? launch_staged<16, Out, false, kStW, kStKPL, true, 0, true>(a, out, st, dev, tickets)
                           : launch_staged<32, Out, false, kStW, kStKPL, true, 0, true>(a, out, st, dev, tickets);
  }
  return kNoVariant;
}

// 112: the r02 record store order (header halves first, {mbits, key} halves
// a round later)
template <class Go>
static int hook_records(const OutRec &out, Go &&go) {
  if (tuning_variant() != 112) return kNoVariant;
  return go(OutRecT<false>{out.rec, out.stride, out.hdr, out.ht_index, out.L});
}

}  // namespace pdht
