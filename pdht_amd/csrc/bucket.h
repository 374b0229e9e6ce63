// bucket.h -- destination bucketing of a key batch.
//
// The bulk loader of bench/Meraculous/buildUFXhashBinary.h:83-112 hashes
// every key, counts keys per destination rank (my_heap_sizes[]) and later
// ships each key to its rank.  On the GPU that is a stable counting sort of
// the batch by rank = CityHash64(key) % nranks (libpdht/hash.c:26-29):
//
//   k_bucket_count*    per tile: LDS histogram of ranks -> counts[tile][rank]
//                      (tile-major, so every tile reads/writes one coalesced row)
//   k_bucket_colscan   per (64 ranks, chunk of 32 tiles): exclusive scan down
//                      the chunk in place, chunk sum -> chunks[chunk][rank]
//   k_bucket_chunkscan per rank: exclusive scan over chunks in place + total
//   k_bucket_base      exclusive scan of the totals -> bucket offsets
//   k_bucket_scatter*  per tile: the tile's first slot in bucket r is
//                      base[r] + chunks[c][r] + counts[t][r]; keys go to their
//                      slots in index order (stable).
//
// Scatter kernels:
//   _staged  (8/16/32-B keys below the two-pass threshold) sorts the tile by
//            bucket in LDS first and then writes each bucket's run of the
//            tile with consecutive lanes, so stores are coalesced runs, not 64
//            scattered 8-byte pieces per instruction; tiles are dealt to XCDs
//            in contiguous ranges so that the runs of neighbouring tiles meet
//            in the same L2 and leave it as whole lines.
//   _wg      (any other key length) re-reads keys from L2 in the scatter pass.
// From the two-pass threshold up, 8/16/32-B keys take the tile-local two
// passes (k_bucket_tl_*, below) instead of the count + scatter chain.
#pragma once

#include "kernels.h"

namespace pdht {

constexpr u64 kBucketMinTile = 2048;   // smallest tile of any scatter kernel (workspace sizing)
constexpr u32 kBucketMaxRanks = 8192;  // LDS bins (32 KiB)
constexpr u32 kBucketChunk = 32;       // tiles per colscan chunk
constexpr u32 kStagedMaxRanks = 2048;

__device__ __forceinline__ u64 packed_key_hash(const uint8_t *keys, u64 i, u32 L) {
  return city64(GlobalReader{keys + i * (u64)L}, (u64)L);
}

// First slot of tile t in bucket r (after the scans).
struct TileStarts {
  const u32 *counts;  // [ntiles][nranks], exclusive prefix within the chunk
  const u32 *chunks;  // [nchunks][nranks], exclusive prefix over chunks
  const u64 *base;    // [nranks], exclusive prefix over buckets
  u32 nranks;
  __device__ __forceinline__ u32 at(u32 r, u64 t) const {
    return (u32)(base[r] + chunks[(t / kBucketChunk) * nranks + r] + counts[t * nranks + r]);
  }
};

// XCD-contiguous tile order: workgroup b runs on XCD b % 8 (round-robin
// dispatch), so XCD x is given tiles [x*ntiles/8, (x+1)*ntiles/8) and its
// workgroups walk them in lockstep.
struct TileOrder {
  u64 t, end, step;
  __device__ __forceinline__ TileOrder(u64 ntiles) {
    if (gridDim.x >= 8 && gridDim.x % 8 == 0) {
      const u64 x = blockIdx.x % 8, per = gridDim.x / 8;
      t = x * ntiles / 8 + blockIdx.x / 8;
      end = (x + 1) * ntiles / 8;
      step = per;
    } else {
      t = blockIdx.x;
      end = ntiles;
      step = gridDim.x;
    }
  }
};

// ------------------------------------------------------------- counting ---
__global__ __launch_bounds__(kBlock) void k_bucket_count(const uint8_t *__restrict__ keys, u32 L,
                                                         u64 n, FastMod rk, u32 nranks,
                                                         u32 *__restrict__ counts, u64 ntiles,
                                                         u64 tile) {
  extern __shared__ u32 hist[];  // nranks bins
  for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) hist[r] = 0;
    __syncthreads();
    const u64 k0 = t * tile;
    const u64 kend = (k0 + tile < n) ? k0 + tile : n;
#pragma unroll 4
    for (u64 i = k0 + threadIdx.x; i < kend; i += kBlock)
      atomicAdd(&hist[(u32)rk.mod(packed_key_hash(keys, i, L))], 1u);
    __syncthreads();
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) counts[t * nranks + r] = hist[r];
    __syncthreads();
  }
}

// Non-temporal key loads (r04, late): the bucketing steps before this one
// left up to 256 MiB of write-back output lines in the Infinity Cache, and
// plain (allocating) loads made this kernel evict them -- 61.8 us per 16M
// 8-B keys against 26.9 with nt loads; the step -8.6 % (-4.6 % with the
// outputs rotated over four sets, profiles/r04/ab/ab_bucket*_count_nt.log).
#ifndef PDHT_COUNT_NT
#define PDHT_COUNT_NT true
#endif
// Packed 8/16/32-B keys: 128 B of keys per lane loaded before any is hashed.
template <int L>
__global__ __launch_bounds__(kBlock) void k_bucket_count_reg(const uint8_t *__restrict__ keys, u64 n,
                                                             FastMod rk, u32 nranks,
                                                             u32 *__restrict__ counts, u64 ntiles,
                                                             u64 tile) {
  constexpr int U = 128 / L;
  extern __shared__ u32 hist[];
  for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) hist[r] = 0;
    __syncthreads();
    const u64 k0 = t * tile;
    const u64 kend = (k0 + tile < n) ? k0 + tile : n;
    for (u64 i = k0 + threadIdx.x; i < kend; i += (u64)kBlock * U) {
      RegReader<L / 4> kr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) load_key_regs<L, PDHT_COUNT_NT>(keys, min(i + u * kBlock, n - 1), kr[u]);
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (i + u * kBlock < kend) atomicAdd(&hist[(u32)rk.mod(city64(kr[u], (u64)L))], 1u);
    }
    __syncthreads();
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) counts[t * nranks + r] = hist[r];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- scans ---
// One wave per (64 ranks, chunk): lane = rank.  The chunk's rows are loaded
// before any is written back (a load wait would also wait for the stores).
__global__ __launch_bounds__(64) void k_bucket_colscan(u32 *__restrict__ counts, u64 ntiles,
                                                       u32 nranks, u32 *__restrict__ chunks) {
  const u32 r = blockIdx.x * 64 + threadIdx.x;
  const u64 t0 = (u64)blockIdx.y * kBucketChunk;
  if (r >= nranks) return;
  u32 v[kBucketChunk];
#pragma unroll
  for (u32 j = 0; j < kBucketChunk; ++j) v[j] = t0 + j < ntiles ? counts[(t0 + j) * nranks + r] : 0;
  u32 run = 0;
#pragma unroll
  for (u32 j = 0; j < kBucketChunk; ++j) {
    if (t0 + j < ntiles) counts[(t0 + j) * nranks + r] = run;
    run += v[j];
  }
  chunks[(u64)blockIdx.y * nranks + r] = run;
}

// Exclusive scan over the chunk sums (in place) and the per-rank totals.
// Workgroup = 64 ranks (lane = rank) x kCsWaves waves; wave w scans its own
// contiguous share of the chunks, loading up to 16 rows before it stores any
// (a load wait also waits for older stores), then adds the sums of the waves
// before it: one or two memory round trips instead of nchunks / 16.
constexpr int kCsWaves = 16;
// Returns (last wave, r < nranks) rank r's total, else 0.
__device__ __forceinline__ u64 chunkscan_block(u32 blk, u32 *__restrict__ chunks, u64 nchunks, u32 nranks,
                                               u64 *__restrict__ totals) {
  __shared__ u32 wsum[kCsWaves][64];
  const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u32 r = blk * 64 + lane;
  const u64 per = (nchunks + kCsWaves - 1) / kCsWaves;
  const u64 c0 = min((u64)wave * per, nchunks), c1 = min(c0 + per, nchunks);
  constexpr u32 B = 16;
  u32 local = 0;  // this wave's chunk sum
  if (r < nranks)
    for (u64 c = c0; c < c1; c += B) {
      u32 v[B];
#pragma unroll
      for (u32 j = 0; j < B; ++j) v[j] = c + j < c1 ? chunks[(c + j) * nranks + r] : 0;
#pragma unroll
      for (u32 j = 0; j < B; ++j) local += v[j];
    }
  wsum[wave][lane] = local;
  __syncthreads();
  u64 run = 0;
  for (u32 w = 0; w < wave; ++w) run += wsum[w][lane];
  if (r < nranks) {
    for (u64 c = c0; c < c1; c += B) {
      u32 v[B];
#pragma unroll
      for (u32 j = 0; j < B; ++j) v[j] = c + j < c1 ? chunks[(c + j) * nranks + r] : 0;
#pragma unroll
      for (u32 j = 0; j < B; ++j) {
        if (c + j < c1) chunks[(c + j) * nranks + r] = (u32)run;
        run += v[j];
      }
    }
    if (wave == kCsWaves - 1) {
      totals[r] = run;
      return run;
    }
  }
  return 0;
}
__global__ __launch_bounds__(64 * kCsWaves) void k_bucket_chunkscan(u32 *__restrict__ chunks, u64 nchunks,
                                                                    u32 nranks, u64 *__restrict__ totals) {
  chunkscan_block(blockIdx.x, chunks, nchunks, nranks, totals);
}
// The tile-local two passes' chunk scan: it also turns each block's 64 rank
// totals into in-block exclusive prefixes inpre[r] and the block's sum
// bsum[blk] (n < 2^32: u32), so that pass 2 forms the bucket bases itself
// (k_bucket_tl_pass2: the prefix of bsum + inpre) and no k_bucket_base launch
// runs between the two.
__global__ __launch_bounds__(64 * kCsWaves) void k_bucket_chunkscan_tl(u32 *__restrict__ chunks, u64 nchunks,
                                                                       u32 nranks, u64 *__restrict__ totals,
                                                                       u32 *__restrict__ inpre,
                                                                       u32 *__restrict__ bsum) {
  const u32 t = (u32)chunkscan_block(blockIdx.x, chunks, nchunks, nranks, totals);
  const u32 lane = threadIdx.x & 63, r = blockIdx.x * 64 + lane;
  if ((threadIdx.x >> 6) == kCsWaves - 1) {
    u32 x = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(x, o);
      if (lane >= (u32)o) x += y;
    }
    if (r < nranks) inpre[r] = x - t;
    if (lane == 63) bsum[blockIdx.x] = x;
  }
}

// ------------------------------------------------------------- helpers ---
// Lanes whose r equals mine (AND of per-bit ballots; invalid lanes excluded).
__device__ __forceinline__ u64 same_bucket_lanes(bool valid, u32 r, u32 nbits) {
  u64 same = __ballot(valid);
  for (u32 b = 0; b < nbits; ++b) {
    const u64 m = __ballot(valid && ((r >> b) & 1u));
    same &= ((r >> b) & 1u) ? m : ~m;
  }
  return same;
}


// Exclusive scan of one value per thread over an NW-wave workgroup.
template <int NW, class T = u32>
__device__ __forceinline__ T block_exclusive_scan(T v, T *scratch /* NW words */) {
  const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T y = __shfl_up(x, d);
    if (lane >= (u32)d) x += y;
  }
  if (lane == 63) scratch[wave] = x;
  __syncthreads();
  T off = 0;
#pragma unroll
  for (u32 w = 0; w < (u32)NW; ++w)
    if (w < wave) off += scratch[w];
  __syncthreads();
  return off + x - v;
}

// Per-wave bucket run tables of the staged scatter: u32 counters, or (PACK)
// two u16 counters per u32 word -- a 4096-key tile never counts past 4096 in
// one bucket, so the low half never carries into the high one -- which
// halves the table's LDS (16 -> 8 KiB at 1024 ranks).  Wave w's counters
// start at w * stride (stride = nranks, rounded up to even when packed so a
// word never straddles two waves).
// Exclusive scan of the per-rank totals (one workgroup of kBaseThreads, each
// thread a run of consecutive ranks) -> bucket offsets; zeroes the scatter's
// per-XCD tile tickets.
constexpr u32 kBaseThreads = 1024;
__global__ __launch_bounds__(kBaseThreads) void k_bucket_base(const u64 *__restrict__ totals, u32 nranks,
                                                              u64 *__restrict__ base,
                                                              u64 *__restrict__ offsets_out,
                                                              u32 *__restrict__ tickets) {
  // the totals pass through LDS so that global loads and stores are
  // lane-contiguous (a thread's run of consecutive ranks would make every
  // wave instruction touch 64 lines)
  // 64 KiB of totals + scratch: over the 64 KiB a workgroup may allocate on
  // CDNA3, within gfx950's 160 KiB (the Makefile builds gfx950 only)
  __shared__ u64 tot[kBucketMaxRanks];
  __shared__ u64 scratch[kBaseThreads / 64];
  static_assert(sizeof(tot) + sizeof(scratch) <= 160 * 1024, "gfx950 LDS per workgroup");
  if (tickets && threadIdx.x < 16) tickets[threadIdx.x] = 0;  // per-XCD tile tickets of the scatter kernels
  for (u32 r = threadIdx.x; r < nranks; r += kBaseThreads) tot[r] = totals[r];
  __syncthreads();
  constexpr u32 kMaxPer = kBucketMaxRanks / kBaseThreads;
  const u32 per = (nranks + kBaseThreads - 1) / kBaseThreads;
  const u32 lo = min(threadIdx.x * per, nranks), hi = min(lo + per, nranks);
  u64 v[kMaxPer];
  u64 s = 0;
#pragma unroll
  for (u32 k = 0; k < kMaxPer; ++k) {
    v[k] = lo + k < hi ? tot[lo + k] : 0;
    s += v[k];
  }
  u64 run = block_exclusive_scan<kBaseThreads / 64, u64>(s, scratch);
#pragma unroll
  for (u32 k = 0; k < kMaxPer; ++k)
    if (lo + k < hi) {
      tot[lo + k] = run;  // each thread rewrites only its own run
      run += v[k];
    }
  if (hi == nranks && lo < hi) offsets_out[nranks] = run;
  if (nranks == 0 && threadIdx.x == 0) offsets_out[0] = 0;
  __syncthreads();
  for (u32 r = threadIdx.x; r < nranks; r += kBaseThreads) {
    base[r] = tot[r];
    offsets_out[r] = tot[r];
  }
}


template <bool PACK>
struct RunTab {
  u32 *t;
  u32 stride;
  __device__ __forceinline__ u32 words(u32 W) const { return PACK ? W * stride / 2 : W * stride; }
  __device__ __forceinline__ u32 get(u32 w, u32 r) const {
    const u32 i = w * stride + r;
    return PACK ? (t[i >> 1] >> (16 * (i & 1))) & 0xffffu : t[i];
  }
  // only the thread owning rank pair (r & ~1, r | 1) of every wave writes it
  __device__ __forceinline__ void set(u32 w, u32 r, u32 v) const {
    const u32 i = w * stride + r;
    if constexpr (PACK) {
      const u32 sh = 16 * (i & 1);
      t[i >> 1] = (t[i >> 1] & ~(0xffffu << sh)) | (v << sh);
    } else {
      t[i] = v;
    }
  }
  // returns the counter's old value
  __device__ __forceinline__ u32 add(u32 w, u32 r, u32 v) const {
    const u32 i = w * stride + r;
    if constexpr (PACK) return (atomicAdd(&t[i >> 1], v << (16 * (i & 1))) >> (16 * (i & 1))) & 0xffffu;
    else return atomicAdd(&t[i], v);
  }
};

// Stable tile-local slots of a wave's KPL groups of 64 keys.  Lanes with the
// same bucket find each other by ballots; each group's leader (its lowest
// lane) claims the bucket's next run of slots with one returning LDS atomic on
// the wave's own slot table.  A wave's LDS operations execute in issue order,
// so the KPL atomics go out back to back (group g sees the increments of the
// groups before it) and a single wait precedes the shuffles that hand every
// lane its leader's base: two LDS round trips per tile instead of two per
// group (the r01 form).
template <int KPL, class Tab>
__device__ __forceinline__ void rank_groups(const Tab &run, u32 wave, const u32 (&rr)[KPL], u32 q0, u32 tn,
                                            u32 nbits, u32 (&lp)[KPL]) {
  const u32 lane = threadIdx.x & 63;
  const u64 below = (1ull << lane) - 1;
  u32 al[KPL], base[KPL];  // al = ahead | leader lane << 8
#pragma unroll
  for (int g = 0; g < KPL; ++g) {
    const bool valid = q0 + g * 64 < tn;
    const u64 same = same_bucket_lanes(valid, rr[g], nbits);
    const u32 ahead = (u32)__builtin_popcountll(same & below);
    al[g] = ahead | ((same ? (u32)__builtin_ctzll(same) : 0u) << 8);
    base[g] = 0;
    if (valid && ahead == 0) base[g] = run.add(wave, rr[g], (u32)__builtin_popcountll(same));
  }
#pragma unroll
  for (int g = 0; g < KPL; ++g) lp[g] = (u32)__shfl((int)base[g], (int)(al[g] >> 8)) + (al[g] & 0xffu);
}

// rank_groups without the per-bit ballots: each lane of a group writes its
// lane id into an LDS owner table at its bucket, reads it back, and only the
// lanes that lost (their bucket is shared in the group) are resolved, one
// shared bucket per step (readlane + one ballot).  64 keys over 1024 buckets
// share ~2 buckets per group, against nbits = 10 ballots per group.  OB
// groups at a time, each with its own table (own: the wave's [OB][nranks]
// bytes), so one LDS round trip serves OB groups.
template <int KPL, int OB, class Tab>
__device__ __forceinline__ void rank_groups_owner(const Tab &run, u32 wave, const u32 (&rr)[KPL], u32 q0, u32 tn,
                                                  uint8_t *own, u32 nranks, u32 (&lp)[KPL]) {
  static_assert(KPL % OB == 0, "owner batches");
  const u32 lane = threadIdx.x & 63;
  const u64 below = (1ull << lane) - 1;
  u32 al[KPL], base[KPL];  // al = ahead | leader lane << 8
#pragma unroll
  for (int g0 = 0; g0 < KPL; g0 += OB) {
#pragma unroll
    for (int b = 0; b < OB; ++b)
      if (q0 + (g0 + b) * 64 < tn) own[b * nranks + rr[g0 + b]] = (uint8_t)lane;
    wave_lds_sync();
    u32 ow[OB];
#pragma unroll
    for (int b = 0; b < OB; ++b) ow[b] = q0 + (g0 + b) * 64 < tn ? own[b * nranks + rr[g0 + b]] : lane;
#pragma unroll
    for (int b = 0; b < OB; ++b) {
      const int g = g0 + b;
      const bool valid = q0 + g * 64 < tn;
      u64 same = valid ? 1ull << lane : 0ull;
      u64 losers = __ballot(valid && ow[b] != lane);
      while (losers) {  // wave-uniform
        const u32 src = (u32)__builtin_ctzll(losers);
        const u32 bk = (u32)__builtin_amdgcn_readlane((int)rr[g], (int)src);
        const bool eq = valid && rr[g] == bk;
        const u64 m = __ballot(eq);
        if (eq) same = m;
        losers &= ~m;
      }
      const u32 ahead = (u32)__builtin_popcountll(same & below);
      al[g] = ahead | ((same ? (u32)__builtin_ctzll(same) : 0u) << 8);
      base[g] = 0;
      if (valid && ahead == 0) base[g] = run.add(wave, rr[g], (u32)__builtin_popcountll(same));
    }
    wave_lds_sync();  // the next batch rewrites the tables
  }
#pragma unroll
  for (int g = 0; g < KPL; ++g) lp[g] = (u32)__shfl((int)base[g], (int)(al[g] >> 8)) + (al[g] & 0xffu);
}

template <int L>
__device__ __forceinline__ void store_key_row(uint8_t *dst, const RegReader<L / 4> &k) {
  if constexpr (L == 8) {
    typedef u32 u32x2 __attribute__((ext_vector_type(2)));
    *reinterpret_cast<u32x2 *>(dst) = u32x2{k.d[0], k.d[1]};
  } else {
#pragma unroll
    for (int j = 0; j < L / 16; ++j)
      reinterpret_cast<u32x4 *>(dst)[j] = u32x4{k.d[4 * j], k.d[4 * j + 1], k.d[4 * j + 2], k.d[4 * j + 3]};
  }
}

// Copy one L-byte key row (dword pieces when both rows are 4-B aligned).
__device__ __forceinline__ void copy_row(uint8_t *dst, const uint8_t *src, u32 L) {
  if ((((uintptr_t)dst | (uintptr_t)src | L) & 3) == 0) {
    const u32 *s = reinterpret_cast<const u32 *>(src);
    u32 *d = reinterpret_cast<u32 *>(dst);
    for (u32 j = 0; j < L / 4; ++j) d[j] = s[j];
  } else {
    for (u32 j = 0; j < L; ++j) dst[j] = src[j];
  }
}

// ------------------------------------------------------------- outputs ---
// Where a bucketed key goes; slot = its position in the bucketed batch.
// OutSoA (pdht_bucket_batch_dev): separate arrays, each but mbits optional.
struct OutSoA {
  static constexpr bool kPair8 = false;
  static constexpr bool kJoint = false;
  uint8_t *keys;
  u64 *mbits;
  u32 *ptindex;
  u32 *index;
  FastMod pt;
  u32 L;
  __device__ __forceinline__ void meta(u64 slot, u64 h, u64 i) const {
    mbits[slot] = h;
    if (ptindex) ptindex[slot] = (u32)pt.mod(h);
    if (index) index[slot] = (u32)i;
  }
  __device__ __forceinline__ bool has_keys() const { return keys != nullptr; }
  __device__ __forceinline__ void key8(u64 slot, int c, u64 v) const {  // key bytes [8c, 8c+8)
    *reinterpret_cast<u64 *>(keys + slot * L + 8 * c) = v;
  }
  template <int LL>
  __device__ __forceinline__ void key_row(u64 slot, const RegReader<LL / 4> &k) const {
    store_key_row<LL>(keys + slot * LL, k);
  }
  __device__ __forceinline__ void key_copy(u64 slot, const uint8_t *src) const {
    copy_row(keys + slot * L, src, L);
  }
};

// OutRec (pdht_bucket_records_dev): one wire record per key, laid out as the
// MPI variant's request message (message_t, libmpipdht/pdht.h:120-127) with
// the key as payload:
//   +0 u32 type  +4 u32 rank  +8 u32 ht_index  +12 u32 source index (the
//   struct's alignment padding)  +16 u64 mbits  +24 key[L], zero-padded to
//   the record stride 24 + round_up(L, 8).
// One record per key means one run per bucket and tile instead of four.
// JOINT (8-B keys): both 16-B halves of a record leave back to back, once the
// key has been staged, instead of the header half first and the {mbits, key}
// half a staging round later (by then the header halves' lines had often left
// L2 half-written: 2.1x the record bytes reached HBM, r02 PMC).
template <bool JOINT>
struct OutRecT {
  static constexpr bool kPair8 = true;  // 8-B keys: 32-B records written as two 16-B halves
  static constexpr bool kJoint = JOINT;
  uint8_t *rec;
  u64 stride;
  u64 hdr;  // type | rank << 32
  u32 ht_index;
  u32 L;
  __device__ __forceinline__ u64 *at(u64 slot) const { return reinterpret_cast<u64 *>(rec + slot * stride); }
  typedef u64 u64x2 __attribute__((ext_vector_type(2)));
  __device__ __forceinline__ void head(u64 slot, u64 i) const {  // +0 {type, rank, ht_index, index}
    *reinterpret_cast<u64x2 *>(at(slot)) = u64x2{hdr, ht_index | (i << 32)};
  }
  __device__ __forceinline__ void tail8(u64 slot, u64 h, u64 key) const {  // +16 {mbits, key}
    *reinterpret_cast<u64x2 *>(at(slot) + 2) = u64x2{h, key};
  }
  __device__ __forceinline__ void meta(u64 slot, u64 h, u64 i) const {
    u64 *p = at(slot);
    p[0] = hdr;
    p[1] = ht_index | (i << 32);
    p[2] = h;
  }
  __device__ __forceinline__ bool has_keys() const { return true; }
  __device__ __forceinline__ void key8(u64 slot, int c, u64 v) const { at(slot)[3 + c] = v; }
  template <int LL>
  __device__ __forceinline__ void key_row(u64 slot, const RegReader<LL / 4> &k) const {
    u64 *p = at(slot) + 3;
#pragma unroll
    for (int c = 0; c < LL / 8; ++c) p[c] = (u64)k.d[2 * c] | ((u64)k.d[2 * c + 1] << 32);
  }
  __device__ __forceinline__ void key_copy(u64 slot, const uint8_t *src) const {
    uint8_t *d = rec + slot * stride + 24;
    copy_row(d, src, L);
    for (u32 j = L; j < stride - 24; ++j) d[j] = 0;
  }
};
typedef OutRecT<true> OutRec;

// Phase D/E of the staged scatters: thread j writes staged entry j (digest in
// stage[j]) to slot delta[digit(h)] + j with original index idx(j); then the
// key rows, 8 bytes at a time through the same staging buffer (lp = each
// held key's staged slot).  Stores are runs of consecutive lanes.
template <int L, int KPL, u32 kB, class Out, class Dig, class Idx>
__device__ __forceinline__ void staged_store(u64 *stage, const u32 *delta, u32 tn, const RegReader<L / 4> (&kr)[KPL],
                                             const u32 (&lp)[KPL], u32 q0, const Dig &dig, const Idx &idx,
                                             const Out &out) {
  constexpr int kPer = KPL;  // entries per thread: a tile is kB x KPL keys
  u32 gp[kPer];
  if constexpr (Out::kPair8 && L == 8 && Out::kJoint) {
    // 8-B keys into 32-B records, both 16-B halves ({header, index} and
    // {mbits, key}) stored together once the keys are staged
    u64 hv[kPer];
    u32 si[kPer];
#pragma unroll
    for (int jj = 0; jj < kPer; ++jj) {
      const u32 j = min(jj * kB + threadIdx.x, tn - 1);
      hv[jj] = stage[j];
      gp[jj] = delta[dig(hv[jj], j)] + j;
      si[jj] = j;
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < KPL; ++g)
      if (q0 + g * 64 < tn) stage[lp[g]] = (u64)kr[g].d[0] | ((u64)kr[g].d[1] << 32);
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < kPer; ++jj) {
      const u32 j = jj * kB + threadIdx.x;
      if (j < tn) {
        out.head(gp[jj], idx(si[jj]));
        out.tail8(gp[jj], hv[jj], stage[j]);
      }
    }
    return;
  }
  if constexpr (Out::kPair8 && L == 8) {
    // 8-B keys into 32-B records: two 16-B stores per record, {header,
    // index} and {mbits, key}, half the store instructions of four 8-B ones
    u64 hv[kPer];
#pragma unroll
    for (int jj = 0; jj < kPer; ++jj) {
      const u32 j = min(jj * kB + threadIdx.x, tn - 1);
      hv[jj] = stage[j];
      gp[jj] = delta[dig(hv[jj], j)] + j;
      if (jj * kB + threadIdx.x < tn) out.head(gp[jj], idx(j));
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < KPL; ++g)
      if (q0 + g * 64 < tn) stage[lp[g]] = (u64)kr[g].d[0] | ((u64)kr[g].d[1] << 32);
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < kPer; ++jj) {
      const u32 j = jj * kB + threadIdx.x;
      if (j < tn) out.tail8(gp[jj], hv[jj], stage[j]);
    }
    return;
  }
#pragma unroll
  for (int jj = 0; jj < kPer; ++jj) {
    const u32 j = jj * kB + threadIdx.x;
    if (j < tn) {
      const u64 hv = stage[j];
      gp[jj] = delta[dig(hv, j)] + j;
      out.meta(gp[jj], hv, idx(j));
    }
  }
  if (out.has_keys()) {
#pragma unroll
    for (int c = 0; c < L / 8; ++c) {
      __syncthreads();
#pragma unroll
      for (int g = 0; g < KPL; ++g)
        if (q0 + g * 64 < tn) stage[lp[g]] = (u64)kr[g].d[2 * c] | ((u64)kr[g].d[2 * c + 1] << 32);
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < kPer; ++jj) {
        const u32 j = jj * kB + threadIdx.x;
        if (j < tn) out.key8(gp[jj], c, stage[j]);
      }
    }
  }
}

// ------------------------------------------------------ staged scatter ---
// Tile = 4 waves x 16 groups x 64 lanes = 4096 keys; wave w owns the
// contiguous quarter [w*1024, (w+1)*1024).
//   A: load + hash the wave's keys into VGPRs, count them into run[w][r];
//   B: tile-local bucket starts ls[r] (block scan); run[w][r] = ls[r] + keys of
//      bucket r in waves < w; delta[r] = (global start of the tile's run) - ls[r];
//   C: each key's tile-local sorted slot lp (ballot rank within the group,
//      leader advances run[w][r]); digest and tile offset staged at lp;
//   D: thread j takes staged entry j -> global slot delta[r] + j: mbits,
//      ptindex and index stores are runs of consecutive lanes;
//   E: the keys, 8 bytes at a time, through the same staging buffer.
// Shapes tried (r01): 8x16 and 8x8 tiles, 4x8, slots of D kept in LDS, tile
// starts prefetched with the keys -- all 8-45 % slower than this one on 16M x
// 8-B keys, 1024 ranks.
constexpr int kStW = 4, kStKPL = 16;
constexpr u32 kStTile = kStW * kStKPL * 64;
constexpr size_t kStagedStaticLds = 64;  // >= the staged kernels' static __shared__ bytes (<= 40)
constexpr size_t staged_lds_bytes(u32 nranks, int W = kStW, int KPL = kStKPL, bool PACK = false, int OB = 0) {
  return (size_t)W * KPL * 64 * 10 + (PACK ? (size_t)W * ((nranks + 1) & ~1u) * 2 : (size_t)W * nranks * 4) +
         (size_t)nranks * 4 + (size_t)W * OB * nranks;
}
// Per-entry branches around the stores measured 12 % faster than clamped
// branch-free stores (r01), although the branch-free form has no SGPR spills:
// the compiler then batches each array's stores, and the store order changes
// how the runs meet in L2.
// Work items [0, nitems) dealt to the 8 XCDs in contiguous ranges (workgroup
// b on XCD b % 8) and handed out inside each range in order, one ticket
// (vector atomic) per item: the items in flight on an XCD stay one
// contiguous window however its workgroups drift.  Needs gridDim.x % 8 == 0
// and zeroed tickets[8].
struct XcdTickets {
  u32 *tickets;
  u64 lo, hi;
  u32 x;
  __device__ __forceinline__ XcdTickets(u32 *tk, u64 nitems) : tickets(tk) {
    x = blockIdx.x % 8;
    lo = x * nitems / 8;
    hi = (x + 1) * nitems / 8;
  }
  // block-uniform; every thread must call it
  __device__ __forceinline__ u64 next(u32 *slot) const {
    if (threadIdx.x == 0) *slot = atomicAdd(&tickets[x], 1u);
    __syncthreads();
    return lo + *slot;
  }
};

// NTK: the keys loaded non-temporally.  Plain loads measured faster (r06,
// profiles/r06/ab/bucket_staged_key_loads.log: 1024 ranks 8-B keys -1.9 %,
// 8-B records -4.1 %, 16-B -1.9 %, 32-B -12 %).
// DYN: tiles handed out by a per-XCD ticket (one vector atomic per tile)
// instead of the static stride of TileOrder, so the tiles in flight on an XCD
// stay one contiguous window however the workgroups drift: the runs of one
// bucket from neighbouring tiles are written close in time and leave L2 as
// whole lines.
template <int L, class Out, int W = kStW, int KPL = kStKPL, bool PACK = false, bool DYN = false, int OB = 0,
          bool NTK = false>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(PACK ? 3 : (L == 8 || W == 8) ? 2 : 1)))
void k_bucket_scatter_staged(
    const uint8_t *__restrict__ keys, u64 n, FastMod rk, u32 nranks, u32 nbits, TileStarts ts, u64 ntiles,
    Out out, u32 *__restrict__ tickets = nullptr) {
  constexpr u32 kTile = W * KPL * 64, kB = W * 64;
  extern __shared__ u64 lds64[];
  u64 *stage = lds64;                                              // [kTile]
  uint16_t *sidx = reinterpret_cast<uint16_t *>(stage + kTile);  // [kTile]
  const RunTab<PACK> run{reinterpret_cast<u32 *>(sidx + kTile), PACK ? (nranks + 1) & ~1u : nranks};
  u32 *delta = run.t + run.words(W);                            // [nranks]
  __shared__ u32 scan_scratch[W];
  constexpr u32 kSub = KPL * 64;
  const u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // each thread owns a run of ranks for the scan (an even run when packed:
  // a word's two counters then have one owner)
  u32 per = (nranks + kB - 1) / kB;
  if (PACK) per = (per + 1) & ~1u;
  const u32 rb0 = min(threadIdx.x * per, nranks), rb1 = min(rb0 + per, nranks);
  __shared__ u32 s_ticket;
  const XcdTickets tk(tickets, ntiles);
  TileOrder o(ntiles);
  if constexpr (DYN) o.t = tk.next(&s_ticket), o.end = tk.hi;
  for (; o.t < o.end; o.t = DYN ? tk.next(&s_ticket) : o.t + o.step) {
    const u64 t = o.t;
    const u64 tbase = t * kTile;
    const u32 tn = (u32)min((u64)kTile, n - tbase);
    for (u32 j = threadIdx.x; j < run.words(W); j += kB) run.t[j] = 0;
    const u32 q0 = wave * kSub + lane;
    RegReader<L / 4> kr[KPL];
#pragma unroll
    for (int g = 0; g < KPL; ++g) load_key_regs<L, NTK>(keys, min(tbase + q0 + g * 64, n - 1), kr[g]);
    u64 h[KPL];
    u32 rr[KPL];
#pragma unroll
    for (int g = 0; g < KPL; ++g) {
      h[g] = city64(kr[g], (u64)L);
      rr[g] = (u32)rk.mod(h[g]);
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < KPL; ++g)
      if (q0 + g * 64 < tn) run.add(wave, rr[g], 1u);
    __syncthreads();
    u32 s = 0;
    for (u32 r = rb0; r < rb1; ++r)
#pragma unroll
      for (int w = 0; w < W; ++w) s += run.get(w, r);
    u32 acc = block_exclusive_scan<W>(s, scan_scratch);
    for (u32 r = rb0; r < rb1; ++r) {
      delta[r] = ts.at(r, t) - acc;
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const u32 v = run.get(w, r);
        run.set(w, r, acc);
        acc += v;
      }
    }
    __syncthreads();
    u32 lp[KPL];
    if constexpr (OB > 0)
      rank_groups_owner<KPL, OB>(run, wave, rr, q0, tn,
                                 reinterpret_cast<uint8_t *>(delta + nranks) + wave * OB * nranks, nranks, lp);
    else
      rank_groups<KPL>(run, wave, rr, q0, tn, nbits, lp);
    // (staging the bucket as well, u16 per slot, so that the store phase
    // reads it instead of reducing the digest again, measured slower: r02)
#pragma unroll
    for (int g = 0; g < KPL; ++g)
      if (q0 + g * 64 < tn) {
        stage[lp[g]] = h[g];
        sidx[lp[g]] = (uint16_t)(q0 + g * 64);
      }
    __syncthreads();
    staged_store<L, KPL, kB>(
        stage, delta, tn, kr, lp, q0, [&](u64 hv, u32) { return (u32)rk.mod(hv); },
        [&](u32 j) { return tbase + sidx[j]; }, out);
    __syncthreads();
  }
}

// ------------------------------------------------------------ two passes ---
// Sizes shared by the two-pass sort below (k_bucket_tl_*).  The r02-r05 form
// (a counting kernel ahead of pass 1, pass 1 writing global fine-bucket runs)
// lives in tuning/bucket_two_pass_r05.h, compiled into the A/B library only.
#ifndef PDHT_TP_SEG_KEYS
#define PDHT_TP_SEG_KEYS 3840
#endif
// Pass-2 segment: ~this many keys of one fine bucket.  A segment's length
// is a sum of per-chunk counts (binomial): at a mean of 4096 keys (r02-r05)
// half the segments held a few dozen keys more than one 4096-key sub-tile
// and ran a second, nearly empty sub-tile through the whole phase chain.
// 4096 - 4 sigma = 3840 keeps them in one (and in whole 2048 / 1024-key
// sub-tiles): 8-B keys at 8192 / 2048 ranks -10.6 / -6.7 %, 16-B keys at
// 4096 -4.5 %, 8-B records -1.6 %, 32-B keys within +-1.2 %
// (r05 form, profiles/r05/ab/bucket_pass2_segment_keys.log).
constexpr u32 kTpSegKeys = PDHT_TP_SEG_KEYS;
// F, C <= 256.  nranks <= 8192 = 2^13: the balanced split gives F = 2^7,
// C = 2^6; the fine-plus split of 8/16-B array outputs (late r03,
// pdht_bucket.hip) F = 2^8 -- at this bound -- and C = 2^5.  The launcher
// checks both before any two-pass launch.
constexpr u32 kTpMaxDigits = 256;

// Digit-run tables and scan of a tile sorted by a digit < ND <= kB (one thread
// per digit): on return run[w][d] = tile-local start of wave w's keys of
// digit d, and delta[d] = dst(d, tile-local start of d) - that start, i.e.
// the global slot of the tile's first digit-d key minus its local slot.
template <int W, class Dst>
__device__ __forceinline__ void digit_starts(const RunTab<false> &run, u32 ND, u32 *delta, u32 *tcount,
                                             u32 *scan_scratch, const Dst &dst) {
  const u32 d = threadIdx.x;
  u32 s = 0;
  if (d < ND)
#pragma unroll
    for (int w = 0; w < W; ++w) s += run.get(w, d);
  u32 acc = block_exclusive_scan<W>(s, scan_scratch);
  if (d < ND) {
    delta[d] = dst(d) - acc;
    if (tcount) tcount[d] = s;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const u32 v = run.get(w, d);
      run.set(w, d, acc);
      acc += v;
    }
  }
}

// ------------------------------------------ two-pass bucketing, tile-local ---
// One pass writes, per tile, one run per bucket into every output array: at
// 8192 ranks an 8192-key tile has runs of about one key, and the write path
// runs at ~1.3-3 TB/s on runs under 64 B against ~4.5 on >= 128-B runs
// (tools/scatter_probe.hip).  From two_pass_min_ranks() up (pdht_bucket.hip)
// the batch is sorted stably by the two digits of rank = c * F + f (F = 2^fbits
// fine buckets, C = ceil(nranks / F) coarse ones, both ~sqrt(nranks)), in
// passes that write runs of ~TILE / F and ~segment / C keys, at the price of an
// intermediate (key row + u16 index inside its tile):
//   pass 1 (k_bucket_tl_pass1): per tile of TILE keys (one sub-tile), sort by
//          the fine digit f in LDS and write the tile back IN PLACE -- rows
//          [t*TILE, (t+1)*TILE) of the intermediate, one contiguous store run
//          per wave instruction -- as key rows + the u16 index inside the
//          tile, plus the tile's F run starts (u16) startsF[t][f].  Per
//          count-chunk of ct tiles it also keeps the rank histogram (u16
//          pairs in LDS) -> chunkcnt[g][r], so nothing counts ahead of it;
//   scan:  chunkcnt down the chunks per rank, and in-block prefixes of the
//          rank totals (k_bucket_chunkscan_tl); pass 2 forms the bucket
//          bases from those (no k_bucket_base launch);
//   pass 2 (k_bucket_tl_pass2): per segment = (f, a range of count-chunks),
//          GATHER the f-runs of the segment's tiles (each run ~TILE / F
//          keys, contiguous) through an LDS row map, sort by the coarse
//          digit c and store every output at its final slot.  Original
//          index = tile row base | u16.
// Against the r02-r05 form (tuning/bucket_two_pass_r05.h: a counting kernel
// reads and hashes the batch ahead of a pass 1 that writes each tile's
// fine-bucket runs to global positions), one launch and one read of the keys
// fewer, pass-1 stores are whole lines, and the intermediate shrinks from
// L + 4 to L + 2 bytes per key.
constexpr u32 kTlMaxRuns = 512;  // tiles (= f-runs) per pass-2 segment
struct TwoPassTL {
  u32 fbits, F, C, cbits;
  u32 tshift;                 // log2 keys per pass-1 tile
  u32 ct;                     // tiles per count-chunk
  u64 n, ntiles, nchunks;
  u64 nsegf, nseg;            // segments per fine bucket; segments
  // segment order: blocks of og fine buckets x os segments each, the blocks
  // f-group-major (og = 1, os = nsegf: all of f, then f + 1)
  u32 og, os, nsgg;           // nsgg = ceil(nsegf / os)
  uint16_t *startsF;          // [ntiles][F] tile-local first row of fine bucket f
  u32 *chunkcnt;              // [nchunks][nranks] rank histogram of chunk g; after the scan its exclusive prefix
  u32 *inpre, *bsum;          // bucket bases = prefix of bsum[r / 64] + inpre[r] (k_bucket_chunkscan_tl)
  u64 *offsets;               // [nranks + 1] the caller's bucket offsets (pass 2 writes them)
  uint8_t *ikeys;             // [n][L] key rows, each tile sorted by f in place
  uint16_t *ilidx;            // [n] index of the row's key inside its tile
  __device__ __forceinline__ u32 tile_n(u64 t) const {
    const u64 b = t << tshift;
    return (u32)min((u64)1 << tshift, n - b);
  }
};

template <int W, int KPL>
constexpr size_t tl_pass1_lds_bytes(u32 nranks) {
  return (size_t)W * KPL * 64 * (8 + 2) + (size_t)((nranks + 1) / 2) * 4;
}
template <int W, int KPL>
constexpr size_t tl_pass2_lds_bytes() { return (size_t)W * KPL * 64 * (8 + 4); }

template <int L, int W, int KPL, int WPE, bool NTK = true>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_bucket_tl_pass1(const uint8_t *__restrict__ keys, FastMod rk, u32 nranks, TwoPassTL tp) {
  constexpr u32 kTile = W * KPL * 64, kB = W * 64, kSub = KPL * 64;
  static_assert(kTile <= 8192 && (kTile & (kTile - 1)) == 0, "u16 tile rows; power-of-two tiles");
  extern __shared__ u64 lds64[];
  u64 *stage = lds64;                                            // [kTile] key pieces in f order
  uint16_t *sidx = reinterpret_cast<uint16_t *>(stage + kTile);  // [kTile] tile-local index in f order
  u32 *hist = reinterpret_cast<u32 *>(sidx + kTile);            // [(nranks+1)/2] u16 pairs: the chunk's ranks
  __shared__ u32 runt[W * kTpMaxDigits];
  __shared__ u32 scan_scratch[W];
  const RunTab<false> run{runt, tp.F};
  const u32 fmask = tp.F - 1;
  const u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32 q0 = wave * kSub + lane;
  const u32 hw = (nranks + 1) / 2;
  const u64 n = tp.n;
  for (TileOrder o(tp.nchunks); o.t < o.end; o.t += o.step) {
    const u64 g = o.t;
    for (u32 j = threadIdx.x; j < hw; j += kB) hist[j] = 0;
    __syncthreads();  // (once per chunk) the rank counts below may start right after the hash
    const u64 t1 = min((g + 1) * tp.ct, tp.ntiles);
    for (u64 t = g * tp.ct; t < t1; ++t) {
      const u64 tbase = t * kTile;
      const u32 tn = (u32)min((u64)kTile, n - tbase);
      for (u32 j = threadIdx.x; j < W * tp.F; j += kB) runt[j] = 0;
      RegReader<L / 4> kr[KPL];
#pragma unroll
      for (int k = 0; k < KPL; ++k) load_key_regs<L, NTK>(keys, min(tbase + q0 + k * 64, n - 1), kr[k]);
      u32 ff[KPL];
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        const u32 r = (u32)rk.mod(city64(kr[k], (u64)L));
        ff[k] = r & fmask;
        if (q0 + k * 64 < tn) atomicAdd(&hist[r >> 1], 1u << (16 * (r & 1)));
      }
      __syncthreads();  // runt zeroed; the previous tile's stage / sidx reads done
#pragma unroll
      for (int k = 0; k < KPL; ++k)
        if (q0 + k * 64 < tn) run.add(wave, ff[k], 1u);
      __syncthreads();
      {  // the tile's f-run starts: out to startsF, and each wave's first slot of every f
        const u32 d = threadIdx.x;
        u32 s = 0;
        if (d < tp.F)
#pragma unroll
          for (int w = 0; w < W; ++w) s += run.get(w, d);
        u32 acc = block_exclusive_scan<W>(s, scan_scratch);
        if (d < tp.F) {
          tp.startsF[t * tp.F + d] = (uint16_t)acc;
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const u32 v = run.get(w, d);
            run.set(w, d, acc);
            acc += v;
          }
        }
      }
      __syncthreads();
      u32 lp[KPL];
      rank_groups<KPL>(run, wave, ff, q0, tn, tp.fbits, lp);
#pragma unroll
      for (int k = 0; k < KPL; ++k)
        if (q0 + k * 64 < tn) {
          stage[lp[k]] = (u64)kr[k].d[0] | ((u64)kr[k].d[1] << 32);
          sidx[lp[k]] = (uint16_t)(q0 + k * 64);
        }
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < KPL; ++jj) {
        const u32 j = jj * kB + threadIdx.x;
        if (j < tn) {
          *reinterpret_cast<u64 *>(tp.ikeys + (tbase + j) * L) = stage[j];
          tp.ilidx[tbase + j] = sidx[j];
        }
      }
#pragma unroll
      for (int c = 1; c < L / 8; ++c) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KPL; ++k)
          if (q0 + k * 64 < tn) stage[lp[k]] = (u64)kr[k].d[2 * c] | ((u64)kr[k].d[2 * c + 1] << 32);
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < KPL; ++jj) {
          const u32 j = jj * kB + threadIdx.x;
          if (j < tn) *reinterpret_cast<u64 *>(tp.ikeys + (tbase + j) * L + 8 * c) = stage[j];
        }
      }
    }
    __syncthreads();  // every atomic of the chunk is in
    for (u32 r = threadIdx.x; r < nranks; r += kB) tp.chunkcnt[g * nranks + r] = (hist[r >> 1] >> (16 * (r & 1))) & 0xffffu;
    __syncthreads();
  }
}

// PROBE (A/B timing only, wrong outputs): 1 = every sub-tile reads its rows
// contiguously from row o.t * 3840 instead of through the row map (what the
// gather costs).
// NTG: the gather's loads non-temporal.  Plain loads keep the lines a
// neighbouring f-run shares in L2 for the segment that reads it next:
// 8-B keys at 8192 / 2048 ranks -3.9 / -1.5 %, 16-B keys -5.7 %, 8-B
// records -4.4 %, 32-B keys equal; 32-B records +2.5 % and keep nt
// (profiles/r06/ab/bucket_tl_gather_temporal.log).
template <int L, class Out, int W, int KPL, int WPE, bool ONE = (L == 8 && !Out::kPair8), int PROBE = 0,
          bool NTG = (L == 32 && Out::kPair8)>
__global__ __launch_bounds__(W * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_bucket_tl_pass2(FastMod rk, u32 nranks, TwoPassTL tp, Out out) {
  static_assert(!ONE || (L == 8 && !Out::kPair8), "one store phase: 8-B keys into arrays");
  constexpr u32 kTile = W * KPL * 64, kB = W * 64, kSub = KPL * 64;
  constexpr u32 RP = (kTlMaxRuns + kB - 1) / kB;  // runs per thread
  extern __shared__ u64 lds64[];
  u64 *stage = lds64;                                  // [kTile] digests / key pieces
  u32 *sidx = reinterpret_cast<u32 *>(stage + kTile);  // [kTile] source rows of the sub-tile, then original indices
  __shared__ u32 runt[W * kTpMaxDigits];
  __shared__ u32 running[kTpMaxDigits];  // next final slot of bucket c*F + f
  __shared__ u32 delta[kTpMaxDigits];
  __shared__ u32 tcount[kTpMaxDigits];
  __shared__ u32 scan_scratch[W];
  __shared__ u32 s_len;
  __shared__ u32 bpre[kBucketMaxRanks / 64];  // first final slot of each block of 64 ranks
  static_assert(kBucketMaxRanks / 64 <= kB, "one thread per 64-rank block");
  {
    const u32 nblk = (nranks + 63) / 64;
    const u32 v = threadIdx.x < nblk ? tp.bsum[threadIdx.x] : 0u;
    const u32 e = block_exclusive_scan<W>(v, scan_scratch);
    if (threadIdx.x < nblk) bpre[threadIdx.x] = e;
    if (blockIdx.x == 0 && threadIdx.x == 0) tp.offsets[nranks] = (u64)tp.n;
    __syncthreads();
  }
  const RunTab<false> run{runt, tp.C};
  const u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32 q0 = wave * kSub + lane;
  const u32 fbits = tp.fbits;
  const u32 tmask = (1u << tp.tshift) - 1;
  auto coarse = [&](u64 h, u32) { return (u32)rk.mod(h) >> fbits; };
  for (TileOrder o(tp.nseg); o.t < o.end; o.t += o.step) {
    // the count-chunks split evenly over the nsegf segments of f
    const u32 ot = (u32)o.t, gs = tp.og * tp.os;
    const u32 blk = ot / gs, wi = ot - blk * gs;
    const u32 f = (blk / tp.nsgg) * tp.og + wi / tp.os;
    const u64 sg = (u64)(blk % tp.nsgg) * tp.os + wi % tp.os;
    if (sg >= tp.nsegf) continue;  // (the ragged last block of an f-group; uniform per workgroup)
    const u64 g0 = sg * tp.nchunks / tp.nsegf, g1 = (sg + 1) * tp.nchunks / tp.nsegf;
    const u64 ta = g0 * tp.ct, tb = min(g1 * tp.ct, tp.ntiles);
    // this thread's runs: tiles ta + threadIdx.x * RP + q (contiguous, so a
    // block scan of the per-thread sums orders them by tile)
    u32 src[RP], cnt[RP], pos[RP];
    u32 mine = 0;
#pragma unroll
    for (int q = 0; q < RP; ++q) {
      const u64 t = ta + (u64)threadIdx.x * RP + q;
      src[q] = cnt[q] = 0;
      if (t < tb) {
        const u32 s = tp.startsF[t * tp.F + f];
        const u32 e = f + 1 < tp.F ? tp.startsF[t * tp.F + f + 1] : tp.tile_n(t);
        src[q] = (u32)(t << tp.tshift) + s;
        cnt[q] = e - s;
      }
      pos[q] = mine;
      mine += cnt[q];
    }
    if (threadIdx.x < tp.C) {
      const u32 r = threadIdx.x * tp.F + f;
      if (r < nranks) {
        const u32 base = bpre[r >> 6] + tp.inpre[r];
        if (sg == 0) tp.offsets[r] = base;  // (every rank once: its fine bucket's first segment)
        running[threadIdx.x] = base + tp.chunkcnt[g0 * nranks + r];
      }
    }
    const u32 before = block_exclusive_scan<W>(mine, scan_scratch);
#pragma unroll
    for (int q = 0; q < RP; ++q) pos[q] += before;
    if (threadIdx.x == kB - 1) s_len = before + mine;
    __syncthreads();
    const u32 slen = s_len;
    for (u32 k0 = 0; k0 < slen; k0 += kTile) {
      const u32 tn = min(kTile, slen - k0);
      // the sub-tile's row map: sidx[p - k0] = intermediate row of segment key p
#pragma unroll
      for (int q = 0; q < RP; ++q) {
        const u32 lo = max(pos[q], k0), hi = min(pos[q] + cnt[q], k0 + tn);
        for (u32 p = lo; p < hi; ++p) sidx[p - k0] = src[q] + (p - pos[q]);
      }
      for (u32 j = threadIdx.x; j < W * tp.C; j += kB) runt[j] = 0;
      __syncthreads();
      RegReader<L / 4> kr[KPL];
      u32 ix[KPL];
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        const u32 row = PROBE == 1 ? (u32)((o.t * 3840 + k0 + min(q0 + k * 64, tn - 1)) % tp.n)
                                   : sidx[min(q0 + k * 64, tn - 1)];
        load_key_regs<L, NTG>(tp.ikeys, row, kr[k]);
        ix[k] = (row & ~tmask) | (u32)(NTG ? __builtin_nontemporal_load(tp.ilidx + row) : tp.ilidx[row]);
      }
      u64 h[ONE ? 1 : KPL];
      u32 cc[KPL];
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        const u64 hh = city64(kr[k], (u64)L);
        if constexpr (!ONE) h[k] = hh;
        cc[k] = coarse(hh, 0u);
      }
      __syncthreads();  // the row map is read
#pragma unroll
      for (int k = 0; k < KPL; ++k)
        if (q0 + k * 64 < tn) run.add(wave, cc[k], 1u);
      __syncthreads();
      digit_starts<W>(run, tp.C, delta, tcount, scan_scratch, [&](u32 c) { return running[c]; });
      __syncthreads();
      u32 lp[KPL];
      rank_groups<KPL>(run, wave, cc, q0, tn, tp.cbits, lp);
#pragma unroll
      for (int k = 0; k < KPL; ++k)
        if (q0 + k * 64 < tn) {
          if constexpr (ONE)
            stage[lp[k]] = (u64)kr[k].d[0] | ((u64)kr[k].d[1] << 32);
          else
            stage[lp[k]] = h[k];
          sidx[lp[k]] = ix[k];
        }
      __syncthreads();
      if constexpr (ONE) {
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

// ------------------------------------------------- generic-length scatter ---
// Tile = W waves x 32 groups; wave w owns a contiguous 2048-key sub-range.
// Counting pass hashes; the scatter pass hashes again from L2-resident keys
// (32 unrolled generic-length hashes per lane do not fit in VGPRs).
constexpr int kScatKPL = 32;
template <int W, class Out>
__global__ __launch_bounds__(W * 64) void k_bucket_scatter_wg(const uint8_t *__restrict__ keys, u32 L, u64 n,
                                                              FastMod rk, u32 nranks, u32 nbits,
                                                              TileStarts ts, u64 ntiles, Out out) {
  extern __shared__ u32 run[];  // [W][nranks]
  constexpr u64 kSub = (u64)kScatKPL * 64, kTile = W * kSub;
  const u32 wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u64 below = (1ull << lane) - 1;
  u32 *myrun = run + wave * nranks;
  for (TileOrder o(ntiles); o.t < o.end; o.t += o.step) {
    const u64 t = o.t;
    for (u32 j = threadIdx.x; j < W * nranks; j += W * 64) run[j] = 0;
    __syncthreads();
    const u64 k0 = t * kTile + wave * kSub + lane;
#pragma unroll 4
    for (int g = 0; g < kScatKPL; ++g) {
      const u64 i = k0 + (u64)g * 64;
      if (i < n) atomicAdd(&myrun[(u32)rk.mod(packed_key_hash(keys, i, L))], 1u);
    }
    __syncthreads();
    for (u32 r = threadIdx.x; r < nranks; r += W * 64) {
      u32 acc = ts.at(r, t);
#pragma unroll
      for (int w = 0; w < W; ++w) {
        const u32 v = run[w * nranks + r];
        run[w * nranks + r] = acc;
        acc += v;
      }
    }
    __syncthreads();
#pragma unroll 2
    for (int g = 0; g < kScatKPL; ++g) {
      const u64 i = k0 + (u64)g * 64;
      const bool valid = i < n;
      const u64 h = valid ? packed_key_hash(keys, i, L) : 0;
      const u32 r = (u32)rk.mod(h);
      const u64 same = same_bucket_lanes(valid, r, nbits);
      const u32 ahead = (u32)__builtin_popcountll(same & below);
      const u32 pos = valid ? myrun[r] + ahead : 0;
      wave_lds_sync();
      if (valid && ahead == 0) myrun[r] += (u32)__builtin_popcountll(same);
      if (valid) {
        out.meta(pos, h, i);
        if (out.has_keys()) out.key_copy(pos, keys + i * (u64)L);
      }
      wave_lds_sync();
    }
    __syncthreads();
  }
}

}  // namespace pdht
