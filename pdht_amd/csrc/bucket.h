// bucket.h -- destination bucketing of a key batch.
//
// The bulk loader of bench/Meraculous/buildUFXhashBinary.h:83-112 hashes
// every key, counts keys per destination rank (my_heap_sizes[]) and later
// ships each key to its rank.  On the GPU that is a counting sort of the
// batch by rank = CityHash64(key) % nranks (libpdht/hash.c:26-29):
//
//   k_bucket_count   per 4096-key tile: LDS histogram of ranks
//                    -> counts[rank][tile]
//   k_bucket_scan    per rank: exclusive scan over tiles (in place) + total
//   k_bucket_base    exclusive scan of the totals -> bucket offsets
//   k_bucket_scatter per tile, one wave, key groups of 64 in index order:
//                    lanes with the same rank find each other with
//                    ceil(log2 nranks) ballots; the group leader advances the
//                    bucket's running position in LDS.  Keys, digests,
//                    PTE indices and original indices land at their bucket
//                    position.
//
// The order inside a bucket is the original key order (stable), so the
// output is deterministic.  Digests are recomputed in the scatter pass
// instead of being stored between passes (hashing costs less than a round
// trip of 8 B per key through HBM).
#pragma once

#include "kernels.h"

namespace pdht {

constexpr u64 kBucketTile = 4096;      // keys per tile
constexpr u32 kBucketMaxRanks = 8192;  // LDS bins (32 KiB)

__device__ __forceinline__ u64 packed_key_hash(const uint8_t *keys, u64 i, u32 L) {
  return city64(GlobalReader{keys + i * (u64)L}, (u64)L);
}

__global__ __launch_bounds__(kBlock) void k_bucket_count(const uint8_t *__restrict__ keys, u32 L,
                                                         u64 n, FastMod rk, u32 nranks,
                                                         u32 *__restrict__ counts, u64 ntiles) {
  extern __shared__ u32 hist[];  // nranks bins
  for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) hist[r] = 0;
    __syncthreads();
    const u64 k0 = t * kBucketTile;
    const u64 kend = (k0 + kBucketTile < n) ? k0 + kBucketTile : n;
    for (u64 i = k0 + threadIdx.x; i < kend; i += kBlock)
      atomicAdd(&hist[(u32)rk.mod(packed_key_hash(keys, i, L))], 1u);
    __syncthreads();
    for (u32 r = threadIdx.x; r < nranks; r += kBlock) counts[(u64)r * ntiles + t] = hist[r];
    __syncthreads();
  }
}

// One workgroup per rank: exclusive scan of counts[rank][0..ntiles) in place,
// the rank's total to totals[rank].
__global__ __launch_bounds__(kBlock) void k_bucket_scan(u32 *__restrict__ counts, u64 ntiles,
                                                        u64 *__restrict__ totals) {
  __shared__ u64 part[kBlock];
  u32 *row = counts + (u64)blockIdx.x * ntiles;
  const u64 per = (ntiles + kBlock - 1) / kBlock;
  const u64 lo = threadIdx.x * per;
  const u64 hi = (lo + per < ntiles) ? lo + per : ntiles;
  u64 s = 0;
  for (u64 t = lo; t < hi; ++t) s += row[t];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 run = 0;
    for (int k = 0; k < kBlock; ++k) {
      const u64 v = part[k];
      part[k] = run;
      run += v;
    }
    totals[blockIdx.x] = run;
  }
  __syncthreads();
  u64 run = part[threadIdx.x];
  for (u64 t = lo; t < hi; ++t) {
    const u32 v = row[t];
    row[t] = (u32)run;
    run += v;
  }
}

// Exclusive scan of the per-rank totals (one workgroup) -> bucket offsets.
__global__ __launch_bounds__(kBlock) void k_bucket_base(const u64 *__restrict__ totals, u32 nranks,
                                                        u64 *__restrict__ base,
                                                        u64 *__restrict__ offsets_out) {
  __shared__ u64 part[kBlock];
  const u32 per = (nranks + kBlock - 1) / kBlock;
  const u32 lo = threadIdx.x * per;
  const u32 hi = (lo + per < nranks) ? lo + per : nranks;
  u64 s = 0;
  for (u32 r = lo; r < hi; ++r) s += totals[r];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 run = 0;
    for (int k = 0; k < kBlock; ++k) {
      const u64 v = part[k];
      part[k] = run;
      run += v;
    }
    offsets_out[nranks] = run;
  }
  __syncthreads();
  u64 run = part[threadIdx.x];
  for (u32 r = lo; r < hi; ++r) {
    base[r] = run;
    offsets_out[r] = run;
    run += totals[r];
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

// One wave per workgroup; tile t's keys are visited in index order, 64 at a
// time.  run[r] = next free slot of bucket r for this tile (global position).
__global__ __launch_bounds__(64) void k_bucket_scatter(
    const uint8_t *__restrict__ keys, u32 L, u64 n, FastMod pt, FastMod rk, u32 nranks, u32 nbits,
    const u32 *__restrict__ counts, const u64 *__restrict__ base, u64 ntiles,
    uint8_t *__restrict__ keys_out, u64 *__restrict__ mbits_out, u32 *__restrict__ ptindex_out,
    u64 *__restrict__ index_out) {
  extern __shared__ u32 run[];  // nranks
  const u32 lane = threadIdx.x;
  const u64 below = (1ull << lane) - 1;
  for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
    for (u32 r = lane; r < nranks; r += 64) run[r] = (u32)(base[r] + counts[(u64)r * ntiles + t]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const u64 k0 = t * kBucketTile;
    const u64 kend = (k0 + kBucketTile < n) ? k0 + kBucketTile : n;
    for (u64 g = k0; g < kend; g += 64) {
      const u64 i = g + lane;
      const bool valid = i < kend;
      u64 h = 0;
      u32 r = 0;
      if (valid) {
        h = packed_key_hash(keys, i, L);
        r = (u32)rk.mod(h);
      }
      // lanes holding the same rank: AND of per-bit ballots
      u64 same = __ballot(valid);
      for (u32 b = 0; b < nbits; ++b) {
        const u64 m = __ballot(valid && ((r >> b) & 1u));
        same &= ((r >> b) & 1u) ? m : ~m;
      }
      const u32 ahead = (u32)__builtin_popcountll(same & below);
      const u32 size = (u32)__builtin_popcountll(same);
      u32 pos = 0;
      if (valid) pos = run[r] + ahead;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // every lane has read run[] before it moves
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (valid && ahead == 0) run[r] += size;
      if (valid) {
        mbits_out[pos] = h;
        if (ptindex_out) ptindex_out[pos] = (u32)pt.mod(h);
        if (index_out) index_out[pos] = i;
        if (keys_out) copy_row(keys_out + (u64)pos * L, keys + i * (u64)L, L);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
}

}  // namespace pdht
