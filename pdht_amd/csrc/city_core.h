// city_core.h -- CityHash v1.0.x arithmetic, written once for host and gfx950.
//
// Product code (not the oracle).  Every routine is __host__ __device__ and
// templated on a *reader*, the object that delivers key bytes.  Readers hand
// out SPANS: span<N>(o) returns bytes [o, o+N) of the key as a Words<N/4>
// register array (little-endian dwords) in ONE batched load, and all further
// word extraction uses compile-time offsets into that array.  CityHash only
// ever reads 8/16/32/40/64-byte windows at run-time positions (city.c:138-263,
// :276-400, :407-473), so the algorithm is written in those windows:
//   * HostReader    -- the scalar host API (memcpy)              city_host.hip
//   * RegReader<W>  -- fixed-length keys already in VGPRs; with a constant
//                      length every window folds to register renaming
//   * LdsReader     -- keys in an LDS window at arbitrary byte offsets:
//                      unaligned ds_read_b128/b64/b32 per window (r04; the
//                      r01-r03 dword runs + v_alignbyte_b32 are LdsReaderFunnel)
//   * GlobalReader  -- the same straight from global memory (keys that do not
//                      fit the LDS window)
// Behaviour follows /root/reference/libpdht/city.c; each routine cites the
// lines whose semantics it reproduces.  Parity: tests/ (oracle + golden).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <utility>

#define PDHT_HD __host__ __device__ __forceinline__

namespace pdht {

typedef uint64_t u64;
typedef uint32_t u32;

struct u128 {  // city.h:58-65: first = low 64 bits, second = high 64 bits
  u64 lo, hi;
};

// city.c:94-97, :103
constexpr u64 kK0 = 0xc3a5c85c97cb3127ULL;
constexpr u64 kK1 = 0xb492b66fbe98f273ULL;
constexpr u64 kK2 = 0x9ae16a3b2f90404fULL;
constexpr u64 kK3 = 0xc949d7c7509e6557ULL;
constexpr u64 kMul = 0x9ddfea08eb382d69ULL;

// ---------------------------------------------------------------- bit ops ---
// city.c:115-125.  rotr_nz needs 1 <= s <= 63 (every call site but the
// CRC-256 chunk, which keeps the shift-0 guard of Rotate() through rotr).
PDHT_HD u64 rotr_nz(u64 v, u32 s) { return (v >> s) | (v << (64 - s)); }
PDHT_HD u64 rotr(u64 v, u32 s) { return s == 0 ? v : rotr_nz(v, s); }
PDHT_HD u64 smix(u64 v) { return v ^ (v >> 47); }  // city.c:127-129

// u64 x u64, low 64 bits (every CityHash multiply goes through here).  The
// compiler emits v_mad_u64_u32 (lo x lo) + 2 v_mul_lo_u32 + v_add3_u32; r04
// tried three v_mad_u64_u32 instead (each cross term folded into the high
// half): 112 -> 85 multiply VALU on the 64-B Crc128 hash but +49 v_mov_b32 to
// zero-extend the addends, so more cycles (the `make exp` A/B build keeps the
// switch point).
PDHT_HD u64 mul64(u64 a, u64 b) { return a * b; }

// city.c:101-110 Hash128to64 == city.c:131-136 HashLen16(u, v)
PDHT_HD u64 mix16(u64 u, u64 v) {
  u64 a = smix(mul64((u ^ v), kMul));
  u64 b = smix(mul64((v ^ a), kMul));
  return mul64(b, kMul);
}

// ------------------------------------------------------------ key windows ---
// W dwords of key bytes in registers; offsets are compile-time constants.
template <int W>
struct Words {
  u32 d[W];
  PDHT_HD u64 w64(u32 b) const { return ((u64)d[(b >> 2) + 1] << 32) | d[b >> 2]; }
  PDHT_HD u32 w32(u32 b) const { return d[b >> 2]; }
};

// ---------------------------------------------------------------- readers ---
// A reader R exposes  template <int N> Words<N/4> span(off),  u32 w32(off)
// and u32 b8(off) (the <= 8-byte paths).
struct HostReader {
  const uint8_t *p;
  template <int N>
  PDHT_HD Words<N / 4> span(size_t o) const {
    Words<N / 4> w;
    memcpy(w.d, p + o, N);
    return w;
  }
  PDHT_HD u32 w32(size_t o) const {
    u32 r;
    memcpy(&r, p + o, 4);
    return r;
  }
  PDHT_HD u32 b8(size_t o) const { return p[o]; }
};

// Key bytes held in registers as W little-endian dwords (fixed-length
// kernels); offsets are constants after inlining.
template <int W>
struct RegReader {
  u32 d[W];
  PDHT_HD u32 dw(u32 b) const {  // dword at any byte offset
    const u32 q = b >> 2, r = b & 3;
    if (r == 0) return d[q];
    const u32 hi = (q + 1 < (u32)W) ? d[q + 1] : 0u;
    return (u32)((((u64)hi << 32) | d[q]) >> (8 * r));
  }
  template <int N>
  PDHT_HD Words<N / 4> span(u32 o) const {
    Words<N / 4> w;
#pragma unroll
    for (int j = 0; j < N / 4; ++j) w.d[j] = dw(o + 4 * j);
    return w;
  }
  PDHT_HD u32 w32(u32 o) const { return dw(o); }
  PDHT_HD u32 b8(u32 o) const { return dw(o) & 0xffu; }
};

// A view `off` bytes into another reader.  Holds a reference, never a copy:
// copying a RegReader's register array would force it into scratch memory.
template <class R>
struct Shifted {
  const R &r;
  u32 off;
  template <int N>
  PDHT_HD Words<N / 4> span(u32 o) const {
    return r.template span<N>(o + off);
  }
  PDHT_HD u32 w32(u32 o) const { return r.w32(o + off); }
  PDHT_HD u32 b8(u32 o) const { return r.b8(o + off); }
};

// Zero-padded view used by CityHashCrc256Short (city.c:476-481): bytes past
// `len` of the underlying key read as 0.
template <class R>
struct PadReader {
  const R &r;
  u32 len;
  template <int N>
  PDHT_HD Words<N / 4> span(u32 o) const {
    if (o + N <= len) return r.template span<N>(o);
    Words<N / 4> w;
#pragma unroll
    for (int j = 0; j < N / 4; ++j) {
      u32 v = 0;
      for (u32 i = 0; i < 4; ++i)
        if (o + 4 * j + i < len) v |= r.b8(o + 4 * j + i) << (8 * i);
      w.d[j] = v;
    }
    return w;
  }
  PDHT_HD u32 w32(u32 o) const { return span<4>(o).d[0]; }
  PDHT_HD u32 b8(u32 o) const { return o < len ? r.b8(o) : 0u; }
};

template <class R>
PDHT_HD u64 fetch64(const R &s, u32 o) {
  return s.template span<8>(o).w64(0);
}

// ----------------------------------------------------------- CityHash64 ---
// city.c:138-157
template <class R>
PDHT_HD u64 len0to16(const R &s, u64 len) {
  const u32 n = (u32)len;
  if (len > 8) {
    const u64 a = fetch64(s, 0);
    const u64 b = fetch64(s, n - 8);
    return mix16(a, rotr_nz(b + len, n)) ^ b;
  }
  if (len >= 4) {
    const u64 a = s.w32(0);
    return mix16(len + (a << 3), (u64)s.w32(n - 4));
  }
  if (len > 0) {
    const u32 a = s.b8(0), b = s.b8(n >> 1), c = s.b8(n - 1);
    const u32 y = a + (b << 8);
    const u32 z = n + (c << 2);
    return mul64(smix((u64)mul64(y, kK2) ^ (u64)mul64(z, kK3)), kK2);
  }
  return kK2;
}

// city.c:161-168 (head = bytes [0,16), tail = bytes [len-16, len))
template <class R>
PDHT_HD u64 len17to32(const R &s, u64 len) {
  const Words<4> h = s.template span<16>(0);
  const Words<4> t = s.template span<16>((u32)len - 16);
  const u64 a = mul64(h.w64(0), kK1);
  const u64 b = h.w64(8);
  const u64 c = mul64(t.w64(8), kK2);
  const u64 d = mul64(t.w64(0), kK0);
  return mix16(rotr_nz(a - b, 43) + rotr_nz(c, 30) + d,
               a + rotr_nz(b ^ kK3, 20) - c + len);
}

// city.c:173-198 -- WeakHashLen32WithSeeds
PDHT_HD u128 weak32(u64 w, u64 x, u64 y, u64 z, u64 a, u64 b) {
  a += w;
  b = rotr_nz(b + a + z, 21);
  const u64 c = a;
  a += x;
  a += y;
  b += rotr_nz(a, 44);
  return u128{a + z, b + c};
}
template <int W>
PDHT_HD u128 weak32_at(const Words<W> &c, u32 o, u64 a, u64 b) {
  return weak32(c.w64(o), c.w64(o + 8), c.w64(o + 16), c.w64(o + 24), a, b);
}

// city.c:201-222 -- 33..64 bytes (head = [0,32), tail = [len-32, len))
template <class R>
PDHT_HD u64 len33to64(const R &s, u64 len) {
  const Words<8> h = s.template span<32>(0);
  const Words<8> t = s.template span<32>((u32)len - 32);
  u64 z = h.w64(24);
  u64 a = h.w64(0) + mul64((len + t.w64(16)), kK0);
  u64 b = rotr_nz(a + z, 52);
  u64 c = rotr_nz(a, 37);
  a += h.w64(8);
  c += rotr_nz(a, 7);
  a += h.w64(16);
  const u64 vf = a + z;
  const u64 vs = b + rotr_nz(a, 31) + c;
  a = h.w64(16) + t.w64(0);
  z = t.w64(24);
  b = rotr_nz(a + z, 52);
  c = rotr_nz(a, 37);
  a += t.w64(8);
  c += rotr_nz(a, 7);
  a += t.w64(16);
  const u64 wf = a + z;
  const u64 ws = b + rotr_nz(a, 31) + c;
  const u64 r = smix(mul64((vf + ws), kK2) + mul64((wf + vs), kK0));
  return mul64(smix(mul64(r, kK0) + vs), kK2);
}

// 56 bytes of running state of the >64-byte loops (city.c:236-260, :315-350)
struct LongState {
  u64 x, y, z;
  u128 v, w;
};

// One 64-byte round over chunk c, including the z<->x exchange
// (city.c:248-257 == :329-338 == :340-349).
PDHT_HD void round64(LongState &st, const Words<16> &c) {
  u64 x = mul64(rotr_nz(st.x + st.y + st.v.lo + c.w64(8), 37), kK1);
  u64 y = mul64(rotr_nz(st.y + st.v.hi + c.w64(48), 42), kK1);
  x ^= st.w.hi;
  y += st.v.lo + c.w64(40);
  const u64 z = mul64(rotr_nz(st.z + st.w.lo, 33), kK1);
  const u128 v = weak32_at(c, 0, mul64(st.v.hi, kK1), x + st.w.lo);
  const u128 w = weak32_at(c, 32, z + st.w.hi, y + c.w64(16));
  st.v = v;
  st.w = w;
  st.x = z;
  st.y = y;
  st.z = x;
}

// Tail-first initialisation from the last 64 bytes t (city.c:237-243),
// except the "+ Fetch64(s)" of x, which the caller adds (the chunk-streaming
// kernel only has the first chunk one step later).
PDHT_HD void city64_long_init(const Words<16> &t, u64 len, LongState &st) {
  const u64 x = t.w64(24);  // s+len-40
  st.y = t.w64(48) + t.w64(8);
  st.z = mix16(t.w64(16) + len, t.w64(40));
  st.v = weak32_at(t, 0, len, st.z);
  st.w = weak32_at(t, 32, st.y + kK1, x);
  st.x = mul64(x, kK1);
}

// city.c:261-262
PDHT_HD u64 city64_long_final(const LongState &st) {
  return mix16(mix16(st.v.lo, st.w.lo) + mul64(smix(st.y), kK1) + st.z, mix16(st.v.hi, st.w.hi) + st.x);
}

// Readers that set kPairs read the >64-byte loop two rounds (128 B, a whole
// line of a 128-B aligned key) per span.
template <class R, class = void>
struct ReaderPairs {
  static constexpr bool value = false;
};
template <class R>
struct ReaderPairs<R, decltype((void)R::kPairs)> {
  static constexpr bool value = R::kPairs;
};
template <int W, int O, int N>
PDHT_HD Words<N> sub_words(const Words<W> &q) {
  Words<N> w;
#pragma unroll
  for (int j = 0; j < N; ++j) w.d[j] = q.d[O + j];
  return w;
}

// city.c:224-263
template <class R>
PDHT_HD u64 city64(const R &s, u64 len) {
  if (len <= 32) return len <= 16 ? len0to16(s, len) : len17to32(s, len);
  if (len <= 64) return len33to64(s, len);
  const u32 n = (u32)len;
  LongState st;
  city64_long_init(s.template span<64>(n - 64), len, st);
  st.x += fetch64(s, 0);
  const u32 rounds = (u32)((len - 1) >> 6);
  u32 r = 0;
  if constexpr (ReaderPairs<R>::value) {
    for (; r + 1 < rounds; r += 2) {
      const Words<32> q = s.template span<128>(r << 6);
      round64(st, sub_words<32, 0, 16>(q));
      round64(st, sub_words<32, 16, 16>(q));
    }
  }
  for (; r < rounds; ++r) round64(st, s.template span<64>(r << 6));
  return city64_long_final(st);
}

// city.c:265-272
template <class R>
PDHT_HD u64 city64_seeds(const R &s, u64 len, u64 seed0, u64 seed1) {
  return mix16(city64(s, len) - seed0, seed1);
}

// ----------------------------------------------------------- CityHash128 ---
// city.c:276-308 (CityMurmur), len < 128
template <class R>
PDHT_HD u128 murmur128(const R &s, u64 len, u128 seed) {
  u64 a = seed.lo, b = seed.hi, c, d;
  if (len <= 16) {
    a = mul64(smix(mul64(a, kK1)), kK1);
    c = mul64(b, kK1) + len0to16(s, len);
    d = smix(a + (len >= 8 ? fetch64(s, 0) : c));
  } else {
    const u32 n = (u32)len;
    const Words<4> t = s.template span<16>(n - 16);
    c = mix16(t.w64(8) + kK1, a);
    d = mix16(b + len, c + t.w64(0));
    a += d;
    const u32 steps = (n - 1) >> 4;  // signed l = len-16; do..while (l > 0)
    for (u32 k = 0; k < steps; ++k) {
      const Words<4> q = s.template span<16>(16 * k);
      a ^= mul64(smix(mul64(q.w64(0), kK1)), kK1);
      a *= kK1;
      b ^= a;
      c ^= mul64(smix(mul64(q.w64(8), kK1)), kK1);
      c *= kK1;
      d ^= c;
    }
  }
  a = mix16(a, c);
  b = mix16(d, b);
  return u128{a ^ b, mix16(b, a)};
}

// city.c:369-375
PDHT_HD u128 city128_final(u64 x, u64 y, u64 z, u128 v, u128 w) {
  x = mix16(x, v.lo);
  y = mix16(y + z, w.lo);
  return u128{mix16(x + v.hi, w.hi) + y, mix16(x + w.hi, y + v.hi)};
}

// city.c:354-366 tail (after the 128-byte loop) and finalisation
template <class R>
PDHT_HD u128 city128_finish(const R &s, u32 o, u64 rem, const LongState &st) {
  u64 x = st.x, y = st.y, z = st.z;
  u128 v = st.v, w = st.w;
  x += mul64(rotr_nz(v.lo + z, 49), kK0);
  z += mul64(rotr_nz(w.lo, 37), kK0);
  // city.c:357-365: up to 4 chunks of 32 B from the end.  All four are
  // loaded before the first is used (one memory round trip, not four); the
  // unused ones stay inside the key, since o >= 128 when rem > 0.
  if (rem == 0) return city128_final(x, y, z, v, w);
  Words<8> p[4];
  const u32 end = o + (u32)rem;
#pragma unroll
  for (int k = 0; k < 4; ++k) p[k] = s.template span<32>(end - 32 * (k + 1));
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (32u * k >= (u32)rem) break;
    y = mul64(rotr_nz(x + y, 42), kK0) + v.hi;
    w.lo += p[k].w64(16);
    x = mul64(x, kK0) + w.lo;
    z += w.hi + p[k].w64(0);
    w.hi += v.lo;
    v = weak32_at(p[k], 0, v.lo + z, v.hi);
  }
  return city128_final(x, y, z, v, w);
}

// city.c:310-376 for len >= 128 on kPairs readers (keys whose 128-B lines
// the reader fetches whole): each 128-byte iteration is one line load.
// (CityHash128 hashes from byte 16 on, so its iterations straddle lines; a
// form that loaded whole lines and carried the 112-B remainder in registers
// measured 5 % slower than plain 64-B spans, r02, and was removed.)
template <class R>
PDHT_HD u128 city128_seed_lines(const R &b, u64 len, u128 seed) {
  LongState st;
  st.x = seed.lo;
  st.y = seed.hi;
  st.z = mul64(len, kK1);
  Words<32> l0 = b.template span<128>(0);  // len >= 128
  st.v.lo = mul64(rotr_nz(st.y ^ kK1, 49), kK1) + l0.w64(0);
  st.v.hi = mul64(rotr_nz(st.v.lo, 42), kK1) + l0.w64(8);
  st.w.lo = mul64(rotr_nz(st.y + st.z, 35), kK1) + st.x;
  st.w.hi = mul64(rotr_nz(st.x + l0.w64(88), 53), kK1);
  u32 o = 0;
  u64 rem = len;
  do {
    if (o) l0 = b.template span<128>(o);
    round64(st, sub_words<32, 0, 16>(l0));
    round64(st, sub_words<32, 16, 16>(l0));
    o += 128;
    rem -= 128;
  } while (rem >= 128);
  return city128_finish(b, o, rem, st);
}

// city.c:310-376
template <class R>
PDHT_HD u128 city128_seed(const R &s, u64 len, u128 seed) {
  if (len < 128) return murmur128(s, len, seed);
  if constexpr (ReaderPairs<R>::value) return city128_seed_lines(s, len, seed);
  LongState st;
  st.x = seed.lo;
  st.y = seed.hi;
  st.z = mul64(len, kK1);
  {
    const Words<4> h = s.template span<16>(0);
    st.v.lo = mul64(rotr_nz(st.y ^ kK1, 49), kK1) + h.w64(0);
    st.v.hi = mul64(rotr_nz(st.v.lo, 42), kK1) + h.w64(8);
  }
  st.w.lo = mul64(rotr_nz(st.y + st.z, 35), kK1) + st.x;
  st.w.hi = mul64(rotr_nz(st.x + fetch64(s, 88), 53), kK1);
  u32 o = 0;
  u64 rem = len;
  do {
    round64(st, s.template span<64>(o));
    round64(st, s.template span<64>(o + 64));
    o += 128;
    rem -= 128;
  } while (rem >= 128);
  return city128_finish(s, o, rem, st);
}

// city.c:378-400
template <class R>
PDHT_HD u128 city128(const R &s, u64 len) {
  if (len >= 16) {
    const Words<4> h = s.template span<16>(0);
    return city128_seed(Shifted<R>{s, 16}, len - 16, u128{h.w64(0) ^ kK3, h.w64(8)});
  }
  if (len >= 8) {
    // WithSeed(NULL, 0, seed): no key byte is read after the seed is formed
    const u128 seed{fetch64(s, 0) ^ (mul64(len, kK0)), fetch64(s, (u32)len - 8) ^ kK1};
    return murmur128(s, 0, seed);
  }
  return murmur128(s, len, u128{kK0, kK1});
}

// ------------------------------------------------- CRC-32C (long CRC path) ---
// _mm_crc32_u64 (city.c:435-439): reflected CRC-32C (poly 0x82F63B78) over the
// 8 little-endian bytes of v, from the low 32 bits of crc, no inversion.
// Slicing-by-8 tables, built at compile time.
struct Crc32cTables {
  u32 t[8][256];
};
constexpr Crc32cTables make_crc32c_tables() {
  Crc32cTables T{};
  for (u32 i = 0; i < 256; ++i) {
    u32 c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    T.t[0][i] = c;
  }
  for (u32 i = 0; i < 256; ++i)
    for (int s = 1; s < 8; ++s) T.t[s][i] = (T.t[s - 1][i] >> 8) ^ T.t[0][T.t[s - 1][i] & 0xff];
  return T;
}

__device__ __constant__ const Crc32cTables kCrcDev = make_crc32c_tables();
static constexpr Crc32cTables kCrcHost = make_crc32c_tables();

// Slicing-by-8 over the compile-time tables: one lookup per byte.
PDHT_HD u32 crc32c_slice8(const Crc32cTables &T, u64 x) {
  return T.t[7][x & 0xff] ^ T.t[6][(x >> 8) & 0xff] ^ T.t[5][(x >> 16) & 0xff] ^ T.t[4][(x >> 24) & 0xff] ^
         T.t[3][(x >> 32) & 0xff] ^ T.t[2][(x >> 40) & 0xff] ^ T.t[1][(x >> 48) & 0xff] ^ T.t[0][x >> 56];
}

// The same map in 6-bit slices: CRC-32C of a 64-bit word with a zero initial
// CRC is GF(2)-linear in the word, so it is the XOR of the contributions of
// its 11 six-bit fields (10 x 6 bits + the top 4), each a 64-entry table:
// T6[k][f] = crc(f << 6k).  11 lookups instead of 8, but 64 lanes reading one
// 64-word table at random indices never conflict in LDS (identical indices
// broadcast; slicing-by-8's 256-entry tables conflicted 4.3x,
// profiles/r01/sq_long); r02's 5-bit form took 13 lookups per word.
struct Crc32c6Tables {
  u32 t[11][64];
};
constexpr Crc32c6Tables make_crc32c6_tables() {
  Crc32c6Tables F{};
  const Crc32cTables S = make_crc32c_tables();
  for (u32 k = 0; k < 11; ++k)
    for (u32 f = 0; f < 64; ++f) {
      const u64 x = k < 10 || f < 16 ? (u64)f << (6 * k) : 0;
      F.t[k][f] = S.t[7][x & 0xff] ^ S.t[6][(x >> 8) & 0xff] ^ S.t[5][(x >> 16) & 0xff] ^
                  S.t[4][(x >> 24) & 0xff] ^ S.t[3][(x >> 32) & 0xff] ^ S.t[2][(x >> 40) & 0xff] ^
                  S.t[1][(x >> 48) & 0xff] ^ S.t[0][x >> 56];
    }
  return F;
}
__device__ __constant__ const Crc32c6Tables kCrc6Dev = make_crc32c6_tables();

// Where the tables live: CrcConstTab = the compile-time slicing-by-8 tables
// (host; device constant memory); kernels.h adds the LDS copy of the 6-bit
// tables for the GPU's long-key path.
struct CrcConstTab {
  PDHT_HD u32 crc64(u64 x) const {
#if defined(__HIP_DEVICE_COMPILE__)
    return crc32c_slice8(kCrcDev, x);
#else
    return crc32c_slice8(kCrcHost, x);
#endif
  }
};

template <class Tab = CrcConstTab>
PDHT_HD u64 crc32c_u64(u64 crc, u64 v, const Tab &T = Tab{}) {
  return T.crc64(v ^ (u32)crc);
}

// city.c:407-473 (CityHashCrc256Long), len >= 240.  Each 240-byte block is
// fetched as ONE span (60 dwords; dwordx4 loads for 16-B aligned keys) and
// its six 40-byte CHUNKs work on compile-time offsets into it: one memory
// round trip per block instead of one per chunk (the long-key kernels read
// each lane's key straight from global memory, and waited on every chunk).
// Readers that set kLines read the 240-B blocks of CityHashCrc256Long as
// whole 128-B lines of the key: block k's load runs on to the end of the line
// its last byte lies in, and that line's remainder (0..112 B, 16 B more per
// block, period 8 blocks) is carried in registers into block k+1, so no line
// is fetched twice (the plain form reads lines 1, 3, 5, 7 of a 1 KiB key in
// two blocks: 1.5x the bytes).
template <class R, class = void>
struct ReaderLines {
  static constexpr bool value = false;
};
template <class R>
struct ReaderLines<R, decltype((void)R::kLines)> {
  static constexpr bool value = R::kLines;
};
// Block at key offset o (o = 240k, C = 16 * (k mod 8) bytes of it carried):
// loads [o + C, o + C + LB), LB = 256 (128 when C = 112).
template <int C, class R>
PDHT_HD void crc_block_lines(const R &s, u32 o, Words<28> &carry, Words<60> &q) {
  constexpr int CD = C / 4, LB = C == 112 ? 128 : 256, USE = (240 - C) / 4, NC = (LB - (240 - C)) / 4;
  const Words<LB / 4> ld = s.template span<LB>(o + C);
#pragma unroll
  for (int i = 0; i < 60; ++i) q.d[i] = i < CD ? carry.d[i < CD ? i : 0] : ld.d[i < CD ? 0 : i - CD];
#pragma unroll
  for (int i = 0; i < NC; ++i) carry.d[i] = ld.d[USE + i];
}
template <class R>
PDHT_HD void crc_block_lines_ph(const R &s, u32 o, u32 ph, Words<28> &carry, Words<60> &q) {
  switch (ph) {
    case 0: crc_block_lines<0>(s, o, carry, q); break;
    case 1: crc_block_lines<16>(s, o, carry, q); break;
    case 2: crc_block_lines<32>(s, o, carry, q); break;
    case 3: crc_block_lines<48>(s, o, carry, q); break;
    case 4: crc_block_lines<64>(s, o, carry, q); break;
    case 5: crc_block_lines<80>(s, o, carry, q); break;
    case 6: crc_block_lines<96>(s, o, carry, q); break;
    default: crc_block_lines<112>(s, o, carry, q); break;
  }
}

// Readers that set kStream run CityHashCrc256Long's block loop as a stream of
// 128-B lines (crc256_stream below).
template <class R, class = void>
struct ReaderStream {
  static constexpr bool value = false;
};
template <class R>
struct ReaderStream<R, decltype((void)R::kStream)> {
  static constexpr bool value = R::kStream;
};

// CityHashCrc256Long's state (city.c:412-423) and its 40-byte CHUNK
// (city.c:425-440).
template <class Tab>
struct Crc256State {
  u64 a, b, c, d, e, f, g, h, i, j, t;
  PDHT_HD void chunk(u64 w0, u64 w1, u64 w2, u64 w3, u64 w4, u64 mult, u32 flip, const Tab &T) {
    const u64 a0 = a;
    a = mul64(rotr(b, 41u ^ flip), mult) + w0;
    b = mul64(rotr(c, 27u ^ flip), mult) + w1;
    c = mul64(rotr(d, 41u ^ flip), mult) + w2;
    d = mul64(rotr(e, 33u ^ flip), mult) + w3;
    e = mul64(rotr(t, 25u ^ flip), mult) + w4;
    t = a0;
    f = crc32c_u64(f, a, T);
    g = crc32c_u64(g, b, T);
    h = crc32c_u64(h, c, T);
    i = crc32c_u64(i, d, T);
    j = crc32c_u64(j, e, T);
  }
};

// The block loop of CityHashCrc256Long (city.c:424-442) as a stream of whole
// 128-B lines (r04).  The 6 * (len / 240) block chunks of 40 B are one run of
// 8-B words over the key: chunk c = words [5c, 5c + 5), with the multiplier
// 1 / k0 and the rotation flip alternating by chunk parity (six chunks per
// block keep the alternation across blocks).  Lines come in two register
// buffers, even lines in A and odd ones in B; the moment a chunk has consumed
// the last word of line l, line l + 2 is requested into l's buffer, so one
// line's load is always in flight behind ~3 chunks of mixing -- per lane 128-B
// line loads (8 x dwordx4) instead of the 256-B line spans of the block form,
// and about half its registers.  Unrolled over 32 chunks = 10 lines (the two
// buffers' roles then repeat); chunks past the block loop are skipped
// (uniform for fixed-length keys).  Lines are read only below len (pieces of
// a line that start at or past len stay zero and are never used).
template <class R, class Tab>
struct Crc256Stream {
  const R &s;
  u64 len, nch, nlines;
  Crc256State<Tab> &st;
  const Tab &T;
  Words<32> A, B;
  PDHT_HD void load(u64 l, Words<32> &dst) const {
    if (l < nlines) dst = s.template line_lim<128>((u32)(128 * l), (u32)len);
  }
  template <int K>
  PDHT_HD u64 word() const {
    constexpr int line = K / 16, at = 8 * (K % 16);
    if constexpr (line % 2 == 0)
      return A.w64(at);
    else
      return B.w64(at);
  }
  // chunk C (0..31) of the double period that starts at chunk c0, line l0
  template <int C>
  PDHT_HD void step(u64 c0, u64 l0) {
    if (c0 + C >= nch) return;  // past the block loop (uniform)
    constexpr int k = 5 * C;
    st.chunk(word<k>(), word<k + 1>(), word<k + 2>(), word<k + 3>(), word<k + 4>(), (C & 1) ? kK0 : 1,
             (C & 1) ? 0u : 1u, T);
    constexpr int l1 = k / 16;
    if constexpr ((k + 5) / 16 > l1) {  // line l1 fully consumed: its buffer takes line l1 + 2
      if constexpr (l1 % 2 == 0)
        load(l0 + l1 + 2, A);
      else
        load(l0 + l1 + 2, B);
    }
  }
  template <int... C>
  PDHT_HD void period(u64 c0, u64 l0, std::integer_sequence<int, C...>) {
    (step<C>(c0, l0), ...);
  }
};

template <class R, class Tab>
PDHT_HD void crc256_stream_blocks(const R &s, u64 len, u32 seed, u64 out[4], Crc256State<Tab> &st,
                                  const Tab &T) {
  const u64 blocks = len / 240;
  Crc256Stream<R, Tab> S{s, len, 6 * blocks, (240 * blocks + 127) / 128, st, T, {}, {}};
  S.load(0, S.A);
  S.load(1, S.B);
  // block 0's opening words (city.c:414-419): bytes 56, 96, 120 (line 0), 184 (line 1)
  st.a = S.A.w64(56) + kK0;
  st.b = S.A.w64(96) + kK0;
  st.c = out[0] = mix16(st.b, len);
  st.d = out[1] = mul64(S.A.w64(120), kK0) + len;
  st.e = S.B.w64(56) + seed;
  st.f = seed;
  st.g = st.h = st.i = st.j = 0;
  st.t = st.c + st.d;
  for (u64 c0 = 0, l0 = 0; c0 < S.nch; c0 += 32, l0 += 10)
    S.period(c0, l0, std::make_integer_sequence<int, 32>{});
}

template <class R, class Tab = CrcConstTab>
PDHT_HD void crc256_long(const R &s, u64 len, u32 seed, u64 out[4], const Tab &T = Tab{}) {
  Crc256State<Tab> st;
  const u64 blocks = len / 240;
  if constexpr (ReaderStream<R>::value) {
    crc256_stream_blocks(s, len, seed, out, st, T);  // kStream readers: 128-B line stream
  } else {
    // line form: block k ends at or before its line-aligned load end B(k) =
    // 240k + 16(k mod 8) + 256 (or + 128); while B <= len the blocks stream as
    // whole lines, after that (only near the key's end) as plain 240-B spans
    Words<60> q;
    Words<28> carry;
    constexpr bool kLn = ReaderLines<R>::value;
    auto line_end = [](u64 k) { return 240 * k + 16 * (k & 7) + ((k & 7) == 7 ? 128 : 256); };
    if (kLn && line_end(0) <= len)
      crc_block_lines<0>(s, 0, carry, q);
    else
      q = s.template span<240>(0);  // block 0 (len >= 240)
    st.a = q.w64(56) + kK0;
    st.b = q.w64(96) + kK0;
    st.c = out[0] = mix16(st.b, len);
    st.d = out[1] = mul64(q.w64(120), kK0) + len;
    st.e = q.w64(184) + seed;
    st.f = seed;
    st.g = st.h = st.i = st.j = 0;
    st.t = st.c + st.d;
    auto chunk_at = [&](const Words<60> &w, u32 base, u64 mult, u32 flip) {
      st.chunk(w.w64(base), w.w64(base + 8), w.w64(base + 16), w.w64(base + 24), w.w64(base + 32), mult, flip,
               T);
    };
    u32 o = 0;
    for (u64 k = 0; k < blocks; ++k) {
      // (prefetching the next block as well measured equal, r02: 165 VGPRs)
      if (k) {
        if (kLn && line_end(k) <= len)  // uniform for fixed-length batches
          crc_block_lines_ph(s, o, (u32)k & 7, carry, q);
        else
          q = s.template span<240>(o);
      }
      chunk_at(q, 0, 1, 1);
      chunk_at(q, 40, kK0, 0);
      chunk_at(q, 80, 1, 1);
      chunk_at(q, 120, kK0, 0);
      chunk_at(q, 160, 1, 1);
      chunk_at(q, 200, kK0, 0);
      o += 240;
    }
  }
  // city.c:443-453: rest / 40 whole chunks, then one ending at len when
  // rest % 40 != 0 (rest < 240: at most 6).  Every chunk's load is issued
  // before the first is mixed (one round trip instead of up to six).
  {
    const u32 o = (u32)(blocks * 240);
    const u64 rest = len - blocks * 240;
    const u32 nt = (u32)(rest / 40) + (rest % 40 ? 1u : 0u);
    Words<10> tw[6];
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if ((u32)k < nt) tw[k] = s.template span<40>((u32)k < rest / 40 ? o + 40u * k : (u32)len - 40u);
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if ((u32)k < nt)
        st.chunk(tw[k].w64(0), tw[k].w64(8), tw[k].w64(16), tw[k].w64(24), tw[k].w64(32), kK0, 0, T);
  }
  // city.c:454-472
  u64 a = st.a, b = st.b, c = st.c, d = st.d, e = st.e, f = st.f, g = st.g, h = st.h, i = st.i, j = st.j,
      t = st.t;
  j += i << 32;
  a = mix16(a, j);
  h += g << 32;
  b += h;
  c = mix16(c, f) + i;
  d = mix16(d, e + out[0]);
  j += e;
  i += mix16(h, t);
  e = mix16(a, d) + j;
  f = mix16(b, c) + a;
  g = mix16(j, i) + c;
  out[0] = e + f + g + h;
  a = mul64(smix(mul64((a + g), kK0)), kK0) + b;
  out[1] += a + out[0];
  a = mul64(smix(mul64(a, kK0)), kK0) + c;
  out[2] = a + out[1];
  a = mul64(smix(mul64((a + e), kK0)), kK0);
  out[3] = a + out[2];
}

// city.c:476-489
template <class R, class Tab = CrcConstTab>
PDHT_HD void crc256(const R &s, u64 len, u64 out[4], const Tab &T = Tab{}) {
  if (len >= 240) {
    crc256_long(s, len, 0u, out, T);
  } else {
    crc256_long(PadReader<R>{s, (u32)len}, 240, ~(u32)len, out, T);
  }
}

// city.c:491-504
template <class R, class Tab = CrcConstTab>
PDHT_HD u128 crc128_seed(const R &s, u64 len, u128 seed, const Tab &T = Tab{}) {
  if (len <= 900) return city128_seed(s, len, seed);
  u64 r[4];
  crc256(s, len, r, T);
  const u64 u = seed.hi + r[0];
  const u64 v = seed.lo + r[1];
  return u128{mix16(u, v + r[2]), mix16(rotr_nz(v, 32), mul64(u, kK0) + r[3])};
}

// city.c:506-517
template <class R, class Tab = CrcConstTab>
PDHT_HD u128 crc128(const R &s, u64 len, const Tab &T = Tab{}) {
  if (len <= 900) return city128(s, len);
  u64 r[4];
  crc256(s, len, r, T);
  return u128{r[2], r[3]};
}

}  // namespace pdht
