/*
 * city_oracle.c -- plain-C99 restatement of pdht's CityHash path.
 *
 * TEST INFRASTRUCTURE ONLY (see city_oracle.h).  Written from the behaviour of
 * /root/reference/libpdht/city.c (CityHash v1.0.x semantics); every function
 * cites the reference lines it restates.  Bytes are assembled explicitly in
 * little-endian order, so the oracle does not depend on host endianness
 * (the reference's uint64_in_expected_order, city.c:50-75).
 */
#ifndef _POSIX_C_SOURCE
#define _POSIX_C_SOURCE 200809L
#endif
#include "city_oracle.h"

#include <pthread.h>
#include <string.h>
#include <time.h>

/* city.c:94-97 and :103 */
#define PK0 0xc3a5c85c97cb3127ULL
#define PK1 0xb492b66fbe98f273ULL
#define PK2 0x9ae16a3b2f90404fULL
#define PK3 0xc949d7c7509e6557ULL
#define PKMUL 0x9ddfea08eb382d69ULL

typedef struct {
  uint64_t lo; /* uint128.first  (city.h:58-65) */
  uint64_t hi; /* uint128.second */
} pair64;

/* city.c:38-48, :85-91 -- unaligned little-endian fetches */
static inline uint64_t le64(const uint8_t *p) {
  uint64_t r = 0;
  for (int i = 7; i >= 0; --i) r = (r << 8) | p[i];
  return r;
}
static inline uint32_t le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}

/* city.c:115-118 (Rotate) and :123-125 (RotateByAtLeast1) */
static inline uint64_t ror(uint64_t x, unsigned r) {
  r &= 63;
  return r == 0 ? x : ((x >> r) | (x << (64 - r)));
}
/* city.c:127-129 */
static inline uint64_t fold47(uint64_t x) { return x ^ (x >> 47); }

/* city.c:101-110 (Hash128to64) == city.c:131-136 (HashLen16(u, v)) */
static inline uint64_t mix2(uint64_t u, uint64_t v) {
  uint64_t t = (u ^ v) * PKMUL;
  t = fold47(t);
  uint64_t r = (v ^ t) * PKMUL;
  r = fold47(r);
  return r * PKMUL;
}

/* city.c:138-157 */
static uint64_t h64_short(const uint8_t *s, size_t n) {
  if (n >= 9) {
    uint64_t head = le64(s), tail = le64(s + n - 8);
    return mix2(head, ror(tail + n, (unsigned)n)) ^ tail;
  }
  if (n >= 4) {
    uint64_t head = le32(s);
    return mix2(n + (head << 3), (uint64_t)le32(s + n - 4));
  }
  if (n == 0) return PK2;
  uint32_t y = (uint32_t)s[0] | ((uint32_t)s[n >> 1] << 8);
  uint32_t z = (uint32_t)n + ((uint32_t)s[n - 1] << 2);
  return fold47((uint64_t)y * PK2 ^ (uint64_t)z * PK3) * PK2;
}

/* city.c:161-168 */
static uint64_t h64_mid(const uint8_t *s, size_t n) {
  uint64_t a = le64(s) * PK1;
  uint64_t b = le64(s + 8);
  uint64_t c = le64(s + n - 8) * PK2;
  uint64_t d = le64(s + n - 16) * PK0;
  uint64_t u = ror(a - b, 43) + ror(c, 30) + d;
  uint64_t v = a + ror(b ^ PK3, 20) - c + n;
  return mix2(u, v);
}

/* city.c:173-186 (WeakHashLen32WithSeeds6) */
static pair64 weak32w(uint64_t w, uint64_t x, uint64_t y, uint64_t z,
                      uint64_t a, uint64_t b) {
  a += w;
  b = ror(b + a + z, 21);
  uint64_t keep = a;
  a += x + y;
  b += ror(a, 44);
  pair64 r = {a + z, b + keep};
  return r;
}
/* city.c:190-198 */
static pair64 weak32(const uint8_t *p, uint64_t a, uint64_t b) {
  return weak32w(le64(p), le64(p + 8), le64(p + 16), le64(p + 24), a, b);
}

/* city.c:201-222 -- the 64-byte key path */
static uint64_t h64_upto64(const uint8_t *s, size_t n) {
  const uint8_t *e = s + n;
  /* forward half */
  uint64_t z1 = le64(s + 24);
  uint64_t a = le64(s) + (n + le64(e - 16)) * PK0;
  uint64_t b = ror(a + z1, 52);
  uint64_t c = ror(a, 37);
  a += le64(s + 8);
  c += ror(a, 7);
  a += le64(s + 16);
  uint64_t vf = a + z1, vs = b + ror(a, 31) + c;
  /* backward half */
  a = le64(s + 16) + le64(e - 32);
  uint64_t z2 = le64(e - 8);
  b = ror(a + z2, 52);
  c = ror(a, 37);
  a += le64(e - 24);
  c += ror(a, 7);
  a += le64(e - 16);
  uint64_t wf = a + z2, ws = b + ror(a, 31) + c;
  uint64_t r = fold47((vf + ws) * PK2 + (wf + vs) * PK0);
  return fold47(r * PK0 + vs) * PK2;
}

/* One 64-byte round shared by city.c:248-259 and :329-350.  State order:
 * x, y, z, v, w; the z/x exchange at the end of the round is included. */
typedef struct {
  uint64_t x, y, z;
  pair64 v, w;
} city_state;

static inline void round64(city_state *st, const uint8_t *p) {
  uint64_t x = st->x, y = st->y, z = st->z;
  x = ror(x + y + st->v.lo + le64(p + 8), 37) * PK1;
  y = ror(y + st->v.hi + le64(p + 48), 42) * PK1;
  x ^= st->w.hi;
  y += st->v.lo + le64(p + 40);
  z = ror(z + st->w.lo, 33) * PK1;
  pair64 nv = weak32(p, st->v.hi * PK1, x + st->w.lo);
  pair64 nw = weak32(p + 32, z + st->w.hi, y + le64(p + 16));
  st->v = nv;
  st->w = nw;
  st->x = z; /* exchange, city.c:255-257 */
  st->z = x;
  st->y = y;
}

/* city.c:224-263 */
uint64_t oracle_city64(const uint8_t *s, size_t n) {
  if (n <= 16) return h64_short(s, n);
  if (n <= 32) return h64_mid(s, n);
  if (n <= 64) return h64_upto64(s, n);

  const uint8_t *e = s + n;
  city_state st;
  /* tail-first initialisation, city.c:237-243 */
  st.x = le64(e - 40);
  st.y = le64(e - 16) + le64(e - 56);
  st.z = mix2(le64(e - 48) + n, le64(e - 24));
  st.v = weak32(e - 64, n, st.z);
  st.w = weak32(e - 32, st.y + PK1, st.x);
  st.x = st.x * PK1 + le64(s);
  /* (n-1)/64 full rounds from the front, city.c:246-260 */
  size_t rounds = (n - 1) / 64;
  for (size_t r = 0; r < rounds; ++r) round64(&st, s + 64 * r);
  /* city.c:261-262 */
  return mix2(mix2(st.v.lo, st.w.lo) + fold47(st.y) * PK1 + st.z,
              mix2(st.v.hi, st.w.hi) + st.x);
}

/* city.c:265-272 */
uint64_t oracle_city64_seeds(const uint8_t *s, size_t n, uint64_t seed0,
                             uint64_t seed1) {
  return mix2(oracle_city64(s, n) - seed0, seed1);
}
uint64_t oracle_city64_seed(const uint8_t *s, size_t n, uint64_t seed) {
  return oracle_city64_seeds(s, n, PK2, seed);
}

/* city.c:276-308 (CityMurmur), for n < 128 */
static pair64 murmur128(const uint8_t *s, size_t n, pair64 seed) {
  uint64_t a = seed.lo, b = seed.hi, c, d;
  if (n <= 16) {
    a = fold47(a * PK1) * PK1;
    c = b * PK1 + h64_short(s, n);
    d = fold47(a + (n >= 8 ? le64(s) : c));
  } else {
    c = mix2(le64(s + n - 8) + PK1, a);
    d = mix2(b + n, c + le64(s + n - 16));
    a += d;
    /* signed l = n-16 stepped by 16 while l > 0  ==  (n-1)/16 steps */
    size_t steps = (n - 1) / 16;
    for (size_t k = 0; k < steps; ++k, s += 16) {
      a ^= fold47(le64(s) * PK1) * PK1;
      a *= PK1;
      b ^= a;
      c ^= fold47(le64(s + 8) * PK1) * PK1;
      c *= PK1;
      d ^= c;
    }
  }
  a = mix2(a, c);
  b = mix2(d, b);
  pair64 r = {a ^ b, mix2(b, a)};
  return r;
}

/* city.c:310-376 */
static pair64 city128_seeded(const uint8_t *s, size_t n, pair64 seed) {
  if (n < 128) return murmur128(s, n, seed);

  city_state st;
  st.x = seed.lo;
  st.y = seed.hi;
  st.z = n * PK1;
  st.v.lo = ror(st.y ^ PK1, 49) * PK1 + le64(s);
  st.v.hi = ror(st.v.lo, 42) * PK1 + le64(s + 8);
  st.w.lo = ror(st.y + st.z, 35) * PK1 + st.x;
  st.w.hi = ror(st.x + le64(s + 88), 53) * PK1;
  size_t rem = n;
  do { /* two rounds per 128 bytes, city.c:328-352 */
    round64(&st, s);
    round64(&st, s + 64);
    s += 128;
    rem -= 128;
  } while (rem >= 128);
  uint64_t x = st.x, y = st.y, z = st.z;
  pair64 v = st.v, w = st.w;
  x += ror(v.lo + z, 49) * PK0;
  z += ror(w.lo, 37) * PK0;
  /* up to four 32-byte chunks taken backwards from the end, city.c:357-365 */
  for (size_t back = 32; back <= rem + 31 && rem > 0; back += 32) {
    const uint8_t *p = s + rem - back;
    y = ror(x + y, 42) * PK0 + v.hi;
    w.lo += le64(p + 16);
    x = x * PK0 + w.lo;
    z += w.hi + le64(p);
    w.hi += v.lo;
    v = weak32(p, v.lo + z, v.hi);
  }
  /* city.c:369-375 */
  x = mix2(x, v.lo);
  y = mix2(y + z, w.lo);
  pair64 r = {mix2(x + v.hi, w.hi) + y, mix2(x + w.hi, y + v.hi)};
  return r;
}

/* city.c:378-400 */
static pair64 city128(const uint8_t *s, size_t n) {
  pair64 seed;
  if (n >= 16) {
    seed.lo = le64(s) ^ PK3;
    seed.hi = le64(s + 8);
    return city128_seeded(s + 16, n - 16, seed);
  }
  if (n >= 8) {
    seed.lo = le64(s) ^ (n * PK0);
    seed.hi = le64(s + n - 8) ^ PK1;
    return city128_seeded(NULL, 0, seed);
  }
  seed.lo = PK0;
  seed.hi = PK1;
  return city128_seeded(s, n, seed);
}

void oracle_city128(const uint8_t *s, size_t len, uint64_t out[2]) {
  pair64 r = city128(s, len);
  out[0] = r.lo;
  out[1] = r.hi;
}
void oracle_city128_seed(const uint8_t *s, size_t len, uint64_t seed_lo,
                         uint64_t seed_hi, uint64_t out[2]) {
  pair64 seed = {seed_lo, seed_hi};
  pair64 r = city128_seeded(s, len, seed);
  out[0] = r.lo;
  out[1] = r.hi;
}

/* _mm_crc32_u64 (used at city.c:435-439): reflected CRC-32C, polynomial
 * 0x82F63B78, over the 8 little-endian bytes of v, starting from the low 32
 * bits of crc, with no inversion; result zero-extended. */
uint64_t oracle_crc32c_u64(uint64_t crc, uint64_t v) {
  uint32_t c = (uint32_t)crc;
  for (int byte = 0; byte < 8; ++byte) {
    c ^= (uint32_t)((v >> (8 * byte)) & 0xff);
    for (int bit = 0; bit < 8; ++bit) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
  }
  return c;
}

/* city.c:407-473 (CityHashCrc256Long), requires n >= 240 */
static void crc256_long(const uint8_t *s, size_t n, uint32_t seed,
                        uint64_t out[4]) {
  uint64_t a = le64(s + 56) + PK0;
  uint64_t b = le64(s + 96) + PK0;
  uint64_t c = out[0] = mix2(b, n);
  uint64_t d = out[1] = le64(s + 120) * PK0 + n;
  uint64_t e = le64(s + 184) + seed;
  uint64_t f = seed, g = 0, h = 0, i = 0, j = 0;
  uint64_t t = c + d;

  /* one 40-byte chunk: five rotate-multiply-adds then five CRC lanes */
#define ORACLE_CHUNK(mult, flip)                                \
  do {                                                          \
    uint64_t a0 = a;                                            \
    a = ror(b, 41u ^ (flip)) * (mult) + le64(s);                \
    b = ror(c, 27u ^ (flip)) * (mult) + le64(s + 8);            \
    c = ror(d, 41u ^ (flip)) * (mult) + le64(s + 16);           \
    d = ror(e, 33u ^ (flip)) * (mult) + le64(s + 24);           \
    e = ror(t, 25u ^ (flip)) * (mult) + le64(s + 32);           \
    t = a0;                                                     \
    f = oracle_crc32c_u64(f, a);                                \
    g = oracle_crc32c_u64(g, b);                                \
    h = oracle_crc32c_u64(h, c);                                \
    i = oracle_crc32c_u64(i, d);                                \
    j = oracle_crc32c_u64(j, e);                                \
    s += 40;                                                    \
  } while (0)

  size_t blocks = n / 240; /* >= 1 */
  size_t rest = n - blocks * 240;
  for (size_t k = 0; k < blocks; ++k) {
    ORACLE_CHUNK(1, 1);
    ORACLE_CHUNK(PK0, 0);
    ORACLE_CHUNK(1, 1);
    ORACLE_CHUNK(PK0, 0);
    ORACLE_CHUNK(1, 1);
    ORACLE_CHUNK(PK0, 0);
  }
  for (; rest >= 40; rest -= 40) ORACLE_CHUNK(PK0, 0);
  if (rest > 0) {
    s = s + rest - 40; /* re-read the last 40 bytes, city.c:451-454 */
    ORACLE_CHUNK(PK0, 0);
  }
#undef ORACLE_CHUNK
  /* city.c:455-472 */
  j += i << 32;
  a = mix2(a, j);
  h += g << 32;
  b += h;
  c = mix2(c, f) + i;
  d = mix2(d, e + out[0]);
  j += e;
  i += mix2(h, t);
  e = mix2(a, d) + j;
  f = mix2(b, c) + a;
  g = mix2(j, i) + c;
  out[0] = e + f + g + h;
  a = fold47((a + g) * PK0) * PK0 + b;
  out[1] += a + out[0];
  a = fold47(a * PK0) * PK0 + c;
  out[2] = a + out[1];
  a = fold47((a + e) * PK0) * PK0;
  out[3] = a + out[2];
}

/* city.c:476-489 */
void oracle_citycrc256(const uint8_t *s, size_t n, uint64_t out[4]) {
  if (n >= 240) {
    crc256_long(s, n, 0, out);
  } else {
    uint8_t pad[240];
    memset(pad, 0, sizeof pad);
    if (n) memcpy(pad, s, n);
    crc256_long(pad, 240, ~(uint32_t)n, out);
  }
}

/* city.c:491-504 */
void oracle_citycrc128_seed(const uint8_t *s, size_t n, uint64_t seed_lo,
                            uint64_t seed_hi, uint64_t out[2]) {
  if (n <= 900) {
    oracle_city128_seed(s, n, seed_lo, seed_hi, out);
    return;
  }
  uint64_t r[4];
  oracle_citycrc256(s, n, r);
  uint64_t u = seed_hi + r[0];
  uint64_t v = seed_lo + r[1];
  out[0] = mix2(u, v + r[2]);
  out[1] = mix2(ror(v, 32), u * PK0 + r[3]);
}
/* city.c:506-517 */
void oracle_citycrc128(const uint8_t *s, size_t n, uint64_t out[2]) {
  if (n <= 900) {
    oracle_city128(s, n, out);
    return;
  }
  uint64_t r[4];
  oracle_citycrc256(s, n, r);
  out[0] = r[2];
  out[1] = r[3];
}

/* libpdht/hash.c:25-30: mbits = CityHash64(key, keysize); ptindex = mbits %
 * nptes (u32 store); rank = mbits % c->size (int promoted to u64). */
void oracle_pdht_hash(const void *key, unsigned keysize, unsigned nptes,
                      int nranks, uint64_t *mbits, uint32_t *ptindex,
                      uint32_t *rank) {
  uint64_t m = oracle_city64((const uint8_t *)key, keysize);
  *mbits = m;
  if (ptindex) *ptindex = (uint32_t)(m % (uint64_t)nptes);
  if (rank) *rank = (uint32_t)(m % (uint64_t)(int64_t)nranks);
}

/* ---- batch loops --------------------------------------------------------- */
void oracle_city64_fixed(const uint8_t *keys, size_t stride, size_t len,
                         size_t n, uint64_t *out) {
  for (size_t i = 0; i < n; ++i) out[i] = oracle_city64(keys + i * stride, len);
}
void oracle_city64_var(const uint8_t *bytes, const uint64_t *off, size_t n,
                       uint64_t *out) {
  for (size_t i = 0; i < n; ++i)
    out[i] = oracle_city64(bytes + off[i], (size_t)(off[i + 1] - off[i]));
}
void oracle_city128_fixed(const uint8_t *keys, size_t stride, size_t len,
                          size_t n, uint64_t *out) {
  for (size_t i = 0; i < n; ++i) oracle_city128(keys + i * stride, len, out + 2 * i);
}
void oracle_citycrc128_fixed(const uint8_t *keys, size_t stride, size_t len,
                             size_t n, uint64_t *out) {
  for (size_t i = 0; i < n; ++i)
    oracle_citycrc128(keys + i * stride, len, out + 2 * i);
}
void oracle_city128_var(const uint8_t *bytes, const uint64_t *off, size_t n,
                        uint64_t *out) {
  for (size_t i = 0; i < n; ++i)
    oracle_city128(bytes + off[i], (size_t)(off[i + 1] - off[i]), out + 2 * i);
}
void oracle_citycrc128_var(const uint8_t *bytes, const uint64_t *off, size_t n,
                           uint64_t *out) {
  for (size_t i = 0; i < n; ++i)
    oracle_citycrc128(bytes + off[i], (size_t)(off[i + 1] - off[i]), out + 2 * i);
}
void oracle_pdht_hash_fixed(const uint8_t *keys, unsigned keysize, size_t n,
                            unsigned nptes, int nranks, uint64_t *mbits,
                            uint32_t *ptindex, uint32_t *rank) {
  for (size_t i = 0; i < n; ++i)
    oracle_pdht_hash(keys + (size_t)keysize * i, keysize, nptes, nranks,
                     mbits + i, ptindex ? ptindex + i : NULL,
                     rank ? rank + i : NULL);
}

uint64_t oracle_fold64(const uint64_t *d, size_t n, uint64_t first_index) {
  uint64_t acc = 0;
  for (size_t i = 0; i < n; ++i) acc += d[i] * (2 * (first_index + i) + 1);
  return acc;
}

/* splitmix64 (Steele/Lea/Flood; the JDK SplittableRandom finaliser):
 * output k = mix(seed + (k+1) * 0x9e3779b97f4a7c15). */
void oracle_splitmix64_fill(uint64_t seed, uint64_t start, size_t nwords,
                            uint64_t *out) {
  for (size_t w = 0; w < nwords; ++w) {
    uint64_t z = seed + (start + w + 1) * 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    out[w] = z ^ (z >> 31);
  }
}

/* ---- CPU timing harness --------------------------------------------------- */
uint64_t oracle_city64_c(const char *s, size_t len) {
  return oracle_city64((const uint8_t *)s, len);
}

typedef struct {
  oracle_city64_fn fn;
  const uint8_t *keys;
  size_t len, lo, hi;
  int reps;
  uint64_t *out;
} time_job;

static void *time_worker(void *arg) {
  time_job *jb = (time_job *)arg;
  for (int r = 0; r < jb->reps; ++r)
    for (size_t i = jb->lo; i < jb->hi; ++i)
      jb->out[i] = jb->fn((const char *)(jb->keys + i * jb->len), jb->len);
  return NULL;
}

double oracle_time_city64(oracle_city64_fn fn, const uint8_t *keys, size_t len,
                          size_t n, int threads, int reps, uint64_t *out) {
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t tid[512];
  time_job jobs[512];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC_RAW, &t0);
  for (int t = 0; t < threads; ++t) {
    jobs[t].fn = fn;
    jobs[t].keys = keys;
    jobs[t].len = len;
    jobs[t].lo = n * (size_t)t / (size_t)threads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
    jobs[t].reps = reps;
    jobs[t].out = out;
    if (t > 0) pthread_create(&tid[t], NULL, time_worker, &jobs[t]);
  }
  time_worker(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
  clock_gettime(CLOCK_MONOTONIC_RAW, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- generic batch apply over an external function ----------------------- */
typedef struct {
  oracle_city64_fn f64;
  oracle_city128_fn f128;
  const uint8_t *bytes;
  const uint64_t *off;
  size_t stride, len, lo, hi;
  uint64_t *out;
} apply_job;

static void *apply_worker(void *arg) {
  apply_job *jb = (apply_job *)arg;
  for (size_t i = jb->lo; i < jb->hi; ++i) {
    const uint8_t *p;
    size_t n;
    if (jb->off) {
      p = jb->bytes + jb->off[i];
      n = (size_t)(jb->off[i + 1] - jb->off[i]);
    } else {
      p = jb->bytes + i * jb->stride;
      n = jb->len;
    }
    if (jb->f64) {
      jb->out[i] = jb->f64((const char *)p, n);
    } else {
      oracle_u128 r = jb->f128((const char *)p, n);
      jb->out[2 * i] = r.first;
      jb->out[2 * i + 1] = r.second;
    }
  }
  return NULL;
}

static void apply_run(apply_job proto, size_t n, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t tid[512];
  apply_job jobs[512];
  for (int t = 0; t < threads; ++t) {
    jobs[t] = proto;
    jobs[t].lo = n * (size_t)t / (size_t)threads;
    jobs[t].hi = n * (size_t)(t + 1) / (size_t)threads;
    if (t > 0) pthread_create(&tid[t], NULL, apply_worker, &jobs[t]);
  }
  apply_worker(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
}

void oracle_apply64(oracle_city64_fn fn, const uint8_t *bytes,
                    const uint64_t *offsets, size_t stride, size_t len,
                    size_t n, uint64_t *out, int threads) {
  apply_job p = {fn, NULL, bytes, offsets, stride, len, 0, 0, out};
  apply_run(p, n, threads);
}

void oracle_apply128(oracle_city128_fn fn, const uint8_t *bytes,
                     const uint64_t *offsets, size_t stride, size_t len,
                     size_t n, uint64_t *out, int threads) {
  apply_job p = {NULL, fn, bytes, offsets, stride, len, 0, 0, out};
  apply_run(p, n, threads);
}

/* ---- the product's pdht_hashfunc over a batch ----------------------------- */
/* n calls of a pdht_hashfunc (libpdht/pdht.h:196) over packed keys, as n calls
 * of dht->hashfn (putget.c:53) would make them: lets the tests run the
 * PRODUCT's scalar pdht_hash over a whole config (cfg1) in C.  rank8 is a
 * ptl_process_t array (8 bytes per entry, .rank = the low 32 bits). */
typedef void (*oracle_hashfunc)(void *dht, void *key, uint64_t *mbits, uint32_t *ptindex,
                                void *rank);
void oracle_apply_hashfn(oracle_hashfunc fn, void *dht, const uint8_t *keys, size_t keysize,
                         size_t n, uint64_t *mbits, uint32_t *ptindex, uint64_t *rank8) {
  for (size_t i = 0; i < n; ++i)
    fn(dht, (void *)(keys + i * keysize), mbits + i, ptindex + i, rank8 + i);
}

/* ---- CPU baseline harness (bench.py cpu_baseline) ------------------------- */
/* `threads` pthreads over contiguous slices, `reps` passes.  mode 0: out[i] =
 * f64(key_i); 1: {out[2i], out[2i+1]} = f128(key_i); 2: pdht_hash semantics
 * (libpdht/hash.c:25-30): out[i] = mbits = f64(key_i), pt[i] = mbits % nptes,
 * rk[i] = mbits % nranks (run-time divisors, real divides as in the
 * reference).  Keys fixed (key i at bytes + i*stride, len bytes) or
 * offset-indexed (offsets != NULL).  Returns wall seconds measured with
 * CLOCK_MONOTONIC_RAW (the clock of pdht_inline.h:33-41). */
typedef struct {
  int mode;
  oracle_city64_fn f64;
  oracle_city128_fn f128;
  const uint8_t *bytes;
  const uint64_t *off;
  size_t stride, len, lo, hi;
  int reps;
  uint64_t nptes, nranks;
  uint64_t *out;
  uint32_t *pt, *rk;
} bjob;

static void *bworker(void *arg) {
  bjob *j = (bjob *)arg;
  for (int r = 0; r < j->reps; ++r) {
    for (size_t i = j->lo; i < j->hi; ++i) {
      const uint8_t *p;
      size_t n;
      if (j->off) {
        p = j->bytes + j->off[i];
        n = (size_t)(j->off[i + 1] - j->off[i]);
      } else {
        p = j->bytes + i * j->stride;
        n = j->len;
      }
      if (j->mode == 1) {
        oracle_u128 v = j->f128((const char *)p, n);
        j->out[2 * i] = v.first;
        j->out[2 * i + 1] = v.second;
      } else {
        const uint64_t m = j->f64((const char *)p, n);
        j->out[i] = m;
        if (j->mode == 2) {
          j->pt[i] = (uint32_t)(m % j->nptes);
          j->rk[i] = (uint32_t)(m % j->nranks);
        }
      }
    }
  }
  return NULL;
}

double oracle_time_batch(int mode, void *fn, const uint8_t *bytes, const uint64_t *offsets,
                         size_t stride, size_t len, size_t n, int threads, int reps,
                         uint64_t nptes, uint64_t nranks, uint64_t *out, uint32_t *pt,
                         uint32_t *rk) {
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t tid[512];
  bjob jobs[512];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC_RAW, &t0);
  for (int t = 0; t < threads; ++t) {
    bjob j = {mode, NULL, NULL, bytes, offsets, stride, len, 0, 0, reps, nptes ? nptes : 1,
              nranks ? nranks : 1, out, pt, rk};
    if (mode == 1)
      j.f128 = (oracle_city128_fn)fn;
    else
      j.f64 = (oracle_city64_fn)fn;
    j.lo = n * (size_t)t / (size_t)threads;
    j.hi = n * (size_t)(t + 1) / (size_t)threads;
    jobs[t] = j;
    if (t > 0) pthread_create(&tid[t], NULL, bworker, &jobs[t]);
  }
  bworker(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
  clock_gettime(CLOCK_MONOTONIC_RAW, &t1);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- CPU baseline of destination bucketing (bench.py bucket/records) ----- */
/* The count-then-ship shape of the reference's bulk loader
 * (bench/Meraculous/buildUFXhashBinary.h:103-109: hashfn per key,
 * my_heap_sizes[rank]++, ufx_remote_thread[idx] = rank; the keys then go out
 * grouped by rank, :255-279), as a parallel stable counting sort with
 * `threads` pthreads over contiguous slices:
 *   1. every thread hashes its slice (mbits = f64(key), rank = mbits %
 *      nranks, real divides as hash.c:27/:29) and counts its ranks;
 *   2. bucket offsets and per-(rank, thread) starts (thread 0's prefix);
 *   3. every thread scatters its slice to the bucketed positions: arrays
 *      (key, mbits, ptindex = mbits % nptes, original index), or with
 *      `records` the wire record of bucket_records (type, src rank,
 *      ht_index, index, mbits, key; stride 24 + keysize rounded up to 8).
 * The same outputs as the GPU's pdht_bucket_batch_dev /
 * pdht_bucket_records_dev.  Returns wall seconds of `reps` bucketings
 * (CLOCK_MONOTONIC_RAW).  hist: threads * nranks uint32 of scratch. */
typedef struct {
  oracle_city64_fn f64;
  const uint8_t *keys;
  size_t L, lo, hi, n;
  int t, threads, reps, records;
  uint64_t nptes;
  uint32_t nranks, src, ht;
  uint64_t *mb;      /* [n] digests in key order */
  uint32_t *rk;      /* [n] ranks in key order */
  uint32_t *hist;    /* [threads][nranks]: counts, then start positions */
  uint8_t *keys_out; /* arrays form */
  uint64_t *mbits_out;
  uint32_t *pt_out, *idx_out;
  uint8_t *rec_out;  /* records form */
  uint64_t *offsets; /* [nranks + 1] */
  pthread_barrier_t *bar;
} bkjob;

static void *bucket_worker(void *arg) {
  bkjob *j = (bkjob *)arg;
  uint32_t *h = j->hist + (size_t)j->t * j->nranks;
  const size_t rb = 24 + ((j->L + 7) & ~(size_t)7);
  for (int r = 0; r < j->reps; ++r) {
    memset(h, 0, (size_t)j->nranks * 4);
    for (size_t i = j->lo; i < j->hi; ++i) {
      const uint64_t m = j->f64((const char *)(j->keys + i * j->L), j->L);
      const uint32_t k = (uint32_t)(m % j->nranks);
      j->mb[i] = m;
      j->rk[i] = k;
      h[k]++;
    }
    pthread_barrier_wait(j->bar);
    if (j->t == 0) { /* starts: rank-major, thread-minor (stable) */
      uint64_t pos = 0;
      for (uint32_t k = 0; k < j->nranks; ++k) {
        j->offsets[k] = pos;
        for (int t = 0; t < j->threads; ++t) {
          uint32_t *c = j->hist + (size_t)t * j->nranks + k;
          const uint32_t cnt = *c;
          *c = (uint32_t)pos;
          pos += cnt;
        }
      }
      j->offsets[j->nranks] = pos;
    }
    pthread_barrier_wait(j->bar);
    for (size_t i = j->lo; i < j->hi; ++i) {
      const uint32_t p = h[j->rk[i]]++;
      const uint64_t m = j->mb[i];
      if (j->records) {
        uint8_t *q = j->rec_out + (size_t)p * rb;
        const uint32_t hdr[4] = {1u, j->src, j->ht, (uint32_t)i};
        memcpy(q, hdr, 16);
        memcpy(q + 16, &m, 8);
        memcpy(q + 24, j->keys + i * j->L, j->L);
        memset(q + 24 + j->L, 0, rb - 24 - j->L);
      } else {
        memcpy(j->keys_out + (size_t)p * j->L, j->keys + i * j->L, j->L);
        j->mbits_out[p] = m;
        j->pt_out[p] = (uint32_t)(m % j->nptes);
        j->idx_out[p] = (uint32_t)i;
      }
    }
    pthread_barrier_wait(j->bar);
  }
  return NULL;
}

double oracle_time_bucket(oracle_city64_fn fn, const uint8_t *keys, size_t L, size_t n, int threads,
                          int reps, uint64_t nptes, uint32_t nranks, int records, uint32_t src,
                          uint32_t ht, uint64_t *mb, uint32_t *rk, uint32_t *hist, uint8_t *keys_out,
                          uint64_t *mbits_out, uint32_t *pt_out, uint32_t *idx_out, uint8_t *rec_out,
                          uint64_t *offsets) {
  if (threads < 1) threads = 1;
  if (threads > 512) threads = 512;
  pthread_t tid[512];
  static bkjob jobs[512];
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)threads);
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC_RAW, &t0);
  for (int t = 0; t < threads; ++t) {
    bkjob j = {fn, keys, L, n * (size_t)t / (size_t)threads, n * (size_t)(t + 1) / (size_t)threads, n, t,
               threads, reps, records, nptes ? nptes : 1, nranks ? nranks : 1, src, ht, mb, rk, hist,
               keys_out, mbits_out, pt_out, idx_out, rec_out, offsets, &bar};
    jobs[t] = j;
    if (t > 0) pthread_create(&tid[t], NULL, bucket_worker, &jobs[t]);
  }
  bucket_worker(&jobs[0]);
  for (int t = 1; t < threads; ++t) pthread_join(tid[t], NULL);
  clock_gettime(CLOCK_MONOTONIC_RAW, &t1);
  pthread_barrier_destroy(&bar);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

