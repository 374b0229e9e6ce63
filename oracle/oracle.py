"""ctypes view of the parity oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, bench.py's cpu_baseline leg and __graft_entry__.smoke() import
this module, and only as the *checker*.  The product (pdht_amd/) never does.

Two libraries are exposed:
  * ``lib()``  -> oracle/liboracle.so, our C99 restatement of
    /root/reference/libpdht/city.c (+ hash.c:25-30), see city_oracle.c.
  * ``ref()``  -> oracle/_ref/libcityref.so, the reference city.c itself,
    compiled from /root/reference by oracle/Makefile (None if not built).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(HERE, "liboracle.so")
_REF = os.path.join(HERE, "_ref", "libcityref.so")

_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)

_lib = None
_ref = None


class Uint128(C.Structure):
    """city.h:58-65 -- {first = low 64, second = high 64}."""

    _fields_ = [("first", C.c_uint64), ("second", C.c_uint64)]


def build() -> None:
    """Compile liboracle.so (and _ref/ when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        L.oracle_city64.restype = C.c_uint64
        L.oracle_city64.argtypes = [C.c_void_p, C.c_size_t]
        L.oracle_city64_seed.restype = C.c_uint64
        L.oracle_city64_seed.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.oracle_city64_seeds.restype = C.c_uint64
        L.oracle_city64_seeds.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64]
        for name in ("oracle_city128", "oracle_citycrc128"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [C.c_void_p, C.c_size_t, _u64p]
        for name in ("oracle_city128_seed", "oracle_citycrc128_seed"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64, _u64p]
        L.oracle_citycrc256.restype = None
        L.oracle_citycrc256.argtypes = [C.c_void_p, C.c_size_t, _u64p]
        L.oracle_crc32c_u64.restype = C.c_uint64
        L.oracle_crc32c_u64.argtypes = [C.c_uint64, C.c_uint64]
        L.oracle_pdht_hash.restype = None
        L.oracle_pdht_hash.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_int, _u64p, _u32p, _u32p]
        for name in ("oracle_city64_fixed", "oracle_city128_fixed", "oracle_citycrc128_fixed"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_void_p]
        for name in ("oracle_city64_var", "oracle_city128_var", "oracle_citycrc128_var"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.oracle_pdht_hash_fixed.restype = None
        L.oracle_pdht_hash_fixed.argtypes = [C.c_void_p, C.c_uint, C.c_size_t, C.c_uint, C.c_int,
                                             C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_fold64.restype = C.c_uint64
        L.oracle_fold64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.oracle_splitmix64_fill.restype = None
        L.oracle_splitmix64_fill.argtypes = [C.c_uint64, C.c_uint64, C.c_size_t, C.c_void_p]
        L.oracle_time_city64.restype = C.c_double
        L.oracle_time_city64.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                         C.c_int, C.c_int, C.c_void_p]
        L.oracle_apply_hashfn.restype = None
        L.oracle_apply_hashfn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                          C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_time_batch.restype = C.c_double
        L.oracle_time_batch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                        C.c_size_t, C.c_size_t, C.c_int, C.c_int, C.c_uint64,
                                        C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.oracle_time_bucket.restype = C.c_double
        L.oracle_time_bucket.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                         C.c_uint64, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32]
        L.oracle_time_bucket.argtypes += [C.c_void_p] * 9
        for name in ("oracle_apply64", "oracle_apply128"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                          C.c_size_t, C.c_void_p, C.c_int]
        _lib = L
    return _lib


def ref():
    """The reference city.c (compiled from /root/reference); None if absent."""
    global _ref
    if _ref is None:
        if not os.path.exists(_REF):
            return None
        R = C.CDLL(_REF)
        R.CityHash64.restype = C.c_uint64
        R.CityHash64.argtypes = [C.c_void_p, C.c_size_t]
        R.CityHash64WithSeed.restype = C.c_uint64
        R.CityHash64WithSeed.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        R.CityHash64WithSeeds.restype = C.c_uint64
        R.CityHash64WithSeeds.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint64]
        for name in ("CityHash128", "CityHashCrc128"):
            f = getattr(R, name)
            f.restype = Uint128
            f.argtypes = [C.c_void_p, C.c_size_t]
        for name in ("CityHash128WithSeed", "CityHashCrc128WithSeed"):
            f = getattr(R, name)
            f.restype = Uint128
            f.argtypes = [C.c_void_p, C.c_size_t, Uint128]
        R.CityHashCrc256.restype = None
        R.CityHashCrc256.argtypes = [C.c_void_p, C.c_size_t, _u64p]
        _ref = R
    return _ref


def ref_path() -> str | None:
    return _REF if os.path.exists(_REF) else None


# ---------------------------------------------------------------- helpers ---
def _buf(b) -> C.c_void_p:
    if isinstance(b, np.ndarray):
        assert b.flags["C_CONTIGUOUS"]
        return C.c_void_p(b.ctypes.data)
    return C.c_char_p(bytes(b))


def city64(data: bytes) -> int:
    return lib().oracle_city64(_buf(data), len(data))


def city64_seed(data: bytes, seed: int) -> int:
    return lib().oracle_city64_seed(_buf(data), len(data), seed)


def city64_seeds(data: bytes, s0: int, s1: int) -> int:
    return lib().oracle_city64_seeds(_buf(data), len(data), s0, s1)


def city128(data: bytes) -> tuple[int, int]:
    out = (C.c_uint64 * 2)()
    lib().oracle_city128(_buf(data), len(data), out)
    return out[0], out[1]


def city128_seed(data: bytes, lo: int, hi: int) -> tuple[int, int]:
    out = (C.c_uint64 * 2)()
    lib().oracle_city128_seed(_buf(data), len(data), lo, hi, out)
    return out[0], out[1]


def citycrc128(data: bytes) -> tuple[int, int]:
    out = (C.c_uint64 * 2)()
    lib().oracle_citycrc128(_buf(data), len(data), out)
    return out[0], out[1]


def citycrc128_seed(data: bytes, lo: int, hi: int) -> tuple[int, int]:
    out = (C.c_uint64 * 2)()
    lib().oracle_citycrc128_seed(_buf(data), len(data), lo, hi, out)
    return out[0], out[1]


def citycrc256(data: bytes) -> tuple[int, int, int, int]:
    out = (C.c_uint64 * 4)()
    lib().oracle_citycrc256(_buf(data), len(data), out)
    return tuple(out)


def pdht_hash(key: bytes, nptes: int, nranks: int) -> tuple[int, int, int]:
    m, p, r = C.c_uint64(), C.c_uint32(), C.c_uint32()
    lib().oracle_pdht_hash(_buf(key), len(key), nptes, nranks, C.byref(m), C.byref(p), C.byref(r))
    return m.value, p.value, r.value


def city64_fixed(keys: np.ndarray) -> np.ndarray:
    """keys: uint8 [n, L] -> uint64 [n]"""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, L = keys.shape
    out = np.empty(n, dtype=np.uint64)
    lib().oracle_city64_fixed(_buf(keys), L, L, n, _buf(out))
    return out


def city128_fixed(keys: np.ndarray, crc: bool = False) -> np.ndarray:
    """keys: uint8 [n, L] -> uint64 [n, 2] (low, high)"""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, L = keys.shape
    out = np.empty((n, 2), dtype=np.uint64)
    f = lib().oracle_citycrc128_fixed if crc else lib().oracle_city128_fixed
    f(_buf(keys), L, L, n, _buf(out))
    return out


def city64_var(data: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.empty(n, dtype=np.uint64)
    lib().oracle_city64_var(_buf(data), _buf(offsets), n, _buf(out))
    return out


def city128_var(data: np.ndarray, offsets: np.ndarray, crc: bool = False) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offsets.size - 1
    out = np.empty((n, 2), dtype=np.uint64)
    f = lib().oracle_citycrc128_var if crc else lib().oracle_city128_var
    f(_buf(data), _buf(offsets), n, _buf(out))
    return out


def pdht_hash_fixed(keys: np.ndarray, nptes: int, nranks: int):
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, L = keys.shape
    m = np.empty(n, dtype=np.uint64)
    p = np.empty(n, dtype=np.uint32)
    r = np.empty(n, dtype=np.uint32)
    lib().oracle_pdht_hash_fixed(_buf(keys), L, n, nptes, nranks, _buf(m), _buf(p), _buf(r))
    return m, p, r


def fold64(d: np.ndarray, first_index: int = 0) -> int:
    d = np.ascontiguousarray(d, dtype=np.uint64).reshape(-1)
    return lib().oracle_fold64(_buf(d), d.size, first_index)


def splitmix64(seed: int, start: int, nwords: int) -> np.ndarray:
    out = np.empty(nwords, dtype=np.uint64)
    lib().oracle_splitmix64_fill(seed, start, nwords, _buf(out))
    return out


# ------------------------------------------------- synthetic workloads -------
SEED_KEYS = 0x5EED5EED5EED5EED   # key bytes
SEED_LENS = 0x1E575EED1E575EED   # mixed-length lengths stream


def fixed_keys(n: int, L: int, first_key: int = 0, seed: int = SEED_KEYS) -> np.ndarray:
    """Key i = bytes [i*L, (i+1)*L) of the little-endian splitmix64 byte stream."""
    assert (first_key * L) % 8 == 0
    w0 = first_key * L // 8
    nw = (n * L + 7) // 8
    words = splitmix64(seed, w0, nw)
    return words.view(np.uint8)[: n * L].reshape(n, L)


def mixed_lengths(n: int, lo: int = 16, hi: int = 256, first_key: int = 0,
                  seed: int = SEED_LENS) -> np.ndarray:
    """len_i = lo + splitmix64(seed)[i] % (hi - lo + 1)  (16..256 for cfg3)."""
    r = splitmix64(seed, first_key, n)
    return (np.uint64(lo) + r % np.uint64(hi - lo + 1)).astype(np.uint64)


def mixed_keys(n: int, lo: int = 16, hi: int = 256, seed: int = SEED_KEYS,
               lseed: int = SEED_LENS):
    """Packed variable-length keys: (bytes uint8[total], offsets uint64[n+1])."""
    lens = mixed_lengths(n, lo, hi, 0, lseed)
    offsets = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    total = int(offsets[-1])
    words = splitmix64(seed, 0, (total + 7) // 8)
    return words.view(np.uint8)[:total].copy(), offsets


def time_city64(keys: np.ndarray, threads: int, reps: int, use_ref: bool = True):
    """Wall seconds for `reps` passes of CityHash64 over keys [n, L] with
    `threads` pthreads; uses the reference city.c when built, else the port."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, L = keys.shape
    out = np.empty(n, dtype=np.uint64)
    R = ref() if use_ref else None
    if R is not None:
        fn = C.cast(R.CityHash64, C.c_void_p)
        kind = "reference"
    else:
        fn = C.cast(lib().oracle_city64_c, C.c_void_p)
        kind = "port"
    secs = lib().oracle_time_city64(fn, _buf(keys), L, n, threads, reps, _buf(out))
    return secs, out, kind


def apply_ref64(bytes_: np.ndarray, n: int, *, offsets=None, L: int = 0,
                threads: int = 8, fn_name: str = "CityHash64") -> np.ndarray:
    """Run the *reference* CityHash64 (oracle/_ref) over a batch."""
    R = ref()
    assert R is not None, "oracle/_ref not built (needs /root/reference)"
    out = np.empty(n, dtype=np.uint64)
    fn = C.cast(getattr(R, fn_name), C.c_void_p)
    offp = _buf(np.ascontiguousarray(offsets, dtype=np.uint64)) if offsets is not None else None
    lib().oracle_apply64(fn, _buf(bytes_), offp, L, L, n, _buf(out), threads)
    return out


def apply_ref128(bytes_: np.ndarray, n: int, *, offsets=None, L: int = 0,
                 threads: int = 8, fn_name: str = "CityHashCrc128") -> np.ndarray:
    R = ref()
    assert R is not None, "oracle/_ref not built (needs /root/reference)"
    out = np.empty((n, 2), dtype=np.uint64)
    fn = C.cast(getattr(R, fn_name), C.c_void_p)
    offp = _buf(np.ascontiguousarray(offsets, dtype=np.uint64)) if offsets is not None else None
    lib().oracle_apply128(fn, _buf(bytes_), offp, L, L, n, _buf(out), threads)
    return out


def apply_hashfn(fn_ptr: int, dht_ptr: int, keys: np.ndarray):
    """n calls of a pdht_hashfunc (e.g. the PRODUCT's pdht_hash) over packed
    keys [n, keysize], in C.  Returns (mbits u64[n], ptindex u32[n], rank
    u32[n]); ptindex is pre-filled with 0xFFFFFFFF so an implementation that
    leaves it untouched (libmpipdht/hash.c:6-9) is visible."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, L = keys.shape
    m = np.empty(n, np.uint64)
    p = np.full(n, 0xFFFFFFFF, np.uint32)
    r = np.zeros(n, np.uint64)  # ptl_process_t[n]
    lib().oracle_apply_hashfn(C.c_void_p(fn_ptr), C.c_void_p(dht_ptr), _buf(keys), L, n, _buf(m), _buf(p),
                              _buf(r))
    return m, p, (r & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def cpu_fn(name: str = "CityHash64", use_ref: bool = True):
    """(function pointer, kind) of a CityHash function for the CPU baseline:
    the reference city.c (oracle/_ref, kind "reference") when built, else the
    oracle port (kind "port")."""
    R = ref() if use_ref else None
    if R is not None:
        return C.cast(getattr(R, name), C.c_void_p).value, "reference"
    port = {"CityHash64": "oracle_city64_c"}
    if name not in port:
        raise RuntimeError(f"no port of {name} for the CPU baseline (oracle/_ref not built)")
    return C.cast(getattr(lib(), port[name]), C.c_void_p).value, "port"


def time_batch(mode: int, fn: int, data: np.ndarray, n: int, *, offsets=None, L: int = 0,
               threads: int = 1, reps: int = 1, nptes: int = 1, nranks: int = 1, outs=None):
    """Wall seconds (CLOCK_MONOTONIC_RAW) of `reps` passes over a batch with
    `threads` pthreads; mode 0 = 64-bit digests, 1 = 128-bit, 2 = pdht_hash
    semantics (hash.c:25-30).  Returns (secs, digests, ptindex, rank).
    `outs` = (digests, ptindex, rank) of an earlier call to reuse: fresh
    arrays would put their first-touch page faults inside the timing."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    if outs is not None:
        out, pt, rk = outs
    else:
        out = np.zeros(2 * n if mode == 1 else n, np.uint64)
        pt = np.zeros(n, np.uint32) if mode == 2 else None
        rk = np.zeros(n, np.uint32) if mode == 2 else None
    offp = _buf(np.ascontiguousarray(offsets, dtype=np.uint64)) if offsets is not None else None
    secs = lib().oracle_time_batch(mode, C.c_void_p(fn), _buf(data), offp, L, L, n, threads, reps, nptes,
                                   nranks, _buf(out), _buf(pt) if pt is not None else None,
                                   _buf(rk) if rk is not None else None)
    return secs, out, pt, rk


class BucketBufs:
    """Output and scratch arrays of time_bucket (allocated once and touched,
    so that first-touch page faults stay out of the timing)."""

    def __init__(self, n: int, L: int, nranks: int, threads: int, records: bool):
        self.mb = np.zeros(n, np.uint64)
        self.rk = np.zeros(n, np.uint32)
        self.hist = np.zeros(max(threads, 1) * nranks, np.uint32)
        self.offsets = np.zeros(nranks + 1, np.uint64)
        rb = 24 + (L + 7) // 8 * 8
        if records:
            self.rec = np.zeros((n, rb), np.uint8)
            self.keys = self.mbits = self.pt = self.idx = None
        else:
            self.rec = None
            self.keys = np.zeros((n, L), np.uint8)
            self.mbits = np.zeros(n, np.uint64)
            self.pt = np.zeros(n, np.uint32)
            self.idx = np.zeros(n, np.uint32)


def time_bucket(fn: int, keys: np.ndarray, nptes: int, nranks: int, *, threads: int = 1, reps: int = 1,
                records: bool = False, src_rank: int = 0, ht_index: int = 0, bufs: BucketBufs | None = None):
    """Wall seconds (CLOCK_MONOTONIC_RAW) of `reps` destination bucketings of
    keys [n, L] with `threads` pthreads: hash (fn = CityHash64), count per
    rank, stable scatter (oracle_time_bucket, the reference bulk loader's
    count-then-ship shape).  Returns (secs, bufs): bufs holds the bucketed
    arrays (keys, mbits, pt, idx) or records, and the offsets."""
    keys = np.ascontiguousarray(keys, dtype=np.uint8)
    n, L = keys.shape
    b = bufs or BucketBufs(n, L, nranks, threads, records)
    opt = lambda a: _buf(a) if a is not None else None  # noqa: E731
    secs = lib().oracle_time_bucket(C.c_void_p(fn), _buf(keys), L, n, threads, reps, nptes, nranks,
                                    int(records), src_rank, ht_index, _buf(b.mb), _buf(b.rk), _buf(b.hist),
                                    opt(b.keys), opt(b.mbits), opt(b.pt), opt(b.idx), opt(b.rec),
                                    _buf(b.offsets))
    return secs, b

