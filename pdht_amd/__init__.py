"""pdht_amd -- MI355X batch key-hashing engine for pdht's CityHash path.

Python view of the C-ABI in include/pdht_hip.h / pdht_city.h / pdht_hash.h,
loaded from the in-tree pdht_amd/lib/libpdht_hip.so (built by `make` or
__graft_entry__.build()).  There is no fallback: if the library is missing
the import fails, and the batch entry points fail when no GPU is usable.

torch is used only as device-memory / stream plumbing: tensors are passed to
the C-ABI as raw pointers on torch's current HIP stream.

Mirrors of the reference interface:
  CityHash64 / CityHash64WithSeed(s) / CityHash128(WithSeed) /
  CityHashCrc128(WithSeed) / CityHashCrc256   -- city.h:68-84, citycrc.h:39-46
  PdhtTable.hash (pdht_hash, hash.c:25-30), PdhtTable.sethash (hash.c:39-41)
Batch API (new): city64_batch, city128_batch, citycrc128_batch, *_var,
place_batch (fused pdht_hash over a batch), *_host variants.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "lib", "libpdht_hip.so")

__all__ = [
    "lib", "LIB_PATH", "PdhtError", "CityHash64", "CityHash64WithSeed", "CityHash64WithSeeds",
    "CityHash128", "CityHash128WithSeed", "CityHashCrc128", "CityHashCrc128WithSeed",
    "CityHashCrc256", "city64_batch", "city64_seeds_batch", "city64_var_batch", "city128_batch",
    "city128_seed_batch", "city128_var_batch", "citycrc128_batch", "citycrc128_seed_batch",
    "citycrc128_var_batch", "place_batch", "city64_batch_host", "city64_var_batch_host",
    "citycrc128_batch_host", "place_batch_host", "splitmix64_fill", "mixed_lengths",
    "device_count", "PdhtTable", "K2", "bucket_batch", "bucket_records", "record_fields",
    "bucket_record_bytes", "bucket_workspace_bytes", "WeakHashLen32WithSeeds", "WeakHashLen32WithSeeds6",
    "tuning", "last_kernel", "mpi_lib",
]

K2 = 0x9AE16A3B2F90404F  # city.c:96 (CityHash64WithSeed's seed0)


class PdhtError(RuntimeError):
    pass


class Uint128(C.Structure):
    """city.h:58-65"""

    _fields_ = [("first", C.c_uint64), ("second", C.c_uint64)]


class PtlProcess(C.Union):
    """ptl_process_t stand-in (portals4.h): 8 bytes, .rank is the low uint32."""

    class _Phys(C.Structure):
        _fields_ = [("nid", C.c_uint32), ("pid", C.c_uint32)]

    _fields_ = [("phys", _Phys), ("rank", C.c_uint32)]


_HASHFUNC = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64),
                        C.POINTER(C.c_uint32), C.POINTER(PtlProcess))


class _PdhtT(C.Structure):
    """Stand-in pdht_t of include/pdht_hash.h (keysize, hashfn, ptl.nptes)."""

    _fields_ = [("keysize", C.c_uint), ("hashfn", C.c_void_p), ("nptes", C.c_uint)]


_lib = None        # the library the wrappers call (product, or tuning inside tuning())
_product = None
_tuning = None
_exp = {}  # libpdht_hip_exp[_<tag>].so by tag (tools/ only)
_V = C.c_void_p
_S = C.c_size_t
_U64 = C.c_uint64
_U32 = C.c_uint32
TUNING_LIB_PATH = os.path.join(HERE, "lib", "libpdht_hip_tuning.so")
# tools/ only: the tuning build with a compile-time experiment switched on
# (`make exp EXP=-DPDHT_...`), for A/B of changes a run-time variant cannot select
EXP_LIB_PATH = os.path.join(HERE, "lib", "libpdht_hip_exp.so")
MPI_LIB_PATH = os.path.join(HERE, "lib", "libpdht_hip_mpi.so")


def _declare(L, tuning=False):
    sig = {
        "pdht_hip_version": (C.c_char_p, []),
        "pdht_hip_last_error": (C.c_char_p, []),
        "pdht_hip_last_kernel": (C.c_char_p, []),
        "pdht_hip_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "pdht_hip_set_device": (C.c_int, [C.c_int]),
        "pdht_city64_batch_dev": (C.c_int, [_V, _S, _S, _S, _V, _V]),
        "pdht_city64_seeds_batch_dev": (C.c_int, [_V, _S, _S, _S, _U64, _U64, _V, _V]),
        "pdht_city64_batch_var_dev": (C.c_int, [_V, _S, _V, _S, _V, _V]),
        "pdht_city128_batch_dev": (C.c_int, [_V, _S, _S, _S, _V, _V]),
        "pdht_city128_seed_batch_dev": (C.c_int, [_V, _S, _S, _S, _U64, _U64, _V, _V]),
        "pdht_city128_batch_var_dev": (C.c_int, [_V, _S, _V, _S, _V, _V]),
        "pdht_citycrc128_batch_dev": (C.c_int, [_V, _S, _S, _S, _V, _V]),
        "pdht_citycrc128_seed_batch_dev": (C.c_int, [_V, _S, _S, _S, _U64, _U64, _V, _V]),
        "pdht_citycrc128_batch_var_dev": (C.c_int, [_V, _S, _V, _S, _V, _V]),
        "pdht_place_batch_dev": (C.c_int, [_V, _S, _S, _U32, _U32, _V, _V, _V, _S, _V, _V]),
        "pdht_city64_batch_host": (C.c_int, [_V, _S, _S, _V, C.c_int]),
        "pdht_city64_batch_var_host": (C.c_int, [_V, _V, _S, _V, C.c_int]),
        "pdht_citycrc128_batch_host": (C.c_int, [_V, _S, _S, _V, C.c_int]),
        "pdht_place_batch_host": (C.c_int, [_V, _S, _S, _U32, _U32, _V, _V, _V, _S, C.c_int]),
        "pdht_hip_splitmix64_fill_dev": (C.c_int, [_U64, _U64, _S, _V, _V]),
        "pdht_hip_mixed_lengths_dev": (C.c_int, [_U64, _U64, _S, _U32, _U32, _V, _V]),
        "pdht_hip_read_stream_dev": (C.c_int, [_V, _S, C.c_int, _V, _V]),
        "pdht_hip_key_stream_dev": (C.c_int, [_V, _S, _V, _V]),
        "pdht_hip_key_stream_var_dev": (C.c_int, [_V, _S, _V, _S, _V, _V]),
        "pdht_bucket_workspace_bytes": (C.c_size_t, [_S, _S, _U32]),
        "pdht_bucket_records_workspace_bytes": (C.c_size_t, [_S, _S, _U32]),
        "pdht_bucket_batch_dev": (C.c_int, [_V, _S, _S, _U32, _U32, _V, _S, _V, _V, _V, _V, _V, _V]),
        "pdht_bucket_record_bytes": (C.c_size_t, [_S]),
        "pdht_bucket_records_dev": (C.c_int, [_V, _S, _S, _U32, _U32, _U32, _U32, _V, _S, _V, _V, _V]),
        "CityHash64": (_U64, [_V, _S]),
        "CityHash64WithSeed": (_U64, [_V, _S, _U64]),
        "CityHash64WithSeeds": (_U64, [_V, _S, _U64, _U64]),
        "CityHash128": (Uint128, [_V, _S]),
        "CityHash128WithSeed": (Uint128, [_V, _S, Uint128]),
        "CityHashCrc128": (Uint128, [_V, _S]),
        "CityHashCrc128WithSeed": (Uint128, [_V, _S, Uint128]),
        "CityHashCrc256": (None, [_V, _S, C.POINTER(C.c_uint64)]),
        "WeakHashLen32WithSeeds": (Uint128, [_V, _U64, _U64]),
        "WeakHashLen32WithSeeds6": (Uint128, [_U64, _U64, _U64, _U64, _U64, _U64]),
        "pdht_hash": (None, [_V, _V, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                             C.POINTER(PtlProcess)]),
        "pdht_sethash": (None, [_V, _V]),
        "pdht_hash_batch": (C.c_int, [_V, _V, _S, _V, _V, _V, C.c_int]),
        "pdht_hash_batch_dev": (C.c_int, [_V, _V, _S, _V, _V, _V, _V, _V]),
        "pdht_hip_table_init": (None, [_V, C.c_uint, C.c_uint]),
    }
    if tuning:
        sig["pdht_hip_set_variant"] = (C.c_int, [C.c_int])
        sig["pdht_hip_set_blocks_per_cu"] = (C.c_int, [C.c_int])
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


def _load(path, tuning=False):
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `make -C {ROOT}` or "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    L = C.CDLL(path)
    _declare(L, tuning)
    return L


def lib():
    """The library the batch wrappers call: the product libpdht_hip.so (loaded
    once), or the tuning build inside a `tuning()` block.  Raises if it was
    not built."""
    global _lib, _product
    if _lib is None:
        _product = _load(LIB_PATH)
        _lib = _product
    return _lib


_mpi = None


def mpi_lib():
    """libpdht_hip_mpi.so: the same engine with the libmpipdht flavour of
    pdht_hash / pdht_hash_batch(_dev) (libmpipdht/hash.c:6-9: mbits and rank,
    ptindex never written).  Loaded on demand, beside the product library."""
    global _mpi
    if _mpi is None:
        _mpi = _load(MPI_LIB_PATH)
    return _mpi


class tuning:
    """Context manager for tools/ and the A/B tests: route every wrapper
    through libpdht_hip_tuning.so (same sources, built with the A/B hook
    headers of pdht_amd/csrc/tuning/) with
    kernel variant `variant` and, optionally, `per_cu` workgroups per CU.
    The product library has no variants and no tuning entry points."""

    def __init__(self, variant: int = 0, per_cu: int = 0, exp=False):
        # exp: True = libpdht_hip_exp.so, "<tag>" = libpdht_hip_exp_<tag>.so
        # (compile-time experiments: make exp EXP=... EXP_TAG=<tag>)
        self.variant, self.per_cu, self.exp = variant, per_cu, exp

    def __enter__(self):
        global _lib, _tuning, _exp
        lib()
        if self.exp:
            tag = "" if self.exp is True else str(self.exp)
            if tag not in _exp:
                path = EXP_LIB_PATH if not tag else EXP_LIB_PATH.replace(".so", f"_{tag}.so")
                _exp[tag] = _load(path, tuning=True)
            self._t = _exp[tag]
        else:
            if _tuning is None:
                _tuning = _load(TUNING_LIB_PATH, tuning=True)
            self._t = _tuning
        self._prev = _lib
        self._old = (self._t.pdht_hip_set_variant(self.variant),
                     self._t.pdht_hip_set_blocks_per_cu(self.per_cu))
        _lib = self._t
        return self

    def __exit__(self, *exc):
        global _lib
        self._t.pdht_hip_set_variant(self._old[0])
        self._t.pdht_hip_set_blocks_per_cu(self._old[1])
        _lib = self._prev
        return False


def _check(rc: int, what: str):
    if rc != 0:
        raise PdhtError(f"{what}: {lib().pdht_hip_last_error().decode()}")


def last_kernel() -> str:
    return lib().pdht_hip_last_kernel().decode()


def device_count() -> int:
    c = C.c_int(0)
    _check(lib().pdht_hip_device_count(C.byref(c)), "device_count")
    return c.value


# ------------------------------------------------------------ scalar API ---
def _cbuf(data):
    if isinstance(data, np.ndarray):
        return C.c_void_p(data.ctypes.data), data.nbytes
    b = bytes(data)
    return C.c_char_p(b), len(b)


def CityHash64(data) -> int:
    p, n = _cbuf(data)
    return lib().CityHash64(p, n)


def CityHash64WithSeed(data, seed: int) -> int:
    p, n = _cbuf(data)
    return lib().CityHash64WithSeed(p, n, seed)


def CityHash64WithSeeds(data, seed0: int, seed1: int) -> int:
    p, n = _cbuf(data)
    return lib().CityHash64WithSeeds(p, n, seed0, seed1)


def CityHash128(data) -> tuple[int, int]:
    p, n = _cbuf(data)
    r = lib().CityHash128(p, n)
    return r.first, r.second


def CityHash128WithSeed(data, seed: tuple[int, int]) -> tuple[int, int]:
    p, n = _cbuf(data)
    r = lib().CityHash128WithSeed(p, n, Uint128(*seed))
    return r.first, r.second


def CityHashCrc128(data) -> tuple[int, int]:
    p, n = _cbuf(data)
    r = lib().CityHashCrc128(p, n)
    return r.first, r.second


def CityHashCrc128WithSeed(data, seed: tuple[int, int]) -> tuple[int, int]:
    p, n = _cbuf(data)
    r = lib().CityHashCrc128WithSeed(p, n, Uint128(*seed))
    return r.first, r.second


def CityHashCrc256(data) -> tuple[int, int, int, int]:
    p, n = _cbuf(data)
    out = (C.c_uint64 * 4)()
    lib().CityHashCrc256(p, n, out)
    return tuple(out)


def WeakHashLen32WithSeeds(data, a: int, b: int) -> tuple[int, int]:
    """city.c:190-198 (reads 32 bytes of data)."""
    p, n = _cbuf(data)
    if n < 32:
        raise ValueError("WeakHashLen32WithSeeds reads 32 bytes")
    r = lib().WeakHashLen32WithSeeds(p, a, b)
    return r.first, r.second


def WeakHashLen32WithSeeds6(w: int, x: int, y: int, z: int, a: int, b: int) -> tuple[int, int]:
    """city.c:173-187"""
    r = lib().WeakHashLen32WithSeeds6(w, x, y, z, a, b)
    return r.first, r.second


# ----------------------------------------------------- device batch API ---
# Every device wrapper launches on the device its tensors live on: the C-ABI
# sizes grids for, and launches on, the CURRENT device, so each call runs
# under `with torch.cuda.device(<tensor's device>)` on that device's stream
# (the caller's `stream`, which must belong to the same device, or the
# device's current stream).  Every tensor handed to C is checked for device,
# dtype, contiguity and size first: a wrong one raises instead of letting a
# kernel write past its end.
def _torch():
    import torch
    return torch


class _on:
    """Device guard + stream of one device-side call.  The device switch and
    the current-stream lookup go through torch's raw accessors when they
    exist (a batch call's host cost is what a 1M-key batch waits for:
    tools/call_overhead.py)."""

    __slots__ = ("device", "index", "stream_obj", "prev", "stream")

    def __init__(self, device, stream=None):
        if device.type != "cuda":
            raise ValueError("expected CUDA tensors")
        self.device = device
        self.index = device.index if device.index is not None else _torch().cuda.current_device()
        self.stream_obj = stream
        if stream is not None and stream.device != device:
            raise ValueError(f"stream is on {stream.device}, tensors on {device}")

    def __enter__(self):
        tc = _torch()._C
        if hasattr(tc, "_cuda_getDevice") and hasattr(tc, "_cuda_getCurrentRawStream"):
            self.prev = tc._cuda_getDevice()
            if self.prev != self.index:
                tc._cuda_setDevice(self.index)
            s = self.stream_obj.cuda_stream if self.stream_obj is not None else \
                tc._cuda_getCurrentRawStream(self.index)
        else:
            torch = _torch()
            self.prev = torch.cuda.current_device()
            torch.cuda.set_device(self.index)
            s = (self.stream_obj if self.stream_obj is not None else torch.cuda.current_stream(self.device)).cuda_stream
        self.stream = C.c_void_p(s)
        return self

    def __exit__(self, *exc):
        if self.prev != self.index:
            _torch().cuda.set_device(self.prev)
        return False


def _dptr(t) -> C.c_void_p:
    return C.c_void_p(t.data_ptr())


def _opt(t):
    return _dptr(t) if t is not None else None


def _need(t, name, dtype, device, numel=None, shape=None):
    """A CUDA tensor of `dtype` on `device`, contiguous, with >= numel
    elements (or exactly `shape`)."""
    if t is None:
        raise ValueError(f"{name} is required")
    if not getattr(t, "is_cuda", False) or t.device != device:
        raise ValueError(f"{name} must be a CUDA tensor on {device}")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name} must hold >= {numel} elements, got {t.numel()}")
    return t


def _keys_2d(keys):
    """keys: uint8 CUDA tensor [n, L] with unit inner stride (rows may be strided)."""
    torch = _torch()
    if not isinstance(keys, torch.Tensor) or keys.dtype != torch.uint8 or keys.dim() != 2 or not keys.is_cuda:
        raise ValueError("keys must be a CUDA uint8 tensor of shape [n, keylen]")
    n, L = keys.shape
    if keys.stride(1) != 1 and L > 1 and n > 0:
        raise ValueError("keys rows must be contiguous")
    stride = keys.stride(0) if n > 1 else L
    return n, L, stride


def _out(n, words, device, out=None):
    torch = _torch()
    shape = (n,) if words == 1 else (n, words)
    if out is None:
        return torch.empty(shape, dtype=torch.int64, device=device)
    return _need(out, "out", torch.int64, device, shape=shape)


def city64_batch(keys, out=None, stream=None):
    """CityHash64 of each row of keys [n, L] (uint8, CUDA) -> int64 [n] (bit pattern of u64)."""
    n, L, stride = _keys_2d(keys)
    out = _out(n, 1, keys.device, out)
    with _on(keys.device, stream) as g:
        _check(lib().pdht_city64_batch_dev(_dptr(keys), stride, L, n, _dptr(out), g.stream),
               "pdht_city64_batch_dev")
    return out


def city64_seeds_batch(keys, seed0: int, seed1: int, out=None, stream=None):
    n, L, stride = _keys_2d(keys)
    out = _out(n, 1, keys.device, out)
    with _on(keys.device, stream) as g:
        _check(lib().pdht_city64_seeds_batch_dev(_dptr(keys), stride, L, n, seed0, seed1, _dptr(out),
                                                 g.stream), "pdht_city64_seeds_batch_dev")
    return out


def city64_seed_batch(keys, seed: int, out=None, stream=None):
    """CityHash64WithSeed == WithSeeds(k2, seed) (city.c:265-267)."""
    return city64_seeds_batch(keys, K2, seed, out, stream)


def _check_var(data, offsets, check=True, stream=None):
    """(n, nbytes) of a variable-length batch.  nbytes is what the C ABI takes
    as the key bytes the batch spans: it picks the LDS window and how the
    batch is cut into ~512 MiB launches (launch.h launch_var); it never
    addresses memory.

    check=True (default): read offsets[0] and offsets[n] back ON THE LAUNCH
    STREAM (`stream`, else the device's current stream) -- one 16-B D2H copy
    that waits for the work queued before it on that stream, so this call is
    host-synchronous -- require 0 <= offsets[0] <= offsets[n] <= data.numel()
    (a bad offsets tensor raises instead of sending the window kernel past the
    data buffer) and pass the exact span offsets[n] - offsets[0].
    check=False, or while the launch stream is being captured into a graph:
    no read, fully asynchronous; the caller vouches for the offsets and the
    span passed is data.numel() (an upper bound; a much larger buffer than
    the keys only skews the window/launch-size heuristic, never correctness).
    The kernels trust that offsets never decrease, as the reference trusts
    its key pointers."""
    torch = _torch()
    if data.dtype != torch.uint8 or not data.is_cuda or not data.is_contiguous():
        raise ValueError("data must be a contiguous CUDA uint8 tensor")
    _need(offsets, "offsets", torch.int64, data.device)
    if offsets.dim() != 1 or offsets.numel() < 1:
        raise ValueError("offsets must be a 1-D int64 tensor of n+1 entries")
    n = offsets.numel() - 1
    if check and n:
        s = stream if stream is not None else torch.cuda.current_stream(data.device)
        if s.device != data.device:
            raise ValueError(f"stream is on {s.device}, tensors on {data.device}")
        with torch.cuda.stream(s):
            if not torch.cuda.is_current_stream_capturing():
                lo, hi = (int(x) for x in offsets[[0, n]].tolist())
                if not 0 <= lo <= hi <= data.numel():
                    raise ValueError(f"offsets span bytes [{lo}, {hi}) but data holds {data.numel()}")
                return n, hi - lo
    return n, data.numel()


def city64_var_batch(data, offsets, out=None, stream=None, check=True):
    n, nb = _check_var(data, offsets, check, stream)
    out = _out(n, 1, data.device, out)
    with _on(data.device, stream) as g:
        _check(lib().pdht_city64_batch_var_dev(_dptr(data), nb, _dptr(offsets), n, _dptr(out), g.stream),
               "pdht_city64_batch_var_dev")
    return out


def city128_batch(keys, out=None, stream=None):
    n, L, stride = _keys_2d(keys)
    out = _out(n, 2, keys.device, out)
    with _on(keys.device, stream) as g:
        _check(lib().pdht_city128_batch_dev(_dptr(keys), stride, L, n, _dptr(out), g.stream),
               "pdht_city128_batch_dev")
    return out


def city128_seed_batch(keys, seed: tuple[int, int], out=None, stream=None):
    n, L, stride = _keys_2d(keys)
    out = _out(n, 2, keys.device, out)
    with _on(keys.device, stream) as g:
        _check(lib().pdht_city128_seed_batch_dev(_dptr(keys), stride, L, n, seed[0], seed[1], _dptr(out),
                                                 g.stream), "pdht_city128_seed_batch_dev")
    return out


def city128_var_batch(data, offsets, out=None, stream=None, check=True):
    n, nb = _check_var(data, offsets, check, stream)
    out = _out(n, 2, data.device, out)
    with _on(data.device, stream) as g:
        _check(lib().pdht_city128_batch_var_dev(_dptr(data), nb, _dptr(offsets), n, _dptr(out), g.stream),
               "pdht_city128_batch_var_dev")
    return out


def citycrc128_batch(keys, out=None, stream=None):
    n, L, stride = _keys_2d(keys)
    out = _out(n, 2, keys.device, out)
    with _on(keys.device, stream) as g:
        _check(lib().pdht_citycrc128_batch_dev(_dptr(keys), stride, L, n, _dptr(out), g.stream),
               "pdht_citycrc128_batch_dev")
    return out


def citycrc128_seed_batch(keys, seed: tuple[int, int], out=None, stream=None):
    n, L, stride = _keys_2d(keys)
    out = _out(n, 2, keys.device, out)
    with _on(keys.device, stream) as g:
        _check(lib().pdht_citycrc128_seed_batch_dev(_dptr(keys), stride, L, n, seed[0], seed[1],
                                                    _dptr(out), g.stream), "pdht_citycrc128_seed_batch_dev")
    return out


def citycrc128_var_batch(data, offsets, out=None, stream=None, check=True):
    n, nb = _check_var(data, offsets, check, stream)
    out = _out(n, 2, data.device, out)
    with _on(data.device, stream) as g:
        _check(lib().pdht_citycrc128_batch_var_dev(_dptr(data), nb, _dptr(offsets), n, _dptr(out),
                                                   g.stream), "pdht_citycrc128_batch_var_dev")
    return out


def place_batch(keys, nptes: int, nranks: int, *, ptindex=True, rank=True, hist=None,
                stream=None, out=None):
    """Fused pdht_hash (hash.c:25-30) over keys [n, keysize] (packed, CUDA).

    Returns (mbits int64[n], ptindex int32[n] | None, rank int32[n] | None);
    if `hist` (int64[>= nranks], CUDA) is given, per-rank counts are added to it.
    `out` = a previous return value (same n) to reuse its tensors.
    """
    torch = _torch()
    n, L, stride = _keys_2d(keys)
    if stride != L:
        raise ValueError("place_batch needs packed keys")
    dev = keys.device
    if hist is not None:
        _need(hist, "hist", torch.int64, dev, numel=nranks)
    if out is not None:
        mb, pt, rk = out
        _need(mb, "out[0] (mbits)", torch.int64, dev, shape=(n,))
        if pt is not None:
            _need(pt, "out[1] (ptindex)", torch.int32, dev, shape=(n,))
        if rk is not None:
            _need(rk, "out[2] (rank)", torch.int32, dev, shape=(n,))
    else:
        mb = torch.empty(n, dtype=torch.int64, device=dev)
        pt = torch.empty(n, dtype=torch.int32, device=dev) if ptindex else None
        rk = torch.empty(n, dtype=torch.int32, device=dev) if rank else None
    with _on(dev, stream) as g:
        _check(lib().pdht_place_batch_dev(_dptr(keys), L, n, nptes, nranks, _dptr(mb), _opt(pt), _opt(rk), 4,
                                          _opt(hist), g.stream), "pdht_place_batch_dev")
    return mb, pt, rk


def bind_place_batch(keys, nptes: int, nranks: int, *, hist=None, stream=None, out=None):
    """place_batch prepared once for repeated calls on the same tensors.

    The checks, pointer and stream lookups run here; the returned callable
    makes only the C call (pdht_place_batch_dev on the stream current now),
    i.e. a C caller's per-batch cost.  Returns (call, (mbits, ptindex, rank)).
    The caller keeps keys.device current and the tensors alive.
    """
    torch = _torch()
    n, L, stride = _keys_2d(keys)
    if stride != L:
        raise ValueError("bind_place_batch needs packed keys")
    dev = keys.device
    if hist is not None:
        _need(hist, "hist", torch.int64, dev, numel=nranks)
    if out is None:
        out = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
               torch.empty(n, dtype=torch.int32, device=dev))
    mb, pt, rk = out
    _need(mb, "out[0] (mbits)", torch.int64, dev, shape=(n,))
    _need(pt, "out[1] (ptindex)", torch.int32, dev, shape=(n,))
    _need(rk, "out[2] (rank)", torch.int32, dev, shape=(n,))
    f = lib().pdht_place_batch_dev
    with _on(dev, stream) as g:
        st = g.stream
    vals = (_dptr(keys), L, n, nptes, nranks, _dptr(mb), _dptr(pt), _dptr(rk), 4, _opt(hist), st)
    args = tuple(a if isinstance(a, C._SimpleCData) or a is None else t(a) for t, a in zip(f.argtypes, vals))

    def call():
        rc = f(*args)
        if rc:
            _check(rc, "pdht_place_batch_dev")

    return call, out


def bucket_workspace_bytes(n: int, keysize: int, nranks: int, records: bool = False) -> int:
    """Workspace bytes of bucket_batch (records=False) or bucket_records
    (records=True) on n keysize-byte keys over nranks ranks."""
    if records:
        return lib().pdht_bucket_records_workspace_bytes(n, keysize, nranks)
    return lib().pdht_bucket_workspace_bytes(n, keysize, nranks)


def _workspace(workspace, n, L, nranks, dev, records=False):
    torch = _torch()
    need = bucket_workspace_bytes(n, L, nranks, records)
    if workspace is None:
        return torch.empty(max(need, 1), dtype=torch.uint8, device=dev), need
    _need(workspace, "workspace", torch.uint8, dev, numel=need)
    return workspace, workspace.numel()


def bucket_batch(keys, nptes: int, nranks: int, *, with_keys=True, with_ptindex=True,
                 with_index=True, stream=None, out=None, workspace=None):
    """Destination bucketing (include/pdht_hip.h pdht_bucket_batch_dev): a stable
    counting sort of packed keys [n, L] by rank = CityHash64 % nranks.

    Returns (keys_out [n, L] | None, mbits int64[n], ptindex int32[n] | None,
    index int32[n] (unsigned original positions) | None, offsets
    int64[nranks+1]); bucket r is rows offsets[r]:offsets[r+1], keys in
    original order.  `out` = a previous return value (same n, L, nranks) to
    reuse its tensors; `workspace` = a uint8 CUDA tensor of at least
    bucket_workspace_bytes(n, L, nranks) bytes (allocated per call if None).
    """
    torch = _torch()
    n, L, stride = _keys_2d(keys)
    if stride != L:
        raise ValueError("bucket_batch needs packed keys")
    dev = keys.device
    ws, ws_bytes = _workspace(workspace, n, L, nranks, dev)
    if out is not None:
        ko, mb, pt, ix, offs = out
        if ko is not None:
            _need(ko, "out[0] (keys)", torch.uint8, dev, shape=(n, L))
        _need(mb, "out[1] (mbits)", torch.int64, dev, shape=(n,))
        if pt is not None:
            _need(pt, "out[2] (ptindex)", torch.int32, dev, shape=(n,))
        if ix is not None:
            _need(ix, "out[3] (index)", torch.int32, dev, shape=(n,))
        _need(offs, "out[4] (offsets)", torch.int64, dev, shape=(nranks + 1,))
    else:
        ko = torch.empty_like(keys, memory_format=torch.contiguous_format) if with_keys else None
        mb = torch.empty(n, dtype=torch.int64, device=dev)
        pt = torch.empty(n, dtype=torch.int32, device=dev) if with_ptindex else None
        ix = torch.empty(n, dtype=torch.int32, device=dev) if with_index else None
        offs = torch.empty(nranks + 1, dtype=torch.int64, device=dev)
    with _on(dev, stream) as g:
        _check(lib().pdht_bucket_batch_dev(_dptr(keys), L, n, nptes, nranks, _dptr(ws), ws_bytes, _opt(ko),
                                           _dptr(mb), _opt(pt), _opt(ix), _dptr(offs), g.stream),
               "pdht_bucket_batch_dev")
    return ko, mb, pt, ix, offs


PDHT_PUT = 1  # msg_type pdhtPut (libmpipdht/pdht.h:72)


def bucket_record_bytes(keysize: int) -> int:
    return lib().pdht_bucket_record_bytes(keysize)


def bucket_records(keys, nranks: int, *, msg_type: int = PDHT_PUT, src_rank: int = 0, ht_index: int = 0,
                   stream=None, out=None, workspace=None):
    """Destination bucketing into wire records (include/pdht_hip.h
    pdht_bucket_records_dev): the MPI variant's message_t header + key for
    every key, bucket r = records[offsets[r]:offsets[r+1]].

    Returns (records uint8 [n, pdht_bucket_record_bytes(L)], offsets int64
    [nranks+1]); record_fields() splits them into tensors.  `out` = a previous
    return value to reuse; `workspace` as for bucket_batch, of at least
    bucket_workspace_bytes(n, L, nranks, records=True) bytes.
    """
    torch = _torch()
    n, L, stride = _keys_2d(keys)
    if stride != L:
        raise ValueError("bucket_records needs packed keys")
    dev = keys.device
    rb = bucket_record_bytes(L)
    ws, ws_bytes = _workspace(workspace, n, L, nranks, dev, records=True)
    if out is not None:
        rec, offs = out
        _need(rec, "out[0] (records)", torch.uint8, dev, shape=(n, rb))
        if rec.data_ptr() % 8:
            raise ValueError("records must be 8-byte aligned")
        _need(offs, "out[1] (offsets)", torch.int64, dev, shape=(nranks + 1,))
    else:
        # int64 storage keeps the records 8-byte aligned
        rec = torch.empty(max(n * rb // 8, 1), dtype=torch.int64, device=dev).view(torch.uint8)[: n * rb]
        rec = rec.view(n, rb)
        offs = torch.empty(nranks + 1, dtype=torch.int64, device=dev)
    with _on(dev, stream) as g:
        _check(lib().pdht_bucket_records_dev(_dptr(keys), L, n, nranks, msg_type, src_rank, ht_index,
                                             _dptr(ws), ws_bytes, _dptr(rec), _dptr(offs), g.stream),
               "pdht_bucket_records_dev")
    return rec, offs


def record_fields(records, keysize: int):
    """Views of a record batch [m, stride] (uint8): (type int32[m], rank
    int32[m], ht_index int32[m], index int32[m] (unsigned), mbits int64[m],
    keys uint8[m, keysize])."""
    torch = _torch()
    m, rb = records.shape
    flat = records.contiguous().view(-1)
    w32 = flat.view(torch.int32).view(m, rb // 4)
    w64 = flat.view(torch.int64).view(m, rb // 8)
    return w32[:, 0], w32[:, 1], w32[:, 2], w32[:, 3], w64[:, 2], records[:, 24:24 + keysize]


def splitmix64_fill(seed: int, first: int, nwords: int, out=None, device="cuda", stream=None):
    torch = _torch()
    if out is None:
        out = torch.empty(nwords, dtype=torch.int64, device=device)
    else:
        _need(out, "out", torch.int64, out.device, numel=nwords)
    with _on(out.device, stream) as g:
        _check(lib().pdht_hip_splitmix64_fill_dev(seed, first, nwords, _dptr(out), g.stream),
               "pdht_hip_splitmix64_fill_dev")
    return out


def read_stream(buf, nt: bool = False, out=None, stream=None):
    """HBM read-bandwidth calibration: XOR-fold of a CUDA buffer (16-B multiple)."""
    torch = _torch()
    if not buf.is_contiguous():
        raise ValueError("buf must be contiguous")
    if out is None:
        out = torch.zeros(1, dtype=torch.int64, device=buf.device)
    _need(out, "out", torch.int64, buf.device, numel=1)
    with _on(buf.device, stream) as g:
        _check(lib().pdht_hip_read_stream_dev(_dptr(buf), buf.numel() * buf.element_size(), int(nt),
                                              _dptr(out), g.stream), "pdht_hip_read_stream_dev")
    return out


def key_stream(keys, out=None, stream=None):
    """Calibration: the 64-B kernel's data movement with an XOR fold for a hash."""
    torch = _torch()
    n = keys.shape[0]
    if keys.dim() != 2 or keys.shape[1] != 64 or keys.dtype != torch.uint8 or not keys.is_contiguous():
        raise PdhtError("key_stream takes a contiguous (n, 64) uint8 tensor")
    out = _out(n, 1, keys.device, out)
    with _on(keys.device, stream) as g:
        _check(lib().pdht_hip_key_stream_dev(_dptr(keys), n, _dptr(out), g.stream), "pdht_hip_key_stream_dev")
    return out


def key_stream_var(data, offsets, out=None, stream=None, check=True):
    """Calibration: the variable-length kernel's data movement with an XOR fold."""
    n, nb = _check_var(data, offsets, check, stream)
    out = _out(n, 1, data.device, out)
    with _on(data.device, stream) as g:
        _check(lib().pdht_hip_key_stream_var_dev(_dptr(data), nb, _dptr(offsets), n, _dptr(out), g.stream),
               "pdht_hip_key_stream_var_dev")
    return out


def mixed_lengths(seed: int, first: int, n: int, lo: int, hi: int, device="cuda", stream=None):
    torch = _torch()
    out = torch.empty(n, dtype=torch.int64, device=device)
    with _on(out.device, stream) as g:
        _check(lib().pdht_hip_mixed_lengths_dev(seed, first, n, lo, hi, _dptr(out), g.stream),
               "pdht_hip_mixed_lengths_dev")
    return out


# ------------------------------------------------------- host batch API ---
# Host buffers: numpy arrays or CPU torch tensors (pinned ones take the
# zero-copy path).  Everything is checked before C sees it: dtype,
# C-contiguity and size, so a strided view or a short `out` raises instead
# of producing wrong digests or writing past a host buffer.
def _host_arr(a, name, dtype, shape=None, numel=None):
    """numpy array or CPU torch tensor of `dtype` (numpy dtype), C-contiguous."""
    if isinstance(a, np.ndarray):
        if a.dtype != dtype:
            raise ValueError(f"{name} must be {np.dtype(dtype)}, got {a.dtype}")
        if not a.flags["C_CONTIGUOUS"]:
            raise ValueError(f"{name} must be C-contiguous")
        shp, size = a.shape, a.size
    else:
        torch = _torch()
        if not isinstance(a, torch.Tensor) or a.is_cuda:
            raise ValueError(f"{name} must be a numpy array or a CPU torch tensor")
        tdt = {np.dtype(np.uint8): torch.uint8, np.dtype(np.uint64): torch.int64,
               np.dtype(np.uint32): torch.int32}[np.dtype(dtype)]
        if a.dtype not in (tdt, {torch.int64: torch.uint64, torch.int32: torch.uint32}.get(tdt, tdt)):
            raise ValueError(f"{name} must be {tdt}, got {a.dtype}")
        if not a.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        shp, size = tuple(a.shape), a.numel()
    if shape is not None and tuple(shp) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(shp)}")
    if numel is not None and size < numel:
        raise ValueError(f"{name} must hold >= {numel} elements, got {size}")
    return a


def _host_keys(keys):
    """Host keys [n, L] uint8, C-contiguous (packed rows)."""
    _host_arr(keys, "keys", np.uint8)
    if len(keys.shape) != 2:
        raise ValueError("keys must be 2-D [n, keylen]")
    return tuple(keys.shape)


def _np_keys(keys: np.ndarray):
    if keys.dtype != np.uint8 or keys.ndim != 2 or not keys.flags["C_CONTIGUOUS"]:
        raise ValueError("keys must be a C-contiguous uint8 array [n, keylen]")
    return keys.shape


def _host_ptr(a):
    """numpy array or (pinned) CPU torch tensor -> address."""
    if isinstance(a, np.ndarray):
        return C.c_void_p(a.ctypes.data)
    return C.c_void_p(a.data_ptr())


def city64_batch_host(keys, out=None, device: int = 0):
    """Host-resident keys (numpy uint8 [n, L] or pinned CPU tensor) -> uint64 [n]."""
    n, L = _host_keys(keys)
    if out is None:
        out = np.empty(n, dtype=np.uint64)
    _host_arr(out, "out", np.uint64, numel=n)
    _check(lib().pdht_city64_batch_host(_host_ptr(keys), L, n, _host_ptr(out), device),
           "pdht_city64_batch_host")
    return out


def city64_var_batch_host(data, offsets, out=None, device: int = 0):
    """Host-resident variable-length keys: data uint8 [nbytes], offsets [n+1]
    (uint64, or int64 with no negative entry -- numpy arrays and CPU tensors
    alike, viewed as uint64 without a copy so pinned buffers stay pinned)."""
    _host_arr(data, "data", np.uint8)
    if isinstance(offsets, np.ndarray) and offsets.dtype == np.int64:
        if offsets.size and int(offsets.min()) < 0:
            raise ValueError("offsets must not be negative")
        offsets = offsets.view(np.uint64)
    elif not isinstance(offsets, np.ndarray) and str(getattr(offsets, "dtype", "")) == "torch.int64":
        if offsets.numel() and int(offsets.min()) < 0:
            raise ValueError("offsets must not be negative")
    offsets = _host_arr(offsets, "offsets", np.uint64)
    n = offsets.size - 1 if isinstance(offsets, np.ndarray) else offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets must hold n+1 entries")
    if n:
        last = int(offsets[-1])
        nbytes = data.nbytes if isinstance(data, np.ndarray) else data.numel()
        if last > nbytes or int(offsets[0]) > last:
            raise ValueError(f"offsets reach byte {last}, data holds {nbytes}")
    if out is None:
        out = np.empty(n, dtype=np.uint64)
    _host_arr(out, "out", np.uint64, numel=n)
    _check(lib().pdht_city64_batch_var_host(_host_ptr(data), _host_ptr(offsets), n, _host_ptr(out), device),
           "pdht_city64_batch_var_host")
    return out


def citycrc128_batch_host(keys, out=None, device: int = 0):
    n, L = _host_keys(keys)
    if out is None:
        out = np.empty((n, 2), dtype=np.uint64)
    _host_arr(out, "out", np.uint64, numel=2 * n)
    _check(lib().pdht_citycrc128_batch_host(_host_ptr(keys), L, n, _host_ptr(out), device),
           "pdht_citycrc128_batch_host")
    return out


def place_batch_host(keys, nptes: int, nranks: int, device: int = 0, out=None):
    """Host-resident fused placement; `out` = (mbits uint64[n], ptindex
    uint32[n], rank uint32[n]) host arrays to fill (pinned ones, with pinned
    keys, take the zero-copy path)."""
    n, L = _host_keys(keys)
    if out is not None:
        mb, pt, rk = out
    else:
        mb = np.empty(n, dtype=np.uint64)
        pt = np.empty(n, dtype=np.uint32)
        rk = np.empty(n, dtype=np.uint32)
    _host_arr(mb, "mbits", np.uint64, numel=n)
    _host_arr(pt, "ptindex", np.uint32, numel=n)
    _host_arr(rk, "rank", np.uint32, numel=n)
    _check(lib().pdht_place_batch_host(_host_ptr(keys), L, n, nptes, nranks, _host_ptr(mb),
                                       _host_ptr(pt), _host_ptr(rk), 4, device),
           "pdht_place_batch_host")
    return mb, pt, rk


# ------------------------------------------------------- pdht_t mirror ---
class PdhtTable:
    """The hash-path view of a pdht table (pdht_create's keysize/nptes,
    init.c:80-94) over the stand-in pdht_t of include/pdht_hash.h.

    hash(key)            -> (mbits, ptindex, rank)       pdht_hash, hash.c:25-30
    sethash(fn)          -> install a plugin              pdht_sethash, hash.c:39-41
    hash_batch(keys)     -> arrays                        pdht_hash_batch (GPU or plugin)
    """

    def __init__(self, keysize: int, nptes: int = 1, nranks: int = 1):
        self._t = _PdhtT()
        lib().pdht_hip_table_init(C.byref(self._t), keysize, nptes)
        self.nranks = nranks
        self._plugin = None

    @property
    def keysize(self) -> int:
        return self._t.keysize

    @property
    def nptes(self) -> int:
        return self._t.nptes

    def _set_ranks(self):
        C.c_int.in_dll(lib(), "pdht_hip_shim_nranks").value = self.nranks

    def sethash(self, fn):
        """fn(table, key_bytes) -> (mbits, ptindex, rank) or a raw C function pointer."""
        if fn is None:
            lib().pdht_sethash(C.byref(self._t), C.cast(lib().pdht_hash, C.c_void_p))
            self._plugin = None
            return
        L = self.keysize

        def tramp(dht, key, mb, pt, rk):
            m, p, r = fn(self, C.string_at(key, L))
            mb[0] = m & 0xFFFFFFFFFFFFFFFF
            pt[0] = p & 0xFFFFFFFF
            rk[0].rank = r & 0xFFFFFFFF

        self._plugin = _HASHFUNC(tramp)
        lib().pdht_sethash(C.byref(self._t), C.cast(self._plugin, C.c_void_p))

    def hash(self, key: bytes):
        if len(key) < self.keysize:
            raise ValueError("key shorter than keysize")
        self._set_ranks()
        mb, pt, rk = C.c_uint64(), C.c_uint32(), PtlProcess()
        # dht->hashfn(dht, key, &mbits, &ptindex, &rank), as putget.c:53 calls it
        fn = _HASHFUNC(self._t.hashfn)
        fn(C.cast(C.byref(self._t), C.c_void_p), C.c_char_p(bytes(key)), C.byref(mb), C.byref(pt),
           C.byref(rk))
        return mb.value, pt.value, rk.rank

    def hash_batch(self, keys: np.ndarray, device: int = 0):
        """keys uint8 [n, keysize] (host) -> (mbits u64[n], ptindex u32[n], rank u32[n])."""
        n, L = _np_keys(keys)
        if L != self.keysize:
            raise ValueError("key width != keysize")
        self._set_ranks()
        mb = np.empty(n, dtype=np.uint64)
        pt = np.empty(n, dtype=np.uint32)
        rk = (PtlProcess * max(n, 1))()
        _check(lib().pdht_hash_batch(C.byref(self._t), _host_ptr(keys), n, _host_ptr(mb),
                                     _host_ptr(pt), C.cast(rk, C.c_void_p), device),
               "pdht_hash_batch")
        ranks = np.frombuffer(rk, dtype=np.uint32).reshape(-1, 2)[:n, 0].copy()
        return mb, pt, ranks
