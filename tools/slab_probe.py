#!/usr/bin/env python3
"""Does the allocation a key buffer lives in change the 64-B stream's rate?

BASELINE configs[4] (1B keys in one 64 GiB allocation) has measured up to 5 %
above cfg2 (16M keys in a 1 GiB allocation) with the same kernel and launch
shape.  This times cfg2's step (CityHash64 of 16M x 64 B, 2 launches of
512 MiB) on the same keys placed at the start of allocations of 1 / 8 / 16 /
32 / 64 GiB, interleaved round by round in one process, after an Infinity
Cache flush per round.

  python tools/slab_probe.py [--rounds 7] [--reps 20] [--sizes 1,8,16,32,64]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pdht_amd as P  # noqa: E402

SEED = 0x5EED5EED5EED5EED
G = 1 << 30


def cfg3(a, dev):
    """cfg3 (64M mixed 16..256 B, offset-indexed): its own allocations against
    the same bytes, offsets and digests carved from one 16 / 32 GiB slab."""
    n = 64 << 20
    lens = P.mixed_lengths(0x1E575EED1E575EED, 0, n, 16, 256, device=dev)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    del lens
    total = int(offs[-1].item())
    data = P.splitmix64_fill(SEED, 0, (total + 7) // 8, device=dev).view(torch.uint8)[:total]
    out = torch.empty(n, dtype=torch.int64, device=dev)
    ref = P.city64_var_batch(data, offs, out=torch.empty_like(out))
    sets = {0: (data, offs, out)}
    for gib in (int(x) for x in a.sizes.split(",") if int(x) >= 16):
        slab = torch.empty(gib * G, dtype=torch.uint8, device=dev)
        d = slab[:total]
        d.copy_(data)
        o0 = (total + (2 << 20)) & ~((2 << 20) - 1)
        of = slab[o0:o0 + (n + 1) * 8].view(torch.int64)
        of.copy_(offs)
        o1 = (o0 + (n + 1) * 8 + (2 << 20)) & ~((2 << 20) - 1)
        ou = slab[o1:o1 + n * 8].view(torch.int64)
        sets[gib] = (d, of, ou, slab)
    scratch = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    res = {g: [] for g in sets}
    for _ in range(a.rounds):
        for g, st in sets.items():
            d, of, ou = st[0], st[1], st[2]
            scratch.fill_(1)
            P.city64_var_batch(d, of, out=ou, check=False)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(max(1, a.reps // 4)):
                P.city64_var_batch(d, of, out=ou, check=False)
            e1.record()
            torch.cuda.synchronize()
            res[g].append(e0.elapsed_time(e1) / max(1, a.reps // 4))
    for g, st in sets.items():
        med = float(np.median(res[g]))
        print(json.dumps({"work": "cfg3", "alloc_GiB": g or "own", "ok": bool(torch.equal(st[2], ref)),
                          "median_ms": round(med, 4),
                          "frac_8TBps": round((total + 16 * n) / (med / 1e3) / 1e9 / 8000, 4)}), flush=True)


def hip_buffer(nbytes, flags, dev):
    """A uint8 CUDA tensor over hipExtMallocWithFlags(flags) memory (probe
    only: never freed)."""
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    ptr = C.c_void_p()
    rc = hip.hipExtMallocWithFlags(C.byref(ptr), C.c_size_t(nbytes), C.c_uint(flags))
    if rc != 0:
        raise RuntimeError(f"hipExtMallocWithFlags({nbytes}, {flags}) -> {rc}")

    class Buf:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr.value, False),
                                    "version": 3, "strides": None}
    return torch.as_tensor(Buf(), device=dev)


def contiguous(a, dev):
    """cfg2 on 1 GiB key buffers from hipMalloc (torch) and from
    hipExtMallocWithFlags(hipDeviceMallocContiguous), three of each, interleaved."""
    n = 16 << 20
    words = P.splitmix64_fill(SEED, 0, n * 8, device=dev)
    ref = P.city64_batch(words.view(torch.uint8).view(n, 64))
    bufs = {}
    for j, kind in enumerate(a.kinds.split(",")):
        if kind == "torch":
            b = torch.empty(n * 64, dtype=torch.uint8, device=dev)
        else:
            b = hip_buffer(n * 64, {"contig": 4, "default": 0}[kind], dev)
        b.copy_(words.view(torch.uint8))
        bufs[(j, kind)] = (b, b.view(n, 64), torch.empty(n, dtype=torch.int64, device=dev))
    scratch = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    res = {g: [] for g in bufs}
    for _ in range(a.rounds):
        for g, (_, keys, out) in bufs.items():
            scratch.fill_(1)
            P.city64_batch(keys, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                P.city64_batch(keys, out=out)
            e1.record()
            torch.cuda.synchronize()
            res[g].append(e0.elapsed_time(e1) / a.reps)
    for g, (b, _, out) in bufs.items():
        med = float(np.median(res[g]))
        print(json.dumps({"alloc": g[1], "order": g[0], "ok": bool(torch.equal(out, ref)), "va": hex(b.data_ptr()),
                          "median_ms": round(med, 4),
                          "frac_8TBps": round(n * 72 / (med / 1e3) / 1e9 / 8000, 4)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--sizes", default="1,8,16,32,64")
    ap.add_argument("--work", default="cfg2", choices=["cfg2", "cfg3", "contig"])
    ap.add_argument("--kinds", default="torch,contig,torch,contig,default,contig")
    ap.add_argument("--keys-m", type=int, default=16, help="cfg2: millions of 64-B keys (128 = cfg5)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.work == "cfg3":
        cfg3(a, dev)
        return
    if a.work == "contig":
        contiguous(a, dev)
        return
    n = a.keys_m << 20
    words = P.splitmix64_fill(SEED, 0, n * 8, device=dev)
    ref = P.city64_batch(words.view(torch.uint8).view(n, 64))
    bufs = {}
    for j, gib in enumerate(int(x) for x in a.sizes.split(",")):  # in allocation order
        slab = torch.empty(gib * G, dtype=torch.uint8, device=dev)
        keys = slab[:n * 64].view(n, 64)
        keys.view(-1).copy_(words.view(torch.uint8))
        bufs[(j, gib)] = (slab, keys, torch.empty(n, dtype=torch.int64, device=dev))
    del words
    scratch = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    res = {g: [] for g in bufs}
    for _ in range(a.rounds):
        for g, (_, keys, out) in bufs.items():
            scratch.fill_(1)  # Infinity Cache flush
            P.city64_batch(keys, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                P.city64_batch(keys, out=out)
            e1.record()
            torch.cuda.synchronize()
            res[g].append(e0.elapsed_time(e1) / a.reps)
    for g, (_, _, out) in bufs.items():
        ok = bool(torch.equal(out, ref))
        med = float(np.median(res[g]))
        print(json.dumps({"keys_M": a.keys_m, "alloc_order": g[0], "alloc_GiB": g[1], "ok": ok,
                          "va": hex(bufs[g][0].data_ptr()), "median_ms": round(med, 4),
                          "frac_8TBps": round(n * 72 / (med / 1e3) / 1e9 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    main()
