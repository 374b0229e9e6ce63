#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ FROM THE REFERENCE ITSELF.

Runs only where /root/reference exists: it compiles the reference
libpdht/city.c from where it lies (oracle/Makefile -> oracle/_ref/) and calls
its CityHash64 / CityHash128 / CityHashCrc128 / CityHashCrc256 symbols.  Only
data (inputs are regenerated from documented patterns; outputs are digests)
is written; no reference source goes into the repo.

pdht_hash placement (libpdht/hash.c:25-30) cannot be compiled here (pdht.h
needs portals4.h), so its vectors are the reference CityHash64 digest plus
the two modulo reductions of hash.c:27 and :29 done in Python.

  python tests/golden/gen_golden.py          # small fixtures (seconds)
  python tests/golden/gen_golden.py --full   # + full-config fold checksums
  python tests/golden/gen_golden.py --extra  # + place/bucket/long folds (added)
  python tests/golden/gen_golden.py --r02    # + WeakHashLen32WithSeeds(6) vectors
  python tests/golden/gen_golden.py --bucket8k  # + 8192-rank bucketing folds
                                             #   and cfg1 pdht_hash placement folds (added)
  python tests/golden/gen_golden.py --multirank # + per-rank cfg1/cfg3/cfg4 folds of the
                                             #   N > 1 weak-scaling shards (added)
  python tests/golden/gen_golden.py --bucket-world  # + exchange/xrecords folds (nranks = N)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
M = 1 << 20

SEED64 = 0x0123456789ABCDEF
SEED128 = (0x0F1E2D3C4B5A6978, 0x8796A5B4C3D2E1F0)


def pattern_a(n: int) -> bytes:
    return bytes(i & 0xFF for i in range(n))


def pattern_b(n: int) -> bytes:
    return bytes((i * 7 + 3) & 0xFF for i in range(n))


def u128(r) -> tuple[int, int]:
    return r.first, r.second


def small(R) -> dict:
    out: dict[str, np.ndarray] = {}
    lens = np.arange(0, 1025, dtype=np.uint64)
    out["lens"] = lens
    for tag, pat in (("A", pattern_a), ("B", pattern_b)):
        buf = pat(1024)
        c64 = np.empty(1025, np.uint64)
        c128 = np.empty((1025, 2), np.uint64)
        crc128 = np.empty((1025, 2), np.uint64)
        for L in range(1025):
            c64[L] = R.CityHash64(buf, L)
            c128[L] = u128(R.CityHash128(buf, L))
            crc128[L] = u128(R.CityHashCrc128(buf, L))
        out[f"pat{tag}_city64"] = c64
        out[f"pat{tag}_city128"] = c128
        # CityHashCrc128 == CityHash128 for len <= 900 (city.c:492-493, :507-508);
        # that identity is asserted by the tests, only 901..1024 is stored.
        assert (crc128[:901] == c128[:901]).all()
        out[f"pat{tag}_crc128_901up"] = crc128[901:]
    # seeded variants and CRC-256 on pattern A (city.h:72-84, citycrc.h:39-46)
    buf = pattern_a(1024)
    s64 = np.empty(1025, np.uint64)
    s64s = np.empty(1025, np.uint64)
    s128 = np.empty((1025, 2), np.uint64)
    scrc = np.empty((1025, 2), np.uint64)
    crc256 = np.empty((1025, 4), np.uint64)
    seed = O.Uint128(*SEED128)
    for L in range(1025):
        s64[L] = R.CityHash64WithSeed(buf, L, SEED64)
        s64s[L] = R.CityHash64WithSeeds(buf, L, SEED128[0], SEED128[1])
        s128[L] = u128(R.CityHash128WithSeed(buf, L, seed))
        scrc[L] = u128(R.CityHashCrc128WithSeed(buf, L, seed))
        r4 = (C.c_uint64 * 4)()
        R.CityHashCrc256(buf, L, r4)
        crc256[L] = tuple(r4)
    out["patA_city64_seed"] = s64
    out["patA_city64_seeds"] = s64s
    out["patA_city128_seed"] = s128
    assert (scrc[:901] == s128[:901]).all()
    out["patA_crc128_seed_901up"] = scrc[901:]
    out["patA_crc256"] = crc256
    out["seed64"] = np.array([SEED64], np.uint64)
    out["seed128"] = np.array(SEED128, np.uint64)
    # long keys (CRC-256 long path, CityHash128 long loop)
    long_lens = np.array([1500, 2047, 2048, 4096, 10007], np.uint64)
    lb = pattern_b(int(long_lens.max()))
    out["long_lens"] = long_lens
    out["longB_city64"] = np.array([R.CityHash64(lb, int(L)) for L in long_lens], np.uint64)
    out["longB_city128"] = np.array([u128(R.CityHash128(lb, int(L))) for L in long_lens], np.uint64)
    out["longB_crc128"] = np.array([u128(R.CityHashCrc128(lb, int(L))) for L in long_lens], np.uint64)
    # splitmix64 stream head (pins the synthetic-key generator)
    out["splitmix_head"] = O.splitmix64(O.SEED_KEYS, 0, 64)
    out["splitmix_lens_head"] = O.splitmix64(O.SEED_LENS, 0, 64)
    # 1024 random 64-byte keys (the cfg2 workload's first keys)
    k64 = O.fixed_keys(1024, 64)
    out["rand64_city64"] = O.apply_ref64(k64, 1024, L=64, fn_name="CityHash64")
    out["rand64_city128"] = O.apply_ref128(k64, 1024, L=64, fn_name="CityHash128")
    assert (O.apply_ref128(k64, 1024, L=64, fn_name="CityHashCrc128") == out["rand64_city128"]).all()
    # 1024 mixed 16..256-byte keys (the cfg3 workload's first keys)
    data, offs = O.mixed_keys(1024)
    out["mixed_offsets"] = offs
    out["mixed_city64"] = O.apply_ref64(data, 1024, offsets=offs)
    out["mixed_city128"] = O.apply_ref128(data, 1024, offsets=offs, fn_name="CityHash128")
    assert (O.apply_ref128(data, 1024, offsets=offs, fn_name="CityHashCrc128")
            == out["mixed_city128"]).all()
    # pdht_hash on `unsigned long` keys 0..255 (test/scaling.c:137 key type)
    keys = np.arange(256, dtype=np.uint64).view(np.uint8).reshape(256, 8)
    mb = O.apply_ref64(keys, 256, L=8)
    out["pdht_u64keys_mbits"] = mb
    nptes = [1, 2, 3, 8]
    nranks = [1, 2, 3, 4, 7, 8, 64, 1000, 65537]
    out["pdht_nptes"] = np.array(nptes, np.uint64)
    out["pdht_nranks"] = np.array(nranks, np.uint64)
    out["pdht_ptindex"] = np.stack([(mb % np.uint64(p)).astype(np.uint32) for p in nptes])
    out["pdht_rank"] = np.stack([(mb % np.uint64(r)).astype(np.uint32) for r in nranks])
    return out


def folds_full(R) -> dict:
    """Fold checksums (sum d_i*(2i+1) mod 2^64) of the full BASELINE configs,
    per 1/8 shard so every world size 1/2/4/8 can check its own slice."""
    res = {}
    thr = os.cpu_count() or 8

    def fixed_fold(n, L, fn, name, shards=8, is128=False):
        per = n // shards
        parts = []
        chunk = 16 * M
        chunks = []  # fold of every 16M-key chunk (weak-scaling shards of bench.py)
        for s in range(shards):
            acc = 0
            for k0 in range(s * per, (s + 1) * per, chunk):
                cnt = min(chunk, (s + 1) * per - k0)
                keys = O.fixed_keys(cnt, L, first_key=k0)
                if is128:
                    d = O.apply_ref128(keys, cnt, L=L, threads=thr, fn_name=fn)
                    # fold over the interleaved {lo,hi} array, index 2i and 2i+1
                    f = O.fold64(d.reshape(-1), 2 * k0)
                else:
                    d = O.apply_ref64(keys, cnt, L=L, threads=thr, fn_name=fn)
                    f = O.fold64(d, k0)
                chunks.append(f)
                acc = (acc + f) % (1 << 64)
            parts.append(acc)
            print(f"  {name} shard {s}: {acc:016x}", flush=True)
        res[name] = {"n": n, "L": L, "shards": [f"{p:016x}" for p in parts],
                     "total": f"{sum(parts) % (1 << 64):016x}"}
        if n > chunk:
            res[name]["chunk_keys"] = chunk
            res[name]["chunks"] = [f"{c:016x}" for c in chunks]

    fixed_fold(1 * M, 64, "CityHash64", "cfg1_city64_1M_x64", shards=1)
    fixed_fold(16 * M, 64, "CityHash64", "cfg2_city64_16M_x64")
    fixed_fold(16 * M, 64, "CityHashCrc128", "cfg4_crc128_16M_x64", is128=True)
    # cfg3: 64M mixed 16..256 B keys
    n = 64 * M
    data, offs = O.mixed_keys(n)
    d = O.apply_ref64(data, n, offsets=offs, threads=thr)
    per = n // 8
    parts = [O.fold64(d[s * per:(s + 1) * per], s * per) for s in range(8)]
    res["cfg3_city64_64M_mixed"] = {"n": n, "lo": 16, "hi": 256, "total_bytes": int(offs[-1]),
                                    "shards": [f"{p:016x}" for p in parts],
                                    "total": f"{sum(parts) % (1 << 64):016x}"}
    del data, offs, d
    fixed_fold(1 << 30, 64, "CityHash64", "cfg5_city64_1B_x64")
    return res


def folds_extra() -> dict:
    """Folds for the bench's secondary configs, per 16M-key weak-scaling shard
    r = 0..7 (keys [r*16M, (r+1)*16M) of the stream), from the reference
    CityHash64 / CityHashCrc128 plus hash.c:27/:29's two reductions:
      place  (8-B keys, nptes 3, nranks 1024): folds of mbits, ptindex, rank
             and the rank histogram;
      bucket (8-B keys, nptes 3, nranks 1024): the stable bucketing of the
             shard: folds of the bucketed mbits, of the original indices and
             of the bucket offsets;
      long   (1M x 1 KiB keys, CityHashCrc128 > 900 B = CityHashCrc256 path):
             fold per shard of 1M keys."""
    thr = os.cpu_count() or 8
    res = {"place_8B_16M": {"n": 16 * M, "L": 8, "nptes": 3, "nranks": 1024, "shards": []},
           "bucket_8B_16M": {"n": 16 * M, "L": 8, "nptes": 3, "nranks": 1024, "shards": []},
           "long_crc128_1M_x1024": {"n": M, "L": 1024, "shards": []}}
    n = 16 * M
    for r in range(8):
        keys = O.fixed_keys(n, 8, first_key=r * n)
        m = O.apply_ref64(keys, n, L=8, threads=thr)
        pt = (m % np.uint64(3)).astype(np.uint64)
        rk = (m % np.uint64(1024)).astype(np.uint64)
        hist = np.bincount(rk.astype(np.int64), minlength=1024).astype(np.uint64)
        res["place_8B_16M"]["shards"].append({
            "mbits": f"{O.fold64(m, r * n):016x}", "ptindex": f"{O.fold64(pt, r * n):016x}",
            "rank": f"{O.fold64(rk, r * n):016x}", "hist": f"{O.fold64(hist, 0):016x}"})
        order = np.argsort(rk, kind="stable")
        offs = np.zeros(1025, np.uint64)
        np.cumsum(hist, out=offs[1:])
        res["bucket_8B_16M"]["shards"].append({
            "mbits": f"{O.fold64(m[order], 0):016x}", "index": f"{O.fold64(order.astype(np.uint64), 0):016x}",
            "offsets": f"{O.fold64(offs, 0):016x}"})
        print(f"  place/bucket shard {r} done", flush=True)
    nl = M
    for r in range(8):
        keys = O.fixed_keys(nl, 1024, first_key=r * nl)
        d = O.apply_ref128(keys, nl, L=1024, threads=thr, fn_name="CityHashCrc128")
        res["long_crc128_1M_x1024"]["shards"].append(f"{O.fold64(d.reshape(-1), 2 * r * nl):016x}")
        print(f"  long shard {r} done", flush=True)
    return res


def folds_bucket8k() -> dict:
    """bucket8k (8-B keys, nptes 3, nranks 8192: the two-pass bucketing path),
    per 16M-key shard r = 0..7: folds of the stably bucketed mbits, of the
    original indices and of the bucket offsets, from the reference CityHash64
    plus hash.c:29's reduction."""
    thr = os.cpu_count() or 8
    res = {"n": 16 * M, "L": 8, "nptes": 3, "nranks": 8192, "shards": []}
    n = 16 * M
    for r in range(8):
        keys = O.fixed_keys(n, 8, first_key=r * n)
        m = O.apply_ref64(keys, n, L=8, threads=thr)
        rk = (m % np.uint64(8192)).astype(np.int64)
        order = np.argsort(rk, kind="stable")
        offs = np.zeros(8193, np.uint64)
        np.cumsum(np.bincount(rk, minlength=8192).astype(np.uint64), out=offs[1:])
        res["shards"].append({"mbits": f"{O.fold64(m[order], 0):016x}",
                              "index": f"{O.fold64(order.astype(np.uint64), 0):016x}",
                              "offsets": f"{O.fold64(offs, 0):016x}"})
        print(f"  bucket8k shard {r} done", flush=True)
    return res


def folds_bucket_world() -> dict:
    """exchange / xrecords at N ranks bucket each rank's 16M-key shard by
    CityHash64 % N (nranks = world size, nptes 3): for N in 1, 2, 4, 8 and
    every shard r < N, folds of the stably bucketed mbits, of the original
    indices and of the bucket offsets (the same fields as folds_bucket8k)."""
    thr = os.cpu_count() or 8
    worlds = (1, 2, 4, 8)
    res = {f"bucket_8B_16M_{w}": {"n": 16 * M, "L": 8, "nptes": 3, "nranks": w, "shards": []} for w in worlds}
    n = 16 * M
    for r in range(max(worlds)):
        m = O.apply_ref64(O.fixed_keys(n, 8, first_key=r * n), n, L=8, threads=thr)
        for w in worlds:
            if r >= w:
                continue
            rk = (m % np.uint64(w)).astype(np.int64)
            order = np.argsort(rk, kind="stable")
            offs = np.zeros(w + 1, np.uint64)
            np.cumsum(np.bincount(rk, minlength=w).astype(np.uint64), out=offs[1:])
            res[f"bucket_8B_16M_{w}"]["shards"].append({
                "mbits": f"{O.fold64(m[order], 0):016x}",
                "index": f"{O.fold64(order.astype(np.uint64), 0):016x}",
                "offsets": f"{O.fold64(offs, 0):016x}"})
        print(f"  bucket-by-world shard {r} done", flush=True)
    return res


def r02_vectors(R) -> dict:
    """WeakHashLen32WithSeeds6 / WeakHashLen32WithSeeds (city.c:173-198;
    exported by the reference although city.h does not declare them) on
    splitmix64 inputs."""
    R.WeakHashLen32WithSeeds6.restype = O.Uint128
    R.WeakHashLen32WithSeeds6.argtypes = [C.c_uint64] * 6
    R.WeakHashLen32WithSeeds.restype = O.Uint128
    R.WeakHashLen32WithSeeds.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64]
    nv = 256
    w6 = O.splitmix64(0xFEEDFACE, 0, nv * 6).reshape(nv, 6)
    o6 = np.array([u128(R.WeakHashLen32WithSeeds6(*(int(x) for x in row))) for row in w6], np.uint64)
    b32 = O.splitmix64(0xFEEDFACE, 10_000, nv * 4).view(np.uint8).reshape(nv, 32)
    sd = O.splitmix64(0xFEEDFACE, 20_000, nv * 2).reshape(nv, 2)
    o32 = np.array([u128(R.WeakHashLen32WithSeeds(C.c_char_p(b32[i].tobytes()), int(sd[i, 0]), int(sd[i, 1])))
                    for i in range(nv)], np.uint64)
    return {"weak6_in": w6, "weak6_out": o6, "weak32_bytes": b32, "weak32_seeds": sd, "weak32_out": o32}


CFG1_PLACEMENTS = [(1, 4), (1, 1), (3, 1000), (8, 7)]  # (nptes, nranks): pdht default 1 PTE, 4 ranks


def cfg1_folds() -> dict:
    """cfg1 (BASELINE configs[0]: 1M x 64 B through hash.c -> CityHash64): the
    reference CityHash64 of every key plus hash.c:27/:29's reductions, for a
    few (nptes, nranks); folds of mbits, ptindex, rank and the per-rank
    histogram (putget.c:55's rankputs)."""
    n, L = M, 64
    keys = O.fixed_keys(n, L)
    m = O.apply_ref64(keys, n, L=L, threads=os.cpu_count() or 8)
    res = {"n": n, "L": L, "mbits": f"{O.fold64(m, 0):016x}", "placements": []}
    for p, r in CFG1_PLACEMENTS:
        pt = (m % np.uint64(p)).astype(np.uint64)
        rk = (m % np.uint64(r)).astype(np.uint64)
        hist = np.bincount(rk.astype(np.int64), minlength=r).astype(np.uint64)
        res["placements"].append({"nptes": p, "nranks": r, "ptindex": f"{O.fold64(pt, 0):016x}",
                                  "rank": f"{O.fold64(rk, 0):016x}", "hist": f"{O.fold64(hist, 0):016x}"})
    return res


def folds_multirank(ranks: int = 8) -> dict:
    """Per-rank folds of the bench's weak-scaling shards at N > 1, for every
    rank r < 8 (so every world size 1/2/4/8 can check each of its ranks):
      cfg3  rank r: 64M mixed keys, lengths from the lengths stream at key
            r*64M, bytes from the key stream at word r << 40 (bench.py's
            disjoint segment); fold at global index r*64M;
      cfg4  rank r: keys [r*16M, (r+1)*16M), CityHashCrc128, fold over the
            interleaved {lo,hi} array at index 2*r*16M;
      cfg1  rank r: keys [r*1M, (r+1)*1M), pdht_hash with nptes 1, nranks 4:
            folds of mbits, ptindex, rank (global index) and the histogram."""
    thr = os.cpu_count() or 8
    out = {"cfg3": [], "cfg4": [], "cfg1": []}
    n3 = 64 * M
    for r in range(ranks):
        lens = O.mixed_lengths(n3, first_key=r * n3)
        offs = np.zeros(n3 + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        del lens
        total = int(offs[-1])
        data = O.splitmix64(O.SEED_KEYS, r << 40, (total + 7) // 8).view(np.uint8)[:total]
        d = O.apply_ref64(data, n3, offsets=offs, threads=thr)
        out["cfg3"].append({"total_bytes": total, "fold": f"{O.fold64(d, r * n3):016x}"})
        del data, offs, d
        print(f"  cfg3 rank {r}: {out['cfg3'][-1]}", flush=True)
    n4 = 16 * M
    for r in range(ranks):
        keys = O.fixed_keys(n4, 64, first_key=r * n4)
        d = O.apply_ref128(keys, n4, L=64, threads=thr, fn_name="CityHashCrc128")
        out["cfg4"].append(f"{O.fold64(d.reshape(-1), 2 * r * n4):016x}")
        print(f"  cfg4 rank {r}: {out['cfg4'][-1]}", flush=True)
    n1 = M
    for r in range(ranks):
        keys = O.fixed_keys(n1, 64, first_key=r * n1)
        m = O.apply_ref64(keys, n1, L=64, threads=thr)
        pt = (m % np.uint64(1)).astype(np.uint64)
        rk = (m % np.uint64(4)).astype(np.uint64)
        hist = np.bincount(rk.astype(np.int64), minlength=4).astype(np.uint64)
        out["cfg1"].append({"mbits": f"{O.fold64(m, r * n1):016x}", "ptindex": f"{O.fold64(pt, r * n1):016x}",
                            "rank": f"{O.fold64(rk, r * n1):016x}", "hist": f"{O.fold64(hist, 0):016x}"})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--extra", action="store_true",
                    help="add the place/bucket/long folds to config_folds.json")
    ap.add_argument("--r02", action="store_true",
                    help="add the WeakHash vectors (npz) and the cfg1 placement folds (json)")
    ap.add_argument("--bucket8k", action="store_true",
                    help="add the 8192-rank bucketing folds (json)")
    ap.add_argument("--bucket-world", action="store_true",
                    help="add the nranks = world-size bucketing folds of exchange/xrecords (json)")
    ap.add_argument("--multirank", action="store_true",
                    help="add per-rank cfg1/cfg3/cfg4 folds of the N > 1 weak-scaling shards (json)")
    a = ap.parse_args()
    O.build()
    R = O.ref()
    if R is None:
        sys.exit("oracle/_ref not built: /root/reference is required to regenerate fixtures")
    if a.multirank:
        path = os.path.join(HERE, "config_folds.json")
        with open(path) as f:
            doc = json.load(f)
        mr = folds_multirank()
        doc["configs"]["cfg3_city64_64M_mixed"]["ranks"] = mr["cfg3"]
        doc["configs"]["cfg4_crc128_16M_x64"]["rank_chunks"] = mr["cfg4"]
        doc["configs"]["cfg1_pdht_hash_1M_x64"]["ranks"] = mr["cfg1"]
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print("added per-rank cfg1/cfg3/cfg4 folds")
        return
    if a.bucket_world:
        path = os.path.join(HERE, "config_folds.json")
        with open(path) as f:
            doc = json.load(f)
        doc["configs"].update(folds_bucket_world())
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print("added nranks = world bucketing folds")
        return
    if a.bucket8k:
        path = os.path.join(HERE, "config_folds.json")
        with open(path) as f:
            doc = json.load(f)
        doc["configs"]["bucket_8B_16M_8192"] = folds_bucket8k()
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print("added bucket8k folds")
        return
    if a.r02:
        npz = os.path.join(HERE, "city_golden.npz")
        with np.load(npz, allow_pickle=False) as z:
            vec = {k: z[k] for k in z.files}
        vec.update(r02_vectors(R))
        np.savez_compressed(npz, **vec)
        path = os.path.join(HERE, "config_folds.json")
        with open(path) as f:
            doc = json.load(f)
        doc["configs"]["cfg1_pdht_hash_1M_x64"] = cfg1_folds()
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print("added WeakHash vectors and cfg1 placement folds")
        return
    if a.extra:
        path = os.path.join(HERE, "config_folds.json")
        with open(path) as f:
            doc = json.load(f)
        doc["configs"].update(folds_extra())
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print("added place/bucket/long folds to config_folds.json")
        return
    vec = small(R)
    np.savez_compressed(os.path.join(HERE, "city_golden.npz"), **vec)
    print("wrote city_golden.npz", os.path.getsize(os.path.join(HERE, "city_golden.npz")), "bytes")
    if a.full:
        res = folds_full(R)
        with open(os.path.join(HERE, "config_folds.json"), "w") as f:
            json.dump({"generator": "tests/golden/gen_golden.py --full (reference city.c via oracle/_ref)",
                       "key_seed": f"{O.SEED_KEYS:016x}", "len_seed": f"{O.SEED_LENS:016x}",
                       "fold": "sum_i d_i*(2i+1) mod 2^64 over global key index i "
                               "(128-bit digests: over the interleaved lo,hi array)",
                       "configs": res}, f, indent=1)
        print("wrote config_folds.json")


if __name__ == "__main__":
    main()
