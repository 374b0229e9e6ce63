"""CPU-side checks of the product library (no GPU needed).

* libpdht_hip.so loads and exports every function include/*.h declares;
* the scalar city.h / citycrc.h API (same city_core.h the kernels run) is
  bit-exact against the reference golden vectors;
* pdht_hash / pdht_sethash through the stand-in pdht_t (hash.c:25-41),
  including a user plugin (test/scaling.c:39-43 style identity hash);
* batch entry points fail loudly (no CPU fallback) when no GPU is usable.
"""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, pattern_a, pattern_b

import pdht_amd as P


def _declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"#ifdef PDHT_HIP_WITH_REAL_PDHT.*?#else", "", src, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{)]*\)\s*;", src)
    return {n for n in names if not n.startswith("pdht_hashfunc") and n not in ("defined",)}


def test_library_exports_every_declared_symbol():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", P.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    want = set()
    for h in ("pdht_hip.h", "pdht_city.h", "pdht_hash.h"):
        want |= _declared(h)
    assert len(want) == 44, sorted(want)
    missing = sorted(want - exported)
    assert not missing, missing
    lib = P.lib()
    for name in want:
        getattr(lib, name)  # resolvable through the loader too
    assert "gfx950" in lib.pdht_hip_version().decode()


def test_scalar_city_api(golden):
    for tag, pat in (("A", pattern_a), ("B", pattern_b)):
        buf = pat(1024)
        for L in range(1025):
            assert P.CityHash64(buf[:L]) == int(golden[f"pat{tag}_city64"][L]), (tag, L)
            assert P.CityHash128(buf[:L]) == tuple(int(x) for x in golden[f"pat{tag}_city128"][L])
            want = golden[f"pat{tag}_city128"][L] if L <= 900 else golden[f"pat{tag}_crc128_901up"][L - 901]
            assert P.CityHashCrc128(buf[:L]) == tuple(int(x) for x in want), (tag, L)


def test_scalar_seeded_crc256_long(golden):
    buf = pattern_a(1024)
    s64 = int(golden["seed64"][0])
    lo, hi = (int(x) for x in golden["seed128"])
    for L in range(1025):
        assert P.CityHash64WithSeed(buf[:L], s64) == int(golden["patA_city64_seed"][L])
        assert P.CityHash64WithSeeds(buf[:L], lo, hi) == int(golden["patA_city64_seeds"][L])
        assert P.CityHash128WithSeed(buf[:L], (lo, hi)) == tuple(int(x) for x in golden["patA_city128_seed"][L])
        want = golden["patA_city128_seed"][L] if L <= 900 else golden["patA_crc128_seed_901up"][L - 901]
        assert P.CityHashCrc128WithSeed(buf[:L], (lo, hi)) == tuple(int(x) for x in want)
        assert P.CityHashCrc256(buf[:L]) == tuple(int(x) for x in golden["patA_crc256"][L])
    lens = [int(x) for x in golden["long_lens"]]
    lb = pattern_b(max(lens))
    for j, L in enumerate(lens):
        assert P.CityHash64(lb[:L]) == int(golden["longB_city64"][j])
        assert P.CityHash128(lb[:L]) == tuple(int(x) for x in golden["longB_city128"][j])
        assert P.CityHashCrc128(lb[:L]) == tuple(int(x) for x in golden["longB_crc128"][j])


def test_scalar_vs_oracle_random(oracle):
    rng = np.random.default_rng(11)
    for L in list(range(0, 260)) + [1000, 4099]:
        d = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        assert P.CityHash64(d) == oracle.city64(d)
        assert P.CityHashCrc128(d) == oracle.citycrc128(d)


def test_pdht_hash_scalar(golden):
    keys = np.arange(256, dtype=np.uint64).view(np.uint8).reshape(256, 8)
    for a, p in enumerate(golden["pdht_nptes"]):
        for b, r in enumerate(golden["pdht_nranks"]):
            t = P.PdhtTable(keysize=8, nptes=int(p), nranks=int(r))
            for i in range(0, 256, 17):
                m, pt, rk = t.hash(keys[i].tobytes())
                assert m == int(golden["pdht_u64keys_mbits"][i])
                assert pt == int(golden["pdht_ptindex"][a][i])
                assert rk == int(golden["pdht_rank"][b][i])


def test_sethash_plugin_scalar_and_batch_on_cpu():
    # identity plugin, test/scaling.c:39-43
    t = P.PdhtTable(keysize=8, nptes=3, nranks=4)

    def ahash(tab, key):
        k = int.from_bytes(key, "little")
        return k, k % tab.nptes, k % tab.nranks

    t.sethash(ahash)
    assert t.hash((10).to_bytes(8, "little")) == (10, 1, 2)
    keys = np.arange(100, dtype=np.uint64).view(np.uint8).reshape(100, 8)
    mb, pt, rk = t.hash_batch(keys)  # plugin path: per-key on the CPU, no GPU needed
    assert (mb == np.arange(100)).all()
    assert (pt == np.arange(100) % 3).all()
    assert (rk == np.arange(100) % 4).all()
    t.sethash(None)  # back to pdht_hash
    assert t.hash((0).to_bytes(8, "little"))[0] == 0xD7C06285B9DE677A


def test_batch_fails_loudly_without_gpu():
    if P.device_count() > 0:
        pytest.skip("a GPU is present")
    keys = np.zeros((10, 64), dtype=np.uint8)
    with pytest.raises(P.PdhtError):
        P.city64_batch_host(keys)
    t = P.PdhtTable(keysize=8)
    with pytest.raises(P.PdhtError):
        t.hash_batch(np.zeros((4, 8), dtype=np.uint8))
