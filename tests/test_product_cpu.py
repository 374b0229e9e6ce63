"""CPU-side checks of the product library (no GPU needed).

* libpdht_hip.so loads and exports every function include/*.h declares;
* the scalar city.h / citycrc.h API (same city_core.h the kernels run) is
  bit-exact against the reference golden vectors;
* pdht_hash / pdht_sethash through the stand-in pdht_t (hash.c:25-41),
  including a user plugin (test/scaling.c:39-43 style identity hash);
* batch entry points fail loudly (no CPU fallback) when no GPU is usable;
* cfg1 (BASELINE configs[0], 1M x 64 B through hash.c -> CityHash64): the
  product's scalar pdht_hash over the whole config against the reference's
  golden folds, for both the libpdht and the libmpipdht flavour;
* the tuning entry points live only in the tuning build;
* the host wrappers reject bad buffers before C sees them.
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
    # the reference city.c's exported symbols, all of them (link-level drop-in)
    ref = os.path.join(ROOT, "oracle", "_ref", "libcityref.so")
    if os.path.exists(ref):
        rsyms = {ln.split()[-1] for ln in subprocess.run(["nm", "-D", "--defined-only", ref],
                                                          capture_output=True, text=True,
                                                          check=True).stdout.splitlines()
                 if " T " in ln}
        assert rsyms and not (rsyms - exported), sorted(rsyms - exported)


def _exports(path):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


TUNING_SYMS = {"pdht_hip_set_variant", "pdht_hip_set_blocks_per_cu"}


def test_tuning_entry_points_only_in_tuning_build():
    """The product has one kernel per path and no process-global knobs: no
    variant / per-CU / phase-counter entry points; the tuning build (tools,
    A/B tests) has them."""
    prod = _exports(P.LIB_PATH)
    assert not (TUNING_SYMS & prod)
    assert not {s for s in prod if "phase" in s or "variant" in s or "hint" in s}
    assert TUNING_SYMS <= _exports(P.TUNING_LIB_PATH)
    src = open(os.path.join(ROOT, "pdht_amd", "csrc", "pdht_hip.hip")).read()
    assert "getenv" not in src


def test_product_sources_carry_no_tuning_code():
    """the A/B alternatives live in pdht_amd/csrc/tuning/
    and reach the sources only through the "pdht_hooks*.h" headers, which the
    product build takes from pdht_amd/csrc/product/ (every hook a no-op): no
    product source or header names the tuning build, its variant state or a
    tuning header, and every product hook header has a tuning counterpart."""
    csrc = os.path.join(ROOT, "pdht_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".hip", ".h")) and f != "pdht_hip_tuning.h":
            src = open(os.path.join(csrc, f)).read()
            for word in ("PDHT_HIP_TUNING", "tuning_variant", "\"tuning/", "kernels_tuning"):
                assert word not in src, (f, word)
    prod = sorted(os.listdir(os.path.join(csrc, "product")))
    assert prod and all(h.startswith("pdht_hooks") for h in prod)
    assert set(prod) <= set(os.listdir(os.path.join(csrc, "tuning")))
    for h in prod:
        assert "tuning_variant" not in open(os.path.join(csrc, "product", h)).read()


def test_weakhash_exports(golden):
    """WeakHashLen32WithSeeds(6) (city.c:173-198): exported by the reference
    although city.h omits them; pinned by vectors from the reference."""
    for row, want in zip(golden["weak6_in"], golden["weak6_out"]):
        assert P.WeakHashLen32WithSeeds6(*(int(x) for x in row)) == tuple(int(x) for x in want)
    for b, sd, want in zip(golden["weak32_bytes"], golden["weak32_seeds"], golden["weak32_out"]):
        assert P.WeakHashLen32WithSeeds(b.tobytes(), int(sd[0]), int(sd[1])) == tuple(int(x) for x in want)


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


def _cfg1_run(libpath, oracle, folds, nptes, nranks):
    """The scalar pdht_hash of `libpath` called once per key over cfg1's 1M x
    64 B keys (C loop: oracle.apply_hashfn drives the function pointer)."""
    import ctypes as C
    L = C.CDLL(libpath)
    L.pdht_hip_table_init.argtypes = [C.c_void_p, C.c_uint, C.c_uint]
    t = P._PdhtT()
    L.pdht_hip_table_init(C.byref(t), 64, nptes)
    C.c_int.in_dll(L, "pdht_hip_shim_nranks").value = nranks
    f = folds["cfg1_pdht_hash_1M_x64"]
    keys = oracle.fixed_keys(f["n"], 64)
    return oracle.apply_hashfn(C.cast(L.pdht_hash, C.c_void_p).value, C.addressof(t), keys), f


def test_cfg1_pdht_hash_1M_x64(oracle, folds):
    """BASELINE configs[0]: 1M x 64 B keys through hash.c -> CityHash64
    (libpdht/hash.c:25-30), the product's scalar pdht_hash per key, against
    folds the reference city.c produced (gen_golden.py --r02)."""
    for pl in folds["cfg1_pdht_hash_1M_x64"]["placements"]:
        (m, pt, rk), f = _cfg1_run(P.LIB_PATH, oracle, folds, pl["nptes"], pl["nranks"])
        assert f"{oracle.fold64(m, 0):016x}" == f["mbits"] == folds["cfg1_city64_1M_x64"]["total"]
        assert f"{oracle.fold64(pt.astype(np.uint64), 0):016x}" == pl["ptindex"]
        assert f"{oracle.fold64(rk.astype(np.uint64), 0):016x}" == pl["rank"]
        hist = np.bincount(rk, minlength=pl["nranks"]).astype(np.uint64)
        assert f"{oracle.fold64(hist, 0):016x}" == pl["hist"]


def test_mpi_flavour_pdht_hash(oracle, folds):
    """libmpipdht/hash.c:6-9: same mbits and rank = mbits % c->size, ptindex
    left untouched (the library built with -DPDHT_HIP_MPI_FLAVOUR)."""
    pl = folds["cfg1_pdht_hash_1M_x64"]["placements"][2]
    (m, pt, rk), f = _cfg1_run(P.MPI_LIB_PATH, oracle, folds, pl["nptes"], pl["nranks"])
    assert f"{oracle.fold64(m, 0):016x}" == f["mbits"]
    assert (pt == 0xFFFFFFFF).all()  # never written
    assert (rk.astype(np.uint64) == m % np.uint64(pl["nranks"])).all()
    assert f"{oracle.fold64(rk.astype(np.uint64), 0):016x}" == pl["rank"]
    # and the libpdht flavour does write it
    (_, pt2, _), _ = _cfg1_run(P.LIB_PATH, oracle, folds, pl["nptes"], pl["nranks"])
    assert f"{oracle.fold64(pt2.astype(np.uint64), 0):016x}" == pl["ptindex"]


def test_host_wrappers_reject_bad_buffers():
    """Checked before the C call (no GPU needed): wrong dtype, strided views,
    short outputs and offsets past the data raise ValueError."""
    k = np.zeros((10, 64), np.uint8)
    with pytest.raises(ValueError):
        P.city64_batch_host(k[:, :8])  # strided view
    with pytest.raises(ValueError):
        P.city64_batch_host(k.view(np.int8))
    with pytest.raises(ValueError):
        P.city64_batch_host(k, out=np.empty(9, np.uint64))
    with pytest.raises(ValueError):
        P.city64_batch_host(k, out=np.empty(10, np.int32))
    with pytest.raises(ValueError):
        P.citycrc128_batch_host(k, out=np.empty(19, np.uint64))
    with pytest.raises(ValueError):
        P.place_batch_host(k[:, :8].copy(), 3, 4, out=(np.empty(10, np.uint64), np.empty(9, np.uint32),
                                                       np.empty(10, np.uint32)))
    data = np.zeros(100, np.uint8)
    with pytest.raises(ValueError):
        P.city64_var_batch_host(data, np.array([0, 50, 101], np.uint64))
    with pytest.raises(ValueError):
        P.city64_var_batch_host(data, np.array([0, 50, 100], np.uint64), out=np.empty(1, np.uint64))
    with pytest.raises(ValueError):  # int64 offsets are accepted, negative ones are not
        P.city64_var_batch_host(data, np.array([0, -1, 100], np.int64))
    import torch
    with pytest.raises(ValueError):
        P.city64_var_batch_host(data, torch.tensor([0, -1, 100], dtype=torch.int64))
    with pytest.raises(ValueError):
        P.city64_batch_host(torch.zeros((10, 64), dtype=torch.uint8)[:, :32])


def test_bucket_workspace_small_at_low_rank_counts():
    """The two-pass intermediate (n x (keysize + 2) B: key rows + u16 in-tile
    indices) is reserved only at the rank counts that take the two-pass sort
    (ADVICE r02)."""
    n = 16 << 20
    for records, L, thr in ((False, 8, 1575), (False, 16, 1575), (False, 32, 2049),
                            (True, 8, 2048), (True, 16, 1463), (True, 32, 256)):
        ws = lambda r: P.bucket_workspace_bytes(n, L, r, records=records)  # noqa: E731
        small = ws(min(thr - 1, 1000))
        assert small < 64 << 20, (L, small)
        assert ws(thr) >= small + n * (L + 2)
        assert ws(thr - 1) < n * (L + 2)
        assert ws(8192) >= P.bucket_workspace_bytes(n, L, 8192)
    # 32-B array callers at 1025..2048 ranks do not reserve records' intermediate
    assert P.bucket_workspace_bytes(n, 32, 2048) < n * 34
    assert P.bucket_workspace_bytes(n, 32, 2048, records=True) >= n * 34
    assert P.bucket_workspace_bytes(n, 8, 7) < 1 << 20
    assert P.bucket_workspace_bytes(n, 13, 8192) < n * 17  # generic lengths never take two passes
    assert b"abi 4" in P.lib().pdht_hip_version()


def test_device_wrappers_reject_cpu_tensors():
    import torch
    with pytest.raises(ValueError):
        P.city64_batch(torch.zeros((4, 64), dtype=torch.uint8))


def test_batch_fails_loudly_without_gpu():
    if P.device_count() > 0:
        pytest.skip("a GPU is present")
    keys = np.zeros((10, 64), dtype=np.uint8)
    with pytest.raises(P.PdhtError):
        P.city64_batch_host(keys)
    t = P.PdhtTable(keysize=8)
    with pytest.raises(P.PdhtError):
        t.hash_batch(np.zeros((4, 8), dtype=np.uint8))


def test_every_tuning_variant_is_documented():
    """Every variant number the sources select on is listed in
    pdht_hip_tuning.h (the list had gone stale)."""
    import glob
    import re
    src = "".join(open(p).read() for p in glob.glob(os.path.join(ROOT, "pdht_amd", "csrc", "*.h*")) +
                  glob.glob(os.path.join(ROOT, "pdht_amd", "csrc", "tuning", "*.h"))
                  if not p.endswith("pdht_hip_tuning.h"))
    used = {int(x) for x in re.findall(r"tuning_variant\(\) == (\d+)", src)}
    used |= {int(x) for x in re.findall(r"\bv == (\d+)", src)}
    for block in re.findall(r"switch \(tuning_variant\(\)\) \{(.*?)\n\s*\}", src, re.S):
        used |= {int(x) for x in re.findall(r"case (\d+):", block)}
    for lo, hi in re.findall(r"v >= (\d+) && v <= (\d+)", src):
        used |= set(range(int(lo), int(hi) + 1))
    doc = open(os.path.join(ROOT, "pdht_amd", "csrc", "pdht_hip_tuning.h")).read()
    listed = {int(x) for x in re.findall(r"\b(\d+)\b", doc)}
    listed |= {n for lo, hi in re.findall(r"\b(\d+)-(\d+)\b", doc) for n in range(int(lo), int(hi) + 1)}
    assert used and not (used - listed), sorted(used - listed)


REF = "/root/reference"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "libpdht", "pdht_impl.h")),
                    reason="reference sources absent (GPU box)")
@pytest.mark.parametrize("flavour", ["libpdht", "libmpipdht"])
def test_real_pdht_integration_branch_compiles(tmp_path, flavour):
    """INTEGRATION.md §1's drop-in: pdht_amd/host/pdht_hash.c built with
    -DPDHT_HIP_WITH_REAL_PDHT against the REAL pdht headers (libpdht/pdht_impl.h
    -> pdht.h, or libmpipdht/pdht.h with -DPDHT_HIP_MPI_FLAVOUR), with the
    reference's own flags (pdht.mk GCFLAGS: --std=c99 -O3
    -D_POSIX_C_SOURCE=199309L).  The image lacks <portals4.h> and
    <slurm/pmi.h>, so test-only stubs (tests/realpdht_stubs/) declare the
    types pdht.h uses, ptl_process_t with the Portals 4 layout; the object's
    static checks pin sizeof(ptl_process_t) == 8 with .rank a u32 at offset
    0 -- the stride the batch entry points write.  Compile only: nothing of
    the reference is linked or run."""
    import subprocess
    inc = [f"-I{REF}/libpdht"]
    flags = []
    if flavour == "libmpipdht":
        mpi = [d for d in ("/opt/conda/include", "/usr/include/mpi", "/usr/lib/x86_64-linux-gnu/openmpi/include")
               if os.path.exists(os.path.join(d, "mpi.h"))]
        if not mpi:
            pytest.skip("no mpi.h for libmpipdht/pdht.h")
        inc = [f"-I{REF}/libmpipdht", f"-I{mpi[0]}"]
        flags = ["-DPDHT_HIP_MPI_FLAVOUR"]
    obj = str(tmp_path / "pdht_hash.o")
    cmd = (["gcc", "--std=c99", "-O3", "-D_POSIX_C_SOURCE=199309L", "-fPIC", "-DPDHT_HIP_WITH_REAL_PDHT"] + flags
           + ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "tests", "realpdht_stubs")] + inc
           + ["-c", "-o", obj, os.path.join(ROOT, "pdht_amd", "host", "pdht_hash.c")])
    p = subprocess.run(cmd, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    # no diagnostics from OUR file (the reference's pdht_impl.h:68 redefines offsetof itself)
    src = os.path.join(ROOT, "pdht_amd", "host", "pdht_hash.c")
    ours = [ln for ln in p.stderr.splitlines() if ln.startswith(src + ":")]
    assert not ours, p.stderr
    syms = subprocess.run(["nm", obj], capture_output=True, text=True, check=True).stdout
    defined = {ln.split()[-1] for ln in syms.splitlines() if " T " in ln}
    assert {"pdht_hash", "pdht_sethash", "pdht_hash_batch", "pdht_hash_batch_dev"} <= defined
    # the real build reads c->size, not the stand-in's rank count
    assert "pdht_hip_shim_nranks" not in syms and "pdht_hip_table_init" not in syms
    undef = {ln.split()[-1] for ln in syms.splitlines() if " U " in ln}
    assert {"CityHash64", "pdht_place_batch_host", "pdht_place_batch_dev", "c"} <= undef, undef
