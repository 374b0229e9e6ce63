"""GPU parity: the HIP kernels against the oracle and the reference golden data.

Bit-exact everywhere (integer hashing).  Small/medium cases compare every
digest with the oracle (oracle/city_oracle.c, itself pinned to the compiled
reference city.c); the full BASELINE configs compare position-weighted fold
checksums with tests/golden/config_folds.json (generated from the reference).
All calls go through the C-ABI (pdht_amd -> libpdht_hip.so).
"""
import numpy as np
import pytest

from conftest import pattern_a

torch = pytest.importorskip("torch")
import pdht_amd as P  # noqa: E402

pytestmark = pytest.mark.gpu
M = 1 << 20


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def u64(t):
    return t.cpu().numpy().view(np.uint64)


def to_dev(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def gpu_fold(d, first_index=0):
    """sum_i d_i * (2(first+i)+1) mod 2^64 on the GPU (int64 wraps)."""
    d = d.reshape(-1)
    idx = torch.arange(d.numel(), device=d.device, dtype=torch.int64) + first_index
    return int((d * (2 * idx + 1)).sum().item()) & 0xFFFFFFFFFFFFFFFF


def device_keys(n, L, first_key=0, dev="cuda"):
    """The BASELINE synthetic keys (splitmix64 byte stream), generated on device."""
    assert (first_key * L) % 8 == 0 and (n * L) % 8 == 0
    w = P.splitmix64_fill(0x5EED5EED5EED5EED, first_key * L // 8, n * L // 8, device=dev)
    return w.view(torch.uint8).view(n, L)


# ------------------------------------------------------------- fixed keys ---
def test_generator_matches_oracle(dev, oracle):
    w = P.splitmix64_fill(oracle.SEED_KEYS, 5, 1000, device=dev)
    assert (u64(w) == oracle.splitmix64(oracle.SEED_KEYS, 5, 1000)).all()
    lens = P.mixed_lengths(oracle.SEED_LENS, 0, 5000, 16, 256, device=dev)
    assert (lens.cpu().numpy().astype(np.uint64) == oracle.mixed_lengths(5000)).all()


SMALL_KERNELS = {8: "k_fixed_direct<8,4,nt>@8", 16: "k_fixed_direct<16,2,nt>@8",
                 32: "k_fixed_direct<32,2,nt>@8", 64: "k_fixed_xpose64<nt,d2>@3"}


def fixed_kernel(L, stride=None, aligned=True, crc=False):
    """launch_fixed's choice for a generic length: the LDS window that holds a
    64-key tile (12 KiB or 16 KiB), else per-lane global reads (16-B loads
    when every key starts 16-B aligned; 2 WG/CU, 8 with the LDS CRC tables)."""
    tile = 63 * (stride or L) + L + 16
    if tile > 16384:
        a16 = aligned and (stride or L) % 16 == 0
        return ("k_global<fixed,a16,lines>" if a16 else "k_global<fixed>") + ("@8" if crc and L > 900 else "@2")
    return "k_window<fixed,nt,16K>@2" if tile > 12288 else "k_window<fixed,nt,12K>@3"


@pytest.mark.parametrize("L", list(range(0, 300)) + [511, 512, 899, 900, 901, 1000, 2047, 4097])
def test_city64_every_length(dev, oracle, L):
    rng = np.random.default_rng(L)
    n = 131  # two full waves + a ragged one
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    got = u64(P.city64_batch(to_dev(k, dev)))
    assert (got == oracle.city64_fixed(k)).all()
    assert P.last_kernel() == SMALL_KERNELS.get(L, fixed_kernel(L))


@pytest.mark.parametrize("L", [0, 1, 3, 8, 13, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 144, 200, 256,
                               271, 272, 400, 527, 528, 899, 900, 901, 960, 1023, 2000, 4096])
def test_city128_crc128_lengths(dev, oracle, L):
    rng = np.random.default_rng(1000 + L)
    n = 70
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    assert (u64(P.city128_batch(kd)) == oracle.city128_fixed(k)).all()
    assert (u64(P.citycrc128_batch(kd)) == oracle.city128_fixed(k, crc=True)).all()


@pytest.mark.parametrize("L", [256, 272, 320, 1024, 8192])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 5000])
def test_long_keys(dev, oracle, L, n):
    """Keys past a 64-key window (k_global): packed and strided rows, ragged
    tiles, aligned and misaligned bases, seeded digests and fused placement."""
    rng = np.random.default_rng(L * 3 + n)
    for stride in (L, L + 48):
        flat = rng.integers(0, 256, (n, stride), dtype=np.uint8)
        k = flat[:, :L]
        kd = to_dev(flat, dev)[:, :L]
        got = u64(P.city64_batch(kd))
        assert P.last_kernel() == fixed_kernel(L, stride)
        assert (got == oracle.city64_fixed(np.ascontiguousarray(k))).all(), (L, n, stride)
    flat = to_dev(rng.integers(0, 256, n * L + 16, dtype=np.uint8), dev)
    for base in (4, 1):
        kd = flat[base:base + n * L].view(n, L)
        assert (u64(P.city64_batch(kd)) == oracle.city64_fixed(kd.cpu().numpy())).all(), base
    kd = to_dev(np.ascontiguousarray(k), dev)
    s0, s1 = 0x0123456789ABCDEF, 0xFEDCBA9876543210
    got = u64(P.city64_seeds_batch(kd, s0, s1))
    assert [int(x) for x in got[:40]] == [oracle.city64_seeds(r.tobytes(), s0, s1) for r in k[:40]]
    mb, pt, rk = P.place_batch(kd, 7, 1000)
    m2, p2, r2 = oracle.pdht_hash_fixed(np.ascontiguousarray(k), 7, 1000)
    assert (u64(mb) == m2).all() and (rk.cpu().numpy().view(np.uint32) == r2).all()


@pytest.mark.parametrize("L", [901, 1000, 1024, 1920, 2200, 4096])
def test_crc128_long_keys_many_tiles(dev, oracle, L):
    """CityHashCrc256 rounds with the LDS CRC tables, every workgroup of the
    grid busy (k_global, 8 WG/CU) and a ragged tail; seeded variant too."""
    rng = np.random.default_rng(L)
    n = 256 * 8 * 256 + 77 if L == 901 else 70_001
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    assert (u64(P.citycrc128_batch(kd)) == oracle.city128_fixed(k, crc=True)).all()
    assert P.last_kernel() == fixed_kernel(L, crc=True)
    s0, s1 = 0x0123456789ABCDEF, 0xFEDCBA9876543210
    got = u64(P.citycrc128_seed_batch(kd[:300], (s0, s1))).reshape(-1, 2)
    assert [tuple(int(x) for x in g) for g in got] == \
        [oracle.citycrc128_seed(r.tobytes(), s0, s1) for r in k[:300]]


@pytest.mark.tuning
@pytest.mark.parametrize("variant", [150, 303])
@pytest.mark.parametrize("L", [901, 1024, 2200])
def test_crc128_long_keys_6bit_tables(dev, oracle, L, variant):
    """Tuning variants 150 / 303: the long-key CRC-32C on r02's 6-bit-slice tables / on 11-bit slices."""
    rng = np.random.default_rng(L + 5)
    k = rng.integers(0, 256, (20_001, L), dtype=np.uint8)
    with P.tuning(variant):
        got = u64(P.citycrc128_batch(to_dev(k, dev)))
    assert (got == oracle.city128_fixed(k, crc=True)).all()


@pytest.mark.tuning
@pytest.mark.parametrize("variant", [190, 191])
@pytest.mark.parametrize("L", [901, 960, 1000, 1024, 1100, 1919, 1920, 2200, 4096])
def test_crc128_long_keys_line_stream(dev, oracle, L, variant):
    """Tuning variants 190/191: CityHashCrc256Long's block loop as a stream of
    128-B lines.  Rows padded to a 16-B stride (the 16-B aligned path), the
    last key at the very end of its allocation; seeded variant too."""
    rng = np.random.default_rng(L + variant)
    n, S = 3001, (L + 15) // 16 * 16
    rows = rng.integers(0, 256, (n, S), dtype=np.uint8)
    k = np.ascontiguousarray(rows[:, :L])
    kd = to_dev(rows, dev)[:, :L]
    with P.tuning(variant):
        got = u64(P.citycrc128_batch(kd))
        kern = P.last_kernel()
        s0, s1 = 0x0123456789ABCDEF, 0xFEDCBA9876543210
        gs = u64(P.citycrc128_seed_batch(kd[:200], (s0, s1))).reshape(-1, 2)
    assert kern.startswith("k_global<fixed,a16,stream>")
    assert (got == oracle.city128_fixed(k, crc=True)).all()
    assert [tuple(int(x) for x in g) for g in gs] == [oracle.citycrc128_seed(r.tobytes(), s0, s1) for r in k[:200]]


@pytest.mark.tuning
@pytest.mark.parametrize("variant", [279, 280, 281])
@pytest.mark.parametrize("L,n", [(1024, 1), (1024, 63), (1024, 64), (1024, 3001), (1024, 70_001),
                                 (2048, 3001), (2048, 20_033), (4096, 5000)])
def test_crc128_long_keys_lds_ring(dev, oracle, L, n, variant):
    """Tuning variants 279-281: packed long keys through an LDS-DMA ring of
    coalesced line-rounds (k_long_ring): single keys, one exact tile, ragged
    tiles, several tiles per wave (70 001 keys) and the key at the very end of
    its allocation; seeded variant too."""
    rng = np.random.default_rng(L + n + variant)
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    with P.tuning(variant):
        got = u64(P.citycrc128_batch(kd))
        kern = P.last_kernel()
        s0, s1 = 0x0123456789ABCDEF, 0xFEDCBA9876543210
        gs = u64(P.citycrc128_seed_batch(kd[:200], (s0, s1))).reshape(-1, 2)
    assert kern.startswith("k_long_ring<"), kern
    assert (got == oracle.city128_fixed(k, crc=True)).all()
    assert [tuple(int(x) for x in g) for g in gs] == [oracle.citycrc128_seed(r.tobytes(), s0, s1) for r in k[:200]]


@pytest.mark.parametrize("L", [0, 5, 8, 16, 24, 32, 64, 100, 256, 300, 384, 400, 1200])
def test_seeded_batches(dev, oracle, L):
    rng = np.random.default_rng(77 + L)
    k = rng.integers(0, 256, (65, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    s0, s1 = 0x0123456789ABCDEF, 0xFEDCBA9876543210
    got = u64(P.city64_seeds_batch(kd, s0, s1))
    assert [int(x) for x in got] == [oracle.city64_seeds(r.tobytes(), s0, s1) for r in k]
    got = u64(P.city64_seed_batch(kd, s1))
    assert [int(x) for x in got] == [oracle.city64_seed(r.tobytes(), s1) for r in k]
    got = u64(P.city128_seed_batch(kd, (s0, s1))).reshape(-1, 2)
    assert [tuple(int(x) for x in g) for g in got] == [oracle.city128_seed(r.tobytes(), s0, s1) for r in k]
    got = u64(P.citycrc128_seed_batch(kd, (s0, s1))).reshape(-1, 2)
    assert [tuple(int(x) for x in g) for g in got] == [oracle.citycrc128_seed(r.tobytes(), s0, s1) for r in k]


def _variants(vs):
    """Variant 0 is the product library; any other variant loads the tuning
    build and runs only with --tuning (conftest.py), so the default -m gpu run
    loads libpdht_hip.so / libpdht_hip_mpi.so only."""
    return [v if v == 0 else pytest.param(v, marks=pytest.mark.tuning) for v in vs]


VARIANT_KERNELS = {0: "k_fixed_xpose64<nt,d2>@3", 7: "k_fixed_xpose64<nt,d1>@4", 188: "k_fixed_xpose64<nt,d2,st16>@3",
                   206: "k_fixed_xpose64<nt,d2,prio1>@3",
                   26: "k_fixed_xpose64<nt-load,plain-store,d2>@3"}


@pytest.mark.tuning
@pytest.mark.parametrize("variant,n", [(250, 1 << 20), (250, 64), (251, 1 << 20), (251, 3 * (1 << 18) + 64 * 5)])
def test_64B_tile_order_probe(dev, oracle, variant, n):
    """Tuning 250 / 251 (r05): the 64-B kernel with the tile order scattered
    over the batch / in per-wave contiguous runs (whole tiles only)."""
    k = oracle.fixed_keys(n, 64)
    with P.tuning(variant):
        got = u64(P.city64_batch(to_dev(k, dev)))
        kern = P.last_kernel()
    assert kern == ("k_fixed_xpose64_order<scatter>@3" if variant == 250 else "k_fixed_xpose64_order<runs>@3")
    assert (got == oracle.city64_fixed(k)).all()


@pytest.mark.parametrize("variant", _variants(sorted(VARIANT_KERNELS)))
def test_64B_kernel_variants_bitexact(dev, oracle, variant):
    """The product kernel, and the tuning build's alternatives (A/B only)."""
    n = M + 13
    k = oracle.fixed_keys(n, 64)
    want = oracle.city64_fixed(k)
    kd = to_dev(k, dev)
    with P.tuning(variant) if variant else _nullctx():
        got = u64(P.city64_batch(kd))
        kern = P.last_kernel()
        got128 = u64(P.citycrc128_batch(kd[:100000]))
    assert kern == VARIANT_KERNELS[variant]
    assert (got == want).all()
    assert (got128 == oracle.city128_fixed(k[:100000], crc=True)).all()
    assert (u64(P.city64_batch(kd[:1000])) == want[:1000]).all()
    assert P.last_kernel() == VARIANT_KERNELS[0]  # back on the product library


def test_golden_random_64B(dev, golden, oracle):
    kd = device_keys(1024, 64, dev=dev)
    assert (u64(P.city64_batch(kd)) == golden["rand64_city64"]).all()
    assert (u64(P.citycrc128_batch(kd)) == golden["rand64_city128"]).all()
    assert (u64(P.city128_batch(kd)) == golden["rand64_city128"]).all()


def test_edge_layouts(dev, oracle):
    rng = np.random.default_rng(5)
    # n = 0 and n = 1
    z = torch.empty((0, 64), dtype=torch.uint8, device=dev)
    assert P.city64_batch(z).numel() == 0
    k1 = rng.integers(0, 256, (1, 64), dtype=np.uint8)
    assert int(u64(P.city64_batch(to_dev(k1, dev)))[0]) == oracle.city64(k1[0].tobytes())
    # strided rows (stride 80, keylen 64) and a 1-byte-misaligned base
    big = rng.integers(0, 256, (1000, 80), dtype=np.uint8)
    bd = to_dev(big, dev)
    got = u64(P.city64_batch(bd[:, :64]))
    assert P.last_kernel() == fixed_kernel(64, 80) == "k_window<fixed,nt,12K>@3"
    assert (got == oracle.city64_fixed(big[:, :64])).all()
    flat = to_dev(rng.integers(0, 256, 64 * 777 + 1, dtype=np.uint8), dev)
    mis = flat[1:].view(777, 64)
    got = u64(P.city64_batch(mis))
    assert (got == oracle.city64_fixed(mis.cpu().numpy())).all()


@pytest.mark.parametrize("nbytes", [16, 4096, 4096 * 1000 + 48])
def test_read_stream_calibration_kernel(dev, nbytes):
    rng = np.random.default_rng(nbytes)
    a = rng.integers(0, 2**63, nbytes // 8, dtype=np.uint64)
    # the kernel XOR-folds every 16-B piece {x,y,z,w} into (x^z) << 32 | (y^w)
    d32 = a.view(np.uint32).reshape(-1, 4)
    x = np.bitwise_xor.reduce(d32[:, 0] ^ d32[:, 2])
    y = np.bitwise_xor.reduce(d32[:, 1] ^ d32[:, 3])
    for nt in (False, True):
        got = int(P.read_stream(to_dev(a.view(np.int64), dev), nt).item()) & 0xFFFFFFFFFFFFFFFF
        assert got == (int(x) << 32) | int(y)


@pytest.mark.parametrize("n", [1, 64, 4096 * 3 + 17])
def test_key_stream_calibration_kernel(dev, n):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 256, (n, 64), dtype=np.uint8)
    got = u64(P.key_stream(to_dev(keys, dev)))
    d = keys.view(np.uint32).reshape(n, 16)
    want = (np.bitwise_xor.reduce(d[:, 1::2], axis=1).astype(np.uint64) << np.uint64(32)) | \
        np.bitwise_xor.reduce(d[:, 0::2], axis=1).astype(np.uint64)
    assert (got == want).all()


def test_key_stream_var_calibration_kernel(dev):
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 300, 5000)
    lens[7] = 20000  # past the LDS window
    offs = np.zeros(lens.size + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    data = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    got = u64(P.key_stream_var(to_dev(data, dev), to_dev(offs.astype(np.int64), dev)))
    for i in range(lens.size):
        k = data[int(offs[i]):int(offs[i + 1])]
        m = len(k) // 16 * 16
        w = k[:m].view(np.uint32).reshape(-1, 4)
        a = int(len(k)) & 0xFFFFFFFF
        b = 0
        if m:
            a ^= int(np.bitwise_xor.reduce(w[:, 0] ^ w[:, 2]))
            b ^= int(np.bitwise_xor.reduce(w[:, 1] ^ w[:, 3]))
        for o in range(m, len(k)):
            a ^= int(k[o]) << (8 * (o & 3))
        assert int(got[i]) == (b << 32) | a, i


def test_errors_are_loud(dev):
    k = torch.zeros((4, 8), dtype=torch.uint8, device=dev)
    with pytest.raises(P.PdhtError):
        P.place_batch(k, nptes=0, nranks=1)
    with pytest.raises(P.PdhtError):
        P.place_batch(k, nptes=1, nranks=0)


# ---------------------------------------------------------- variable keys ---
def test_var_golden_mixed(dev, golden, oracle):
    data, offs = oracle.mixed_keys(1024)
    dd, od = to_dev(data, dev), to_dev(offs.astype(np.int64), dev)
    assert (u64(P.city64_var_batch(dd, od)) == golden["mixed_city64"]).all()
    assert (u64(P.city128_var_batch(dd, od)) == golden["mixed_city128"]).all()
    assert (u64(P.citycrc128_var_batch(dd, od)) == golden["mixed_city128"]).all()


VAR_KERNELS = {0: "auto", 12: "k_window<var,nt,10224>@4", 13: "k_window<var,nt,16K>@2",
               170: "k_window_pipe<var,10224,G1>@4", 171: "k_window_pipe<var,10224,G4>@4",
               172: "k_window_pipe<var,10224,G16>@4", 173: "k_window_pipe<var,10224,G1>@3",
               174: "k_window_pipe<var,10224,G1,funnel>@4", 175: "k_window<var,nt,10224,funnel>@4",
               189: "k_window<var,nt,10224,st16>@4", 203: "k_window<var,nt,10224,prio3>@4",
               204: "k_window<var,nt,10224,prio1>@4", 205: "auto"}  # 205: the product's choice, no s_setprio


@pytest.mark.tuning
@pytest.mark.parametrize("n", [1, 63, 64, 255, 256, 257, 100003, (1 << 20) + 7])
def test_var_wc_kernel(dev, oracle, n):
    """Tuning 252 (r05): the window kernel with workgroup-combined digest
    stores (4 consecutive tiles per workgroup, one 2 KiB store run)."""
    data, offs = oracle.mixed_keys(n)
    with P.tuning(252):
        got = u64(P.city64_var_batch(to_dev(data, dev), to_dev(offs.astype(np.int64), dev)))
        if data.size // n <= 160:  # (wider batches take the 16 KiB window kernel)
            assert P.last_kernel() == "k_window_wc<var,10224>@4"
    assert (got == oracle.city64_var(data, offs)).all()


def auto_var_kernel(total_bytes, n):
    """The product's window choice (launch_var): mean key length > 160 B -> 16 KiB."""
    return "k_window<var,nt,16K>@2" if total_bytes // n > 160 else "k_window<var,nt,10224>@4"


@pytest.mark.parametrize("variant", _variants(sorted(VAR_KERNELS)))
def test_var_edge_cases(dev, oracle, variant):
    with P.tuning(variant) if variant else _nullctx():
        auto = VAR_KERNELS[variant] == "auto"
        total, n = _var_edge_cases(dev, oracle, kernel=VAR_KERNELS[variant] if variant >= 170 and not auto else None)
        want = auto_var_kernel(total, n) if auto else VAR_KERNELS[variant]
        if variant < 170 or auto:  # (170+: CityHash64 kernels only, checked per call inside)
            assert P.last_kernel() == want


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


@pytest.mark.parametrize("variant", _variants(sorted(VAR_KERNELS)))
def test_var_many_tiles_per_wave(dev, oracle, variant):
    """Enough keys that every wave of the persistent grid runs several tiles,
    with a few keys longer than any window and empty keys sprinkled in (runs
    of empty keys fill whole tiles); ragged last tile."""
    rng = np.random.default_rng(23)
    n = 700_001
    lens = rng.integers(0, 300, n)
    lens[rng.integers(0, n, 40)] = 0
    lens[1000:1200] = 0  # whole tiles of empty keys
    lens[rng.integers(0, n, 12)] = rng.integers(11000, 30000, 12)
    offs = np.zeros(n + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    data = rng.integers(0, 256, int(offs[-1]), dtype=np.uint8)
    with P.tuning(variant) if variant else _nullctx():
        got = u64(P.city64_var_batch(to_dev(data, dev), to_dev(offs.astype(np.int64), dev)))
        kern = P.last_kernel()
    assert VAR_KERNELS[variant] == "auto" or kern == VAR_KERNELS[variant]
    assert (got == oracle.city64_var(data, offs)).all()


def _var_edge_cases(dev, oracle, kernel=None):
    rng = np.random.default_rng(9)
    # empty keys, 1..3-byte keys, keys far longer than the LDS window, all mixed
    lens = np.concatenate([np.zeros(40, np.int64), rng.integers(0, 40, 300),
                           rng.integers(0, 300, 300), [0, 20000, 1, 50000, 13000, 0],
                           rng.integers(800, 1100, 50)])
    rng.shuffle(lens)
    offs = np.zeros(lens.size + 1, np.uint64)
    np.cumsum(lens, out=offs[1:])
    data = rng.integers(0, 256, int(offs[-1]) + 3, dtype=np.uint8)
    # misaligned base: hash data[3:] with the same offsets
    for base in (0, 3):
        d = data[base:base + int(offs[-1])]
        dd = to_dev(d, dev)
        od = to_dev(offs.astype(np.int64), dev)
        assert (u64(P.city64_var_batch(dd, od)) == oracle.city64_var(d, offs)).all()
        assert kernel is None or P.last_kernel() == kernel
        assert (u64(P.city128_var_batch(dd, od)) == oracle.city128_var(d, offs)).all()
        assert (u64(P.citycrc128_var_batch(dd, od)) == oracle.city128_var(d, offs, crc=True)).all()
    return int(offs[-1]), lens.size


def test_var_1M_mixed(dev, oracle):
    data, offs = oracle.mixed_keys(M)
    dd, od = to_dev(data, dev), to_dev(offs.astype(np.int64), dev)
    assert (u64(P.city64_var_batch(dd, od)) == oracle.city64_var(data, offs)).all()
    assert P.last_kernel() == auto_var_kernel(data.size, M) == "k_window<var,nt,10224>@4"
    # the same keys through the raw C-ABI with nbytes = 0 (unknown): short-key window
    out = torch.empty(M, dtype=torch.int64, device=dev)
    assert P.lib().pdht_city64_batch_var_dev(dd.data_ptr(), 0, od.data_ptr(), M, out.data_ptr(), None) == 0
    assert P.last_kernel() == "k_window<var,nt,10224>@4"
    assert (u64(out) == oracle.city64_var(data, offs)).all()
    # long keys (mean 192 B): the 16 KiB window, chosen from nbytes / n
    data2, offs2 = oracle.mixed_keys(1 << 18, lo=129, hi=256)
    got = u64(P.city64_var_batch(to_dev(data2, dev), to_dev(offs2.astype(np.int64), dev)))
    assert P.last_kernel() == "k_window<var,nt,16K>@2"
    assert (got == oracle.city64_var(data2, offs2)).all()


# ---------------------------------------------------- fused placement ---
@pytest.mark.parametrize("L", [8, 13, 32, 64])
@pytest.mark.parametrize("nptes,nranks", [(1, 1), (3, 7), (8, 64), (5, 1000), (2, 4096), (7, 4097),
                                          (0xFFFFFFFF, 0x7FFFFFFF), (0x80000000, 65537),
                                          (0xFFFFFFFB, 0x7FFFFFED)])
def test_place_batch(dev, oracle, L, nptes, nranks):
    # nranks is c->size, a positive int (hash.c:29): the largest is 2^31-1
    rng = np.random.default_rng(L * 31 + nranks)
    n = 5000
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    hist = torch.zeros(nranks, dtype=torch.int64, device=dev) if nranks <= 1 << 20 else None
    mb, pt, rk = P.place_batch(to_dev(k, dev), nptes, nranks, hist=hist)
    m2, p2, r2 = oracle.pdht_hash_fixed(k, nptes, nranks)
    assert (u64(mb) == m2).all()
    assert (pt.cpu().numpy().view(np.uint32) == p2).all()
    assert (rk.cpu().numpy().view(np.uint32) == r2).all()
    if hist is not None:
        assert (hist.cpu().numpy() == np.bincount(r2, minlength=nranks)).all()


@pytest.mark.parametrize("L", [8, 16, 64])
def test_place_hist_many_workgroups(dev, oracle, L):
    # enough keys for a full persistent grid; hist accumulates across calls
    rng = np.random.default_rng(L + 5)
    k = rng.integers(0, 256, (1 << 21, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    hist = torch.full((1000,), 5, dtype=torch.int64, device=dev)
    P.place_batch(kd, 3, 1000, hist=hist)
    if L in (8, 16):
        assert P.last_kernel().endswith(",1024>@1" if L == 8 else ",1024>@2")
    else:  # 64-B keys, <= 4M of them, with a histogram: the 1024-thread transpose
        assert P.last_kernel() == "k_fixed_xpose64<nt,d2,1024>@1"
    P.place_batch(kd[:12345], 3, 1000, hist=hist)
    _, _, r2 = oracle.pdht_hash_fixed(k, 3, 1000)
    want = 5 + np.bincount(r2, minlength=1000) + np.bincount(r2[:12345], minlength=1000)
    assert (hist.cpu().numpy() == want).all()


def test_place_hist_64B_large_batch(dev, oracle):
    """Above 4M 64-B keys the histogram placement streams on the 256-thread
    transpose (3 per CU); few ranks, so every workgroup's flush hits one line."""
    n = (4 << 20) + 4097
    words = P.splitmix64_fill(0x1234, 0, n * 8, device=dev)
    kd = words.view(torch.uint8).view(n, 64)
    hist = torch.zeros(4, dtype=torch.int64, device=dev)
    mb, pt, rk = P.place_batch(kd, 1, 4, hist=hist)
    assert P.last_kernel() == "k_fixed_xpose64<nt,d2>@3"
    k = kd[-300000:].cpu().numpy()
    m2, _, r2 = oracle.pdht_hash_fixed(k, 1, 4)
    assert (u64(mb[-300000:]) == m2).all()
    assert (rk[-300000:].cpu().numpy().view(np.uint32) == r2).all()
    r_all = rk.cpu().numpy().view(np.uint32)
    assert (hist.cpu().numpy() == np.bincount(r_all, minlength=4)).all()
    assert (u64(mb) % 4 == r_all).all() and (pt.cpu().numpy() == 0).all()


@pytest.mark.parametrize("L", [8, 64])
def test_bind_place_batch(dev, oracle, L):
    """The prepared call (bench.py cfg1's step): same digests, ptindex and
    ranks as place_batch, and the histogram accumulates over repeated calls."""
    rng = np.random.default_rng(L + 17)
    k = rng.integers(0, 256, (70_001, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    hist = torch.zeros(1000, dtype=torch.int64, device=dev)
    call, (mb, pt, rk) = P.bind_place_batch(kd, 3, 1000, hist=hist)
    call()
    call()
    m2, p2, r2 = oracle.pdht_hash_fixed(k, 3, 1000)
    assert (u64(mb) == m2).all()
    assert (pt.cpu().numpy().view(np.uint32) == p2).all() and (rk.cpu().numpy().view(np.uint32) == r2).all()
    assert (hist.cpu().numpy() == 2 * np.bincount(r2, minlength=1000)).all()


@pytest.mark.parametrize("L", [8, 16, 32])
def test_small_keys(dev, oracle, L):
    rng = np.random.default_rng(L)
    k = rng.integers(0, 256, (70001, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    got = u64(P.city64_batch(kd))
    assert P.last_kernel() == SMALL_KERNELS[L]
    mb, pt, rk = P.place_batch(kd, 7, 1000)
    assert (got == oracle.city64_fixed(k)).all()
    m2, p2, r2 = oracle.pdht_hash_fixed(k, 7, 1000)
    assert (u64(mb) == m2).all()
    assert (pt.cpu().numpy().view(np.uint32) == p2).all()
    assert (rk.cpu().numpy().view(np.uint32) == r2).all()


def test_device_wrappers_validate_outputs(dev):
    """Outputs, histograms and workspaces are checked before any launch: a
    short histogram, a reused `out` of another size or dtype, or a small
    workspace raises instead of letting a kernel write past its end."""
    k = torch.zeros((1000, 8), dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        P.place_batch(k, 3, 1000, hist=torch.zeros(999, dtype=torch.int64, device=dev))
    with pytest.raises(ValueError):
        P.place_batch(k, 3, 1000, hist=torch.zeros(1000, dtype=torch.int32, device=dev))
    mb, pt, rk = P.place_batch(k, 3, 1000)
    with pytest.raises(ValueError):
        P.place_batch(k[:999].contiguous(), 3, 1000, out=(mb, pt, rk))
    with pytest.raises(ValueError):
        P.city64_batch(k, out=torch.empty(999, dtype=torch.int64, device=dev))
    out = P.bucket_batch(k, 3, 16)
    with pytest.raises(ValueError):
        P.bucket_batch(k, 3, 17, out=out)  # offsets sized for 16 ranks
    with pytest.raises(ValueError):
        P.bucket_batch(k, 3, 16, workspace=torch.empty(16, dtype=torch.uint8, device=dev))
    rec = P.bucket_records(k, 16)
    with pytest.raises(ValueError):
        P.bucket_records(k[:500].contiguous(), 16, out=rec)
    with pytest.raises(ValueError):
        P.city64_batch(k.cpu())
    data = torch.zeros(100, dtype=torch.uint8, device=dev)
    for bad in ([0, 50, 101], [60, 70, 50], [-8, 0, 10]):  # past the data, end before start, negative
        with pytest.raises(ValueError):
            P.city64_var_batch(data, torch.tensor(bad, dtype=torch.int64, device=dev))
    assert P.city64_var_batch(data, torch.tensor([0, 50, 100], dtype=torch.int64, device=dev)).numel() == 2
    s_other = torch.cuda.Stream(device=dev)
    assert P.city64_batch(k, stream=s_other).numel() == 1000  # a stream of the right device


BUCKET_CASES = [(L, nr, n, 0) for L in (8, 13, 16, 32, 64) for nr in (1, 2, 7, 1000, 4096, 4097, 8192)
                for n in (0, 1, 4095, 100003)]
# the product's two-pass entry points with the fine-plus digit split:
# arrays: 8/16-B keys from 1575 ranks (the last 8 x 16 owner shape at 1574), 32-B from 2049
BUCKET_CASES += [(L, nr, n, 0) for (L, nr) in ((8, 1536), (8, 1574), (8, 1575), (8, 2047), (16, 1025), (16, 1574),
                                                (16, 1575), (16, 2048))
                 for n in (4095, 300007)]
BUCKET_CASES += [(L, nr, n, 21) for L in (8, 16, 32) for nr in (7, 1000, 2049, 8192) for n in (4095, 300007)]
BUCKET_CASES += [(L, nr, n, v) for v in (70, 71) for L in (8, 16, 32) for nr in (2, 7, 64, 1000, 2048, 2049, 8192)
                 for n in (1, 4095, 300007, (1 << 20) + 5)]
# 321: the staged scatter loading its keys non-temporally (the r02-r06 policy)
BUCKET_CASES += [(L, nr, n, 321) for L in (8, 16, 32) for nr in (7, 600, 1000, 1535) for n in (4097, 300007)]
BUCKET_CASES += [(L, nr, n, 85) for L in (8, 16, 32) for nr in (1, 7, 1000, 1535)
                 for n in (1, 4095, 300007, (1 << 20) + 5, (16 << 20) + 3)]
BUCKET_CASES += [(L, nr, n, v) for v in (83, 87, 89) for L in (8, 16, 32)
                 for nr in (1, 7, 511, 512, 1000, 1462, 1463, 1535)
                 for n in (1, 4095, 300007, (1 << 20) + 5)]
# 202: the r03 two-pass sub-tile shape (4 x 8 @ 4 for both passes)
BUCKET_CASES += [(L, nr, n, v) for v in (202,) for L in (8, 16, 32) for nr in (2049, 8192)
                 for n in (4095, 300007, (1 << 20) + 5)]
# 265 / 266: 8-B arrays' pass 2 as r04-r05 shipped it (two store phases, 4 x 8 @ 4) / one phase in 4 x 8 @ 4
BUCKET_CASES += [(8, nr, n, v) for v in (265, 266) for nr in (1536, 2049, 8192)
                 for n in (4095, 300007, (1 << 20) + 5)]
# 264: the fine counts column-scanned over 32-tile chunks by k_bucket_colscan (r02-r05)
BUCKET_CASES += [(L, nr, n, 264) for L in (8, 16, 32) for nr in (1536, 2049, 8192)
                 for n in (4095, 300007, (1 << 20) + 5, (3 << 20) + 7)]
# 267-269: 16/32-B keys' two passes in 4 keys per lane (r05 spill probe)
BUCKET_CASES += [(L, nr, n, v) for v in (267, 268, 269, 270) for L in (16, 32) for nr in (2049, 8192)
                 for n in (4095, 300007, (1 << 20) + 5)]
# 164: two-pass arrays on the balanced digit split (the product takes one fine bit more)
BUCKET_CASES += [(L, nr, n, 164) for L in (8, 16, 32) for nr in (1025, 2049, 4097, 8192)
                 for n in (4095, 300007, (1 << 20) + 5)]
# the product's fine-plus split at its edges: 71 forces two passes from 2 ranks (nbits 1..3)
BUCKET_CASES += [(L, nr, 70001, 71) for L in (8, 32) for nr in (2, 3, 4, 5, 8, 9)]
# r06 tile-local two passes: count-chunks of ct = 1 / 2 / 4 tiles (ct doubles
# from 512 chunks up: 2M / 4M / 8M keys), pass-2 segments of SG or SG + 1
# chunks split evenly (8192 ranks, n ~1.1M / 2.1M keys: ADVICE r05), 1025 and
# 8192 ranks (F = 64 / 256), ragged last tiles
BUCKET_CASES += [(L, nr, n, 0) for L in (8, 16) for nr in (8192,) for n in ((1 << 20) + 100_003, (2 << 20) + 100_003)]
BUCKET_CASES += [(L, nr, n, 0) for L in (8, 32) for nr in (2049, 8192) for n in ((4 << 20) + 7, (8 << 20) + 4097)]
# 290: the r02-r05 two-pass form (counting kernel ahead of pass 1, global fine-bucket runs);
# 291-293: tile-local shapes (pass 2 in 4 x 8 @ 4 / 8 x 4 @ 2; pass 1 in 16 waves @ 1)
BUCKET_CASES += [(L, nr, n, v) for v in (290, 291, 292, 293, 302, 304, 305, 316, 318, 320, 322, 323) for L in (8, 16, 32) for nr in (2049, 8192)
                 for n in (4095, 300007, (1 << 20) + 5)]


def _bucket_kernel(L, nranks, variant, records=False):
    """Product: the staged scatter for 8/16/32-B keys below the two-pass
    threshold (arrays 1575 / 1575 / 2049 ranks, records 2048 / 1463 / 256 for
    8 / 16 / 32-B keys), two passes from it, the generic
    kernel for other lengths.  Tuning variants: 21 forces the generic-length
    kernel, 70 one pass up to 2048 ranks, 71 two passes from 2 ranks up, 85
    the staged scatter in the static tile order instead of per-XCD tickets,
    83 / 87 / 89 the staged scatter with owner-table ranking on 8 x 16 / 4 x
    16 tiles or with ballots, at any nranks."""
    wg = "k_bucket_scatter_wg<8>" if nranks <= 4096 else "k_bucket_scatter_wg<4>"
    if variant == 21:
        return wg
    if L in (8, 16, 32):
        two_pass_from = ({8: 2048, 16: 1463, 32: 256} if records else {8: 1575, 16: 1575, 32: 2049})[L]
        one_pass = variant == 70 and nranks <= 2048
        if (variant == 71 and nranks >= 2) or (not one_pass and nranks >= two_pass_from):
            # the tile-local form (r06); the r02-r05 form under 290 and its shape variants
            r05 = variant in (290, 202, 264) or 265 <= variant <= 272
            return f"k_bucket_pass2<{L}B>" if r05 else f"k_bucket_tl_pass2<{L}B>"
        # staged_shape(): owner-table ranking for array outputs from 512
        # ranks, on 8 x 16 tiles for 8/16-B keys while 81920 + 52 B per rank
        # of LDS fits a CU, else on 4 x 16 tiles while 40960 + 28 B per rank
        # leaves two workgroups per CU; ballots otherwise
        if variant == 83:
            return f"k_bucket_scatter_staged<{L}B,own,8x16>"
        if variant == 87:
            return f"k_bucket_scatter_staged<{L}B,own>"
        if variant in (85, 89) or records or nranks < 512:
            return f"k_bucket_scatter_staged<{L}B>"
        if L != 32 and 81920 + 52 * nranks + 64 <= 160 * 1024:
            return f"k_bucket_scatter_staged<{L}B,own,8x16>"
        if 40960 + 28 * nranks <= 80 * 1024:
            return f"k_bucket_scatter_staged<{L}B,own>"
        return f"k_bucket_scatter_staged<{L}B>"
    return wg


def _tuning_marked(cases):
    """variant != 0 cases run only with --tuning (conftest.py)."""
    return [c if c[-1] == 0 else pytest.param(*c, marks=pytest.mark.tuning) for c in cases]


@pytest.mark.parametrize("L,nranks,n,variant", _tuning_marked(BUCKET_CASES))
def test_bucket_batch(dev, oracle, L, nranks, n, variant):
    rng = np.random.default_rng(L * 7 + nranks + n)
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    with P.tuning(variant) if variant else _nullctx():
        ko, mb, pt, ix, offs = P.bucket_batch(to_dev(k, dev), 3, nranks)
        if n:
            assert P.last_kernel() == _bucket_kernel(L, nranks, variant)
    m2, p2, r2 = oracle.pdht_hash_fixed(k, 3, nranks) if n else (
        np.zeros(0, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint32))
    order = np.argsort(r2, kind="stable")  # the reference placement, stably bucketed
    assert ix.dtype == torch.int32
    assert (ix.cpu().numpy().view(np.uint32) == order).all()
    assert (u64(mb) == m2[order]).all()
    assert (pt.cpu().numpy().view(np.uint32) == p2[order]).all()
    assert (ko.cpu().numpy() == k[order]).all()
    want_offs = np.concatenate([[0], np.cumsum(np.bincount(r2, minlength=nranks))])
    assert (offs.cpu().numpy() == want_offs).all()


@pytest.mark.parametrize("L,nranks,variant", _tuning_marked([(L, nr, v) for L in (8, 16, 32)
                                                              for nr in (1000, 8192) for v in (0, 70)]))
def test_bucket_skewed(dev, oracle, L, nranks, variant):
    """Few distinct keys: whole batches land in a handful of buckets, so the
    two-pass sort meets segments far longer than its 4096-key sub-tiles and
    tiles whose keys all share one bucket."""
    rng = np.random.default_rng(L + nranks)
    distinct = rng.integers(0, 256, (3, L), dtype=np.uint8)
    k = distinct[rng.integers(0, 3, 700_001)]
    with P.tuning(variant) if variant else _nullctx():
        ko, mb, pt, ix, offs = P.bucket_batch(to_dev(k, dev), 3, nranks)
        assert P.last_kernel() == _bucket_kernel(L, nranks, variant)
    m2, p2, r2 = oracle.pdht_hash_fixed(k, 3, nranks)
    order = np.argsort(r2, kind="stable")
    assert (ix.cpu().numpy().view(np.uint32) == order).all()
    assert (u64(mb) == m2[order]).all()
    assert (ko.cpu().numpy() == k[order]).all()
    want_offs = np.concatenate([[0], np.cumsum(np.bincount(r2, minlength=nranks))])
    assert (offs.cpu().numpy() == want_offs).all()


@pytest.mark.parametrize("L,nranks", [(8, 1000), (16, 1000), (13, 1000), (8, 2049), (16, 2049), (8, 8192),
                                      (16, 8192)])
def test_bucket_optional_outputs(dev, oracle, L, nranks):
    """Each of keys_out / ptindex_out / index_out may be omitted (NULL);
    mbits and the offsets are the same either way -- on the one-pass and on
    the two-pass path (2049 / 8192 ranks)."""
    rng = np.random.default_rng(L)
    n = 50_000
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    kd = to_dev(k, dev)
    m2, p2, r2 = oracle.pdht_hash_fixed(k, 1, nranks)
    order = np.argsort(r2, kind="stable")
    for wk, wp, wi in ((False, False, True), (True, False, False), (False, False, False)):
        ko, mb, pt, ix, offs = P.bucket_batch(kd, 1, nranks, with_keys=wk, with_ptindex=wp, with_index=wi)
        assert (ko is not None) == wk and (pt is not None) == wp and (ix is not None) == wi
        assert (u64(mb) == m2[order]).all()
        if ix is not None:
            assert (ix.cpu().numpy().view(np.uint32) == order).all()
        if ko is not None:
            assert (ko.cpu().numpy() == k[order]).all()


RECORD_CASES = [(L, nr, n, 0) for L in (8, 13, 16, 32, 64) for nr in (1, 7, 1000, 2049, 8192)
                for n in (0, 1, 4095, 100003)]
RECORD_CASES += [(L, nr, n, v) for v in (21, 70, 71) for L in (8, 16, 32) for nr in (7, 1000, 2048, 8192)
                 for n in (4097, 300007)]
RECORD_CASES += [(L, nr, n, 321) for L in (8, 16, 32) for nr in (7, 600, 1000) for n in (4097, 300007)]
RECORD_CASES += [(L, nr, n, 85) for L in (8, 16, 32) for nr in (7, 1000) for n in (4097, (2 << 20) + 9)]
# records switch to owner-table ranking for 16/32-B keys from 512 ranks while
# two workgroups fit a CU (staged_shape): both edges of both thresholds
RECORD_CASES += [(L, nr, 300007, 0) for L in (8, 16, 32) for nr in (511, 512, 1462, 1463)]
# records take two passes from 2048 / 1463 / 256 ranks (8 / 16 / 32-B keys)
RECORD_CASES += [(32, nr, n, 0) for nr in (255, 256, 1024, 1025, 2048) for n in (4097, 300007)]
RECORD_CASES += [(L, nr, n, 0) for (L, nr) in ((8, 1536), (8, 2047), (8, 2048), (16, 1462), (16, 1463))
                 for n in (4097, 300007)]
# two-pass shapes of records: 267-270 (16/32-B keys), 271 / 272 (8-B keys' pass 2 in 4 keys per lane)
RECORD_CASES += [(L, nr, n, v) for v in (267, 268, 269, 270) for L in (16, 32) for nr in (2049, 8192)
                 for n in (4097, 300007)]
RECORD_CASES += [(8, nr, n, v) for v in (271, 272) for nr in (2049, 8192) for n in (4097, 300007, (1 << 20) + 5)]
# 112: the r02 store order of 8-B records (header halves a staging round early)
RECORD_CASES += [(8, nr, n, 112) for nr in (7, 1000, 1463) for n in (4097, (2 << 20) + 9)]
# r06: records on the r02-r05 two-pass form (290) and the tile-local shapes 291-293
RECORD_CASES += [(L, nr, n, v) for v in (290, 291, 292, 293, 302, 304, 305, 316, 318, 320, 322, 323) for L in (8, 16, 32) for nr in (2049, 8192)
                 for n in (4097, 300007)]
RECORD_CASES += [(L, 8192, (4 << 20) + 7, 0) for L in (8, 32)]


@pytest.mark.parametrize("L,nranks,n,variant", _tuning_marked(RECORD_CASES))
def test_bucket_records(dev, oracle, L, nranks, n, variant):
    """Wire records (message_t header + key) at the bucketed positions."""
    rng = np.random.default_rng(L * 11 + nranks + n)
    k = rng.integers(0, 256, (n, L), dtype=np.uint8)
    with P.tuning(variant) if variant else _nullctx():
        rec, offs = P.bucket_records(to_dev(k, dev), nranks, src_rank=5, ht_index=3)
    rb = P.bucket_record_bytes(L)
    assert rb == 24 + (L + 7) // 8 * 8 and tuple(rec.shape) == (n, rb)
    m2, _, r2 = oracle.pdht_hash_fixed(k, 3, nranks) if n else (np.zeros(0, np.uint64), None,
                                                                 np.zeros(0, np.uint32))
    order = np.argsort(r2, kind="stable")
    want_offs = np.concatenate([[0], np.cumsum(np.bincount(r2, minlength=nranks))])
    assert (offs.cpu().numpy() == want_offs).all()
    if n == 0:
        return
    R = rec.cpu().numpy()
    w32 = R[:, :16].copy().view(np.uint32)
    assert (w32[:, 0] == P.PDHT_PUT).all() and (w32[:, 1] == 5).all() and (w32[:, 2] == 3).all()
    assert (w32[:, 3] == order).all()
    assert (R[:, 16:24].copy().view(np.uint64).ravel() == m2[order]).all()
    assert (R[:, 24:24 + L] == k[order]).all()
    assert (R[:, 24 + L:] == 0).all()
    ty, sr, hi, ix, mb, ko = P.record_fields(rec, L)
    assert (u64(mb) == m2[order]).all() and (ix.cpu().numpy().view(np.uint32) == order).all()


@pytest.mark.parametrize("nranks,shard", [(1, 0), (2, 1), (4, 3), (8, 7), (1024, 0), (8192, 5)])
def test_bucket_shard_golden_folds(dev, folds, nranks, shard):
    """The bench's bucketing shards at full size (16M x 8-B keys from key
    shard*16M, nptes 3) against the reference folds: nranks = 1/2/4/8 is what
    exchange / xrecords bucket at N ranks, 1024 the bucket config, 8192 the
    two-pass sort.  Arrays and wire records both."""
    g = folds["bucket_8B_16M" if nranks == 1024 else f"bucket_8B_16M_{nranks}"]
    assert g["nranks"] == nranks
    gs = g["shards"][shard]
    n = g["n"]
    kd = device_keys(n, 8, first_key=shard * n, dev=dev)
    ko, mb, pt, ix, offs = P.bucket_batch(kd, 3, nranks)
    assert f"{gpu_fold(mb):016x}" == gs["mbits"]
    assert f"{gpu_fold(ix.to(torch.int64) & 0xFFFFFFFF):016x}" == gs["index"]
    assert f"{gpu_fold(offs):016x}" == gs["offsets"]
    del ko, pt
    rec, roffs = P.bucket_records(kd, nranks)
    _, _, _, rix, rmb, _ = P.record_fields(rec, 8)
    assert f"{gpu_fold(rmb.contiguous()):016x}" == gs["mbits"]
    assert f"{gpu_fold(rix.to(torch.int64) & 0xFFFFFFFF):016x}" == gs["index"]
    assert f"{gpu_fold(roffs):016x}" == gs["offsets"]


def test_place_golden_u64_keys(dev, golden):
    keys = np.arange(256, dtype=np.uint64).view(np.uint8).reshape(256, 8)
    kd = to_dev(keys, dev)
    for a, p in enumerate(golden["pdht_nptes"]):
        for b, r in enumerate(golden["pdht_nranks"]):
            mb, pt, rk = P.place_batch(kd, int(p), int(r))
            assert (u64(mb) == golden["pdht_u64keys_mbits"]).all()
            assert (pt.cpu().numpy().view(np.uint32) == golden["pdht_ptindex"][a]).all()
            assert (rk.cpu().numpy().view(np.uint32) == golden["pdht_rank"][b]).all()


# -------------------------------------------------------- host-resident ---
def test_host_resident_paths(dev, oracle):
    n = 2 * M + 5  # > 1 chunk of the pipeline (32 MiB of keys)
    k = oracle.fixed_keys(n, 64)
    want = oracle.city64_fixed(k)
    assert (P.city64_batch_host(k) == want).all()  # pageable: staged
    kp = torch.from_numpy(k).pin_memory()
    op = torch.empty(n, dtype=torch.int64).pin_memory()
    P.city64_batch_host(kp, out=op)  # pinned in and out: zero-copy kernel
    assert (op.numpy().view(np.uint64) == want).all()
    # zero-copy on pointers inside pinned allocations (offset rows)
    op2 = torch.zeros(n - 7, dtype=torch.int64).pin_memory()
    P.city64_batch_host(kp[7:], out=op2)
    assert (op2.numpy().view(np.uint64) == want[7:]).all()
    o128 = torch.empty((1000, 2), dtype=torch.int64).pin_memory()
    P.citycrc128_batch_host(kp[3:1003], out=o128)
    assert (o128.numpy().view(np.uint64) == oracle.city128_fixed(k[3:1003], crc=True)).all()
    assert (P.citycrc128_batch_host(k[:300000]) == oracle.city128_fixed(k[:300000], crc=True)).all()
    data, offs = oracle.mixed_keys(600000)
    assert (P.city64_var_batch_host(data, offs) == oracle.city64_var(data, offs)).all()
    k8 = oracle.fixed_keys(100000, 8)
    mb, pt, rk = P.place_batch_host(k8, 3, 12)
    m2, p2, r2 = oracle.pdht_hash_fixed(k8, 3, 12)
    assert (mb == m2).all() and (pt == p2).all() and (rk == r2).all()

    # every buffer pinned: the zero-copy paths (variable-length and placement)
    def pinned(n_, dt):
        return torch.zeros(n_ * np.dtype(dt).itemsize, dtype=torch.uint8).pin_memory().numpy().view(dt)
    pdata = pinned(data.size, np.uint8)
    pdata[:] = data
    poffs = pinned(offs.size, np.uint64)
    poffs[:] = offs
    pout = pinned(offs.size - 1, np.uint64)
    P.city64_var_batch_host(pdata, poffs, out=pout)
    assert (pout == oracle.city64_var(data, offs)).all()
    pk8 = pinned(k8.size, np.uint8).reshape(k8.shape)
    pk8[:] = k8
    outs = (pinned(len(k8), np.uint64), pinned(len(k8), np.uint32), pinned(len(k8), np.uint32))
    P.place_batch_host(pk8, 3, 12, out=outs)
    assert (outs[0] == m2).all() and (outs[1] == p2).all() and (outs[2] == r2).all()


@pytest.mark.tuning
def test_host_pinned_through_copy_pipeline(dev, oracle):
    """Tuning variant 61: pinned buffers forced through the chunked copy
    pipeline (the A/B of zero-copy against staging)."""
    n = 2 * M + 5
    k = oracle.fixed_keys(n, 64)
    kp = torch.from_numpy(k).pin_memory()
    op = torch.zeros(n, dtype=torch.int64).pin_memory()
    with P.tuning(61):
        P.city64_batch_host(kp, out=op)
    assert (op.numpy().view(np.uint64) == oracle.city64_fixed(k)).all()


def test_zero_copy_misaligned_var_keys(dev, oracle):
    """Pinned variable-length keys at every misaligned base, the last key
    ending at the last byte of the buffer: the window kernel reads the pinned
    pages over PCIe, 16-B pieces aligned on ABSOLUTE addresses, so it never
    reads a block that holds no key byte."""
    data, offs = oracle.mixed_keys(20000)
    want = oracle.city64_var(data, offs)
    buf = torch.zeros(data.size + 64, dtype=torch.uint8).pin_memory().numpy()
    poffs = torch.zeros(offs.size * 8, dtype=torch.uint8).pin_memory().numpy().view(np.uint64)
    poffs[:] = offs
    pout = torch.zeros(want.size * 8, dtype=torch.uint8).pin_memory().numpy().view(np.uint64)
    for base in (1, 3, 7, 15, 16 + 9):
        end = buf.size - (base % 16)  # buffers ending at every alignment too
        start = end - data.size
        pdata = buf[start:end]
        pdata[:] = data
        pout[:] = 0
        P.city64_var_batch_host(pdata, poffs, out=pout)
        assert (pout == want).all(), base


def test_pdht_hash_batch_default_and_plugin(dev, oracle):
    t = P.PdhtTable(keysize=13, nptes=4, nranks=10)
    k = oracle.fixed_keys(5000, 13)
    mb, pt, rk = t.hash_batch(k)  # default hash -> GPU, ptl_process_t stride 8
    m2, p2, r2 = oracle.pdht_hash_fixed(k, 4, 10)
    assert (mb == m2).all() and (pt == p2).all() and (rk == r2).all()
    # scalar pdht_hash agrees with the batch
    for i in (0, 1, 4999):
        assert t.hash(k[i].tobytes()) == (int(m2[i]), int(p2[i]), int(r2[i]))


# --------------------------------------------------- full BASELINE configs ---
def test_cfg2_16M_x64_full_fold(dev, folds):
    f = folds["cfg2_city64_16M_x64"]
    kd = device_keys(f["n"], 64, dev=dev)
    d = P.city64_batch(kd)
    assert P.last_kernel() == SMALL_KERNELS[64]
    assert f"{gpu_fold(d):016x}" == f["total"]


def test_cfg4_crc128_16M_full_fold(dev, folds):
    f = folds["cfg4_crc128_16M_x64"]
    kd = device_keys(f["n"], 64, dev=dev)
    d = P.citycrc128_batch(kd)
    assert f"{gpu_fold(d):016x}" == f["total"]


@pytest.mark.parametrize("variant", _variants([0, 13, 118]))
def test_cfg3_64M_mixed_full_fold(dev, folds, variant):
    """8.7 GB of keys: offsets far past 2^31 and 2^32 (64-bit window math)."""
    f = folds["cfg3_city64_64M_mixed"]
    n = f["n"]
    lens = P.mixed_lengths(0x1E575EED1E575EED, 0, n, 16, 256, device=dev)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item())
    assert total == f["total_bytes"]
    words = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, (total + 7) // 8, device=dev)
    data = words.view(torch.uint8)[:total]
    with P.tuning(variant) if variant else _nullctx():
        d = P.city64_var_batch(data, offs)
    assert f"{gpu_fold(d):016x}" == f["total"]


@pytest.mark.parametrize("r", [1, 7])
def test_cfg3_rank_shard(dev, folds, r):
    """cfg3's weak shard of rank r at N > 1, hashed on this GPU exactly as
    bench.py's rank r hashes it (lengths from key r*64M of the length stream,
    bytes from word r << 40 of the key stream: bench.py cfg3 workload), against
    the reference fold of that shard (gen_golden.py --multirank; the
    reference places keys by contiguous slices, libpdht/hash.c:29)."""
    f = folds["cfg3_city64_64M_mixed"]
    n = f["n"]
    want = f["ranks"][r]
    lens = P.mixed_lengths(0x1E575EED1E575EED, r * n, n, 16, 256, device=dev)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    del lens
    total = int(offs[-1].item())
    assert total == want["total_bytes"]
    words = P.splitmix64_fill(0x5EED5EED5EED5EED, r << 40, (total + 7) // 8, device=dev)
    d = P.city64_var_batch(words.view(torch.uint8)[:total], offs)
    assert f"{gpu_fold(d, r * n):016x}" == want["fold"]


@pytest.mark.parametrize("r", [1, 7])
def test_cfg4_rank_shard(dev, folds, r):
    """cfg4's weak shard of rank r (keys [r*16M, (r+1)*16M) of the 64-B
    stream), CityHashCrc128 on this GPU, against the reference fold of that
    shard (128-bit digests fold from global entry 2*r*16M)."""
    f = folds["cfg4_crc128_16M_x64"]
    n = f["n"]
    words = P.splitmix64_fill(0x5EED5EED5EED5EED, r * n * 8, n * 8, device=dev)
    d = P.citycrc128_batch(words.view(torch.uint8).view(n, 64))
    assert f"{gpu_fold(d, 2 * r * n):016x}" == f["rank_chunks"][r]


def test_cfg5_all_shards_of_1B(dev, folds):
    """BASELINE configs[4] (1B x 64 B keys over 8 GPUs) on ONE GPU, one shard
    after another: shard j = keys [j*128M, (j+1)*128M), exactly the slice
    rank j hashes at N = 8, each checked against the reference's fold of that
    shard.  Together the 8 shards cover the whole 1B-key stream."""
    f = folds["cfg5_city64_1B_x64"]
    per = f["n"] // 8
    words = torch.empty(per * 8, dtype=torch.int64, device=dev)
    out = torch.empty(per, dtype=torch.int64, device=dev)
    total = 0
    for j in range(8):
        P.splitmix64_fill(0x5EED5EED5EED5EED, j * per * 8, per * 8, out=words)
        P.city64_batch(words.view(torch.uint8).view(per, 64), out=out)
        fj = gpu_fold(out, j * per)
        assert f"{fj:016x}" == f["shards"][j], j
        total = (total + fj) & 0xFFFFFFFFFFFFFFFF
    assert f"{total:016x}" == f["total"]


def test_cfg1_place_1M_x64(dev, folds):
    """BASELINE configs[0] (1M x 64 B keys through hash.c) as a GPU batch:
    fused placement (mbits, ptindex, rank, rankputs histogram) against the
    reference folds, for each (nptes, nranks) of the fixture; and the same
    placement through pdht_hash_batch (host keys, ptl_process_t ranks)."""
    f = folds["cfg1_pdht_hash_1M_x64"]
    n = f["n"]
    kd = device_keys(n, 64, dev=dev)
    for pl in f["placements"]:
        hist = torch.zeros(pl["nranks"], dtype=torch.int64, device=dev)
        mb, pt, rk = P.place_batch(kd, pl["nptes"], pl["nranks"], hist=hist)
        assert f"{gpu_fold(mb):016x}" == f["mbits"]
        assert f"{gpu_fold(pt.to(torch.int64) & 0xFFFFFFFF):016x}" == pl["ptindex"]
        assert f"{gpu_fold(rk.to(torch.int64) & 0xFFFFFFFF):016x}" == pl["rank"]
        assert f"{gpu_fold(hist):016x}" == pl["hist"]
    pl = f["placements"][0]
    t = P.PdhtTable(keysize=64, nptes=pl["nptes"], nranks=pl["nranks"])
    mb, pt, rk = t.hash_batch(kd.cpu().numpy())
    from oracle import oracle as O
    assert f"{O.fold64(mb, 0):016x}" == f["mbits"]
    assert f"{O.fold64(rk.astype(np.uint64), 0):016x}" == pl["rank"]


def test_cfg1_mpi_flavour_batches(dev, folds):
    """a17, libmpipdht/hash.c:6-9 on the GPU: libpdht_hip_mpi.so's
    pdht_hash_batch (host keys) and pdht_hash_batch_dev (device keys) over
    cfg1's 1M x 64 B keys write mbits and rank = mbits % c->size and leave
    every ptindex (and the nid/pid half of each ptl_process_t) untouched; the
    mbits, rank and rankputs folds equal the reference's."""
    import ctypes as C
    f = folds["cfg1_pdht_hash_1M_x64"]
    n = f["n"]
    kd = device_keys(n, 64, dev=dev)
    kh = kd.cpu().numpy()
    L = P.mpi_lib()
    SENT = 0xA5A5A5A5
    for pl in f["placements"]:
        t = P._PdhtT()
        L.pdht_hip_table_init(C.byref(t), 64, pl["nptes"])
        C.c_int.in_dll(L, "pdht_hip_shim_nranks").value = pl["nranks"]
        # host batch: ptl_process_t[] ranks (stride 8)
        mb = np.empty(n, np.uint64)
        pt = np.full(n, SENT, np.uint32)
        rk = np.full(2 * n, SENT, np.uint32)
        assert L.pdht_hash_batch(C.byref(t), kh.ctypes.data, n, mb.ctypes.data, pt.ctypes.data,
                                 rk.ctypes.data, 0) == 0, L.pdht_hip_last_error()
        r = rk[0::2]
        assert (pt == SENT).all() and (rk[1::2] == SENT).all()
        assert (r.astype(np.uint64) == mb % np.uint64(pl["nranks"])).all()
        from oracle import oracle as O
        assert f"{O.fold64(mb, 0):016x}" == f["mbits"]
        assert f"{O.fold64(r.astype(np.uint64), 0):016x}" == pl["rank"]
        # device batch, with the rankputs histogram
        mbd = torch.empty(n, dtype=torch.int64, device=dev)
        sent32 = SENT - (1 << 32)  # the same bits as an int32
        ptd = torch.full((n,), sent32, dtype=torch.int32, device=dev)
        rkd = torch.full((2 * n,), sent32, dtype=torch.int32, device=dev)
        hist = torch.zeros(pl["nranks"], dtype=torch.int64, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        assert L.pdht_hash_batch_dev(C.byref(t), kd.data_ptr(), n, mbd.data_ptr(), ptd.data_ptr(),
                                     rkd.data_ptr(), hist.data_ptr(), s) == 0, L.pdht_hip_last_error()
        torch.cuda.synchronize()
        assert bool((ptd == sent32).all().item())
        rr = rkd.view(n, 2)
        assert bool((rr[:, 1] == sent32).all().item())
        assert f"{gpu_fold(mbd):016x}" == f["mbits"]
        assert f"{gpu_fold(rr[:, 0].to(torch.int64) & 0xFFFFFFFF):016x}" == pl["rank"]
        assert f"{gpu_fold(hist):016x}" == pl["hist"]


@pytest.mark.parametrize("L", [8, 16, 64])
def test_place_batch_without_ptindex(dev, oracle, folds, L):
    """place_batch(..., ptindex=False): the fused kernel with a NULL ptindex
    (the libmpipdht placement) writes mbits, rank and the histogram only."""
    if L == 64:
        f = folds["cfg1_pdht_hash_1M_x64"]
        kd = device_keys(f["n"], 64, dev=dev)
        for pl in f["placements"]:
            hist = torch.zeros(pl["nranks"], dtype=torch.int64, device=dev)
            mb, pt, rk = P.place_batch(kd, pl["nptes"], pl["nranks"], ptindex=False, hist=hist)
            assert pt is None
            assert f"{gpu_fold(mb):016x}" == f["mbits"]
            assert f"{gpu_fold(rk.to(torch.int64) & 0xFFFFFFFF):016x}" == pl["rank"]
            assert f"{gpu_fold(hist):016x}" == pl["hist"]
        return
    rng = np.random.default_rng(L + 99)
    k = rng.integers(0, 256, (300_001, L), dtype=np.uint8)
    for nranks in (1, 7, 1000):
        mb, pt, rk = P.place_batch(to_dev(k, dev), 3, nranks, ptindex=False)
        m2, _, r2 = oracle.pdht_hash_fixed(k, 3, nranks)
        assert pt is None and (u64(mb) == m2).all() and (rk.cpu().numpy().view(np.uint32) == r2).all()


def test_batches_capture_in_hip_graph(dev, oracle):
    """The batch entry points are capture-safe (no allocation, no
    synchronisation): record hash, placement and bucketing in one hipGraph
    (torch.cuda.CUDAGraph on ROCm), replay it on new keys, check bit-exact."""
    n = 50_000
    keys = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    k8 = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    pl = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.int32, device=dev),
          torch.empty(n, dtype=torch.int32, device=dev))
    ws = torch.empty(P.bucket_workspace_bytes(n, 8, 1000), dtype=torch.uint8, device=dev)
    bk = P.bucket_batch(k8, 3, 1000, workspace=ws)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside capture (lazy device init)
        P.city64_batch(keys, out=out)
        P.place_batch(k8, 3, 1000, out=pl)
        P.bucket_batch(k8, 3, 1000, out=bk, workspace=ws)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        P.city64_batch(keys, out=out)
        P.place_batch(k8, 3, 1000, out=pl)
        P.bucket_batch(k8, 3, 1000, out=bk, workspace=ws)
    for seed in (1, 2):
        rng = np.random.default_rng(seed)
        kh = rng.integers(0, 256, (n, 64), dtype=np.uint8)
        k8h = rng.integers(0, 256, (n, 8), dtype=np.uint8)
        keys.copy_(torch.from_numpy(kh))
        k8.copy_(torch.from_numpy(k8h))
        g.replay()
        torch.cuda.synchronize()
        assert (u64(out) == oracle.city64_fixed(kh)).all()
        m2, p2, r2 = oracle.pdht_hash_fixed(k8h, 3, 1000)
        assert (u64(pl[0]) == m2).all() and (pl[2].cpu().numpy().view(np.uint32) == r2).all()
        order = np.argsort(r2, kind="stable")
        assert (bk[3].cpu().numpy().view(np.uint32) == order).all() and (u64(bk[1]) == m2[order]).all()


@pytest.mark.parametrize("variant", _variants([0, 114]))
def test_chunked_launches(dev, oracle, variant):
    """Batches past launch_chunk_bytes() go out as consecutive launches (512
    MiB in the product, 256 MiB in tuning variant 114): fixed keys (digests,
    128-bit digests, fused placement with a histogram and ptl_process_t-style
    rank stride) and offset-indexed keys, ragged ends, checked against the
    oracle on samples from both sides of every chunk boundary."""
    n = (5 << 20) + 4099  # 320 MiB of 64-B keys: two 256 MiB launches in variant 114
    words = P.splitmix64_fill(0x77, 0, n * 8, device=dev)
    kd = words.view(torch.uint8).view(n, 64)
    step = (256 << 20) // 64
    idx = np.unique(np.concatenate([np.arange(0, 200), np.arange(step - 100, step + 100),
                                    np.arange(n - 200, n)]))
    kh = kd[torch.from_numpy(idx).to(dev)].cpu().numpy()
    with P.tuning(variant) if variant else _nullctx():
        d64 = u64(P.city64_batch(kd))
        d128 = u64(P.city128_batch(kd)).reshape(-1, 2)
        hist = torch.zeros(1000, dtype=torch.int64, device=dev)
        mb, pt, rk = P.place_batch(kd, 3, 1000, hist=hist)
    assert (d64[idx] == oracle.city64_fixed(kh)).all()
    assert (d128[idx] == oracle.city128_fixed(kh)).all()
    m2, p2, r2 = oracle.pdht_hash_fixed(kh, 3, 1000)
    assert (u64(mb)[idx] == m2).all() and (pt.cpu().numpy().view(np.uint32)[idx] == p2).all()
    r_all = rk.cpu().numpy().view(np.uint32)
    assert (r_all[idx] == r2).all() and (u64(mb) % 1000 == r_all).all()
    assert (hist.cpu().numpy() == np.bincount(r_all, minlength=1000)).all()
    # variable-length keys: 3M mixed 16..256 B = ~408 MB
    nv = 3 << 20
    lens = P.mixed_lengths(0x1E575EED1E575EED, 0, nv, 16, 256, device=dev)
    offs = torch.zeros(nv + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item())
    data = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, (total + 7) // 8, device=dev).view(torch.uint8)[:total]
    with P.tuning(variant) if variant else _nullctx():
        dv = u64(P.city64_var_batch(data, offs))
    dh, oh = data.cpu().numpy(), offs.cpu().numpy().astype(np.uint64)
    assert (dv == oracle.city64_var(dh, oh)).all()


def test_more_than_4G_keys(dev, oracle):
    """Batches of more than 2^32 keys (8-B keys: 32 GiB in, 32 GiB of
    digests, then the fused placement with a histogram): every index past
    2^31 and 2^32 lands where it belongs -- checked against the oracle on
    samples around both boundaries and at the ends, the histogram against
    the batch size and the rank array."""
    n = (1 << 32) + 4099
    kd = P.splitmix64_fill(0x4A11, 0, n, device=dev).view(torch.uint8).view(n, 8)
    idx = np.unique(np.concatenate([np.arange(0, 100), np.arange((1 << 31) - 100, (1 << 31) + 100),
                                    np.arange((1 << 32) - 100, (1 << 32) + 100), np.arange(n - 100, n)]))
    kh = kd[torch.from_numpy(idx).to(dev)].cpu().numpy()
    d64 = P.city64_batch(kd)
    assert (u64(d64[torch.from_numpy(idx).to(dev)]) == oracle.city64_fixed(kh)).all()
    del d64
    torch.cuda.empty_cache()
    hist = torch.zeros(7, dtype=torch.int64, device=dev)
    mb, pt, rk = P.place_batch(kd, 3, 7, hist=hist)
    m2, p2, r2 = oracle.pdht_hash_fixed(kh, 3, 7)
    ti = torch.from_numpy(idx).to(dev)
    assert (u64(mb[ti]) == m2).all() and (pt[ti].cpu().numpy().view(np.uint32) == p2).all()
    assert (rk[ti].cpu().numpy().view(np.uint32) == r2).all()
    assert int(hist.sum().item()) == n
    assert [int(hist[r].item()) for r in range(7)] == [int((rk == r).sum().item()) for r in range(7)]
    del kd, mb, pt, rk
    torch.cuda.empty_cache()


@pytest.mark.parametrize("nranks", [1000, 8192])
def test_bucket_largest_batch(dev, oracle, nranks):
    """Bucketing at the ABI's limit, n = 2^32 - 1 keys (32 GiB of 8-B keys;
    the single pass at 1000 ranks, two passes at 8192): the per-rank counts
    equal those of the fused placement over the input, every output key's
    rank is its bucket's, indices rise strictly inside each bucket, each
    output key is the input key its index names, and sampled digests match
    the oracle -- together: the exact stable bucketing."""
    n = (1 << 32) - 1
    kd = P.splitmix64_fill(0xB16B, 0, n, device=dev).view(torch.uint8).view(n, 8)
    hist = torch.zeros(nranks, dtype=torch.int64, device=dev)
    P.place_batch(kd, 3, nranks, ptindex=False, rank=False, hist=hist)
    torch.cuda.empty_cache()
    ko, mb, pt, ix, offs = P.bucket_batch(kd, 3, nranks, with_ptindex=False)
    torch.cuda.empty_cache()
    assert int(offs[-1].item()) == n and int(offs[0].item()) == 0
    assert (offs[1:] - offs[:-1] == hist).all()
    step = 1 << 28
    prev_r = prev_i = None
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        kc = ko[lo:hi]
        _, _, rk = P.place_batch(kc, 3, nranks, ptindex=False)
        rk = rk.long()
        i64 = ix[lo:hi].long() & 0xFFFFFFFF
        assert (rk[1:] >= rk[:-1]).all()  # buckets in rank order
        same = rk[1:] == rk[:-1]
        assert (i64[1:][same] > i64[:-1][same]).all()  # stable inside a bucket
        if prev_r is not None and prev_r == int(rk[0].item()):
            assert int(i64[0].item()) > prev_i
        prev_r, prev_i = int(rk[-1].item()), int(i64[-1].item())
        assert (kd[i64] == kc).all()  # the key its index names
        del rk, i64, same
    # the ranks' bucket bounds: the first key of every non-empty bucket has that rank
    nz = torch.nonzero(hist).flatten()
    starts = offs[nz]
    _, _, rs = P.place_batch(ko[starts].contiguous(), 3, nranks, ptindex=False)
    assert (rs.long() == nz).all()
    sample = torch.from_numpy(np.unique(np.concatenate([np.arange(0, 64), np.arange(n - 64, n),
                                                        np.random.default_rng(5).integers(0, n, 256)]))).to(dev)
    assert (u64(mb[sample]) == oracle.city64_fixed(ko[sample].cpu().numpy())).all()
    del kd, ko, mb, pt, ix, offs
    torch.cuda.empty_cache()


def test_var_keys_past_4GiB(dev, oracle):
    """Offset-indexed keys whose bytes run past 2^32 (36M mixed 16..256-B
    keys, ~4.9 GB in several launches): the keys whose bytes straddle or lie
    beyond the 2^31 / 2^32 byte offsets, and the last ones, against the
    oracle."""
    nv = 36 << 20
    lens = P.mixed_lengths(0x1E575EED1E575EED, 0, nv, 16, 256, device=dev)
    offs = torch.zeros(nv + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item())
    assert total > (1 << 32) + (1 << 28)
    data = P.splitmix64_fill(0x5EED, 0, (total + 7) // 8, device=dev).view(torch.uint8)[:total]
    dv = P.city64_var_batch(data, offs)
    oh = offs.cpu().numpy()
    idx = []
    for b in (1 << 31, 1 << 32):
        j = int(np.searchsorted(oh, b, side="right")) - 1  # the key holding byte b
        idx += list(range(j - 50, j + 50))
    idx = np.unique(np.array(idx + list(range(nv - 100, nv))))
    sub = [data[int(oh[i]):int(oh[i + 1])].cpu().numpy() for i in idx]
    so = np.concatenate([[0], np.cumsum([len(x) for x in sub])]).astype(np.uint64)
    want = oracle.city64_var(np.concatenate(sub), so)
    assert (u64(dv[torch.from_numpy(idx).to(dev)]) == want).all()
    del data, dv, offs, lens
    torch.cuda.empty_cache()


def test_var_offsets_check_on_launch_stream(dev, oracle):
    """The variable-length wrappers' default offsets check reads offsets[0] /
    offsets[n] on the LAUNCH stream: offsets written on a side
    stream are seen, bad ones raise, and capture on that side stream skips
    the host read (the captured call replays correctly)."""
    data, offs = oracle.mixed_keys(20000)
    want = oracle.city64_var(data, offs)
    s = torch.cuda.Stream(device=dev)
    dd = to_dev(data, dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        od = torch.zeros(offs.size, dtype=torch.int64, device=dev)
        od.copy_(torch.from_numpy(offs.astype(np.int64)).pin_memory(), non_blocking=True)
        bad = od.clone()
        bad[-1] = data.size + 1
    got = P.city64_var_batch(dd, od, stream=s)
    s.synchronize()
    assert (u64(got) == want).all()
    with pytest.raises(ValueError, match="offsets span"):
        P.city64_var_batch(dd, bad, stream=s)
    out = torch.zeros(offs.size - 1, dtype=torch.int64, device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        P.city64_var_batch(dd, od, out=out, stream=s)
    g.replay()
    torch.cuda.synchronize()
    assert (u64(out) == want).all()


def test_default_run_loads_product_libraries_only(request):
    """Runs last: without --tuning no test has opened the tuning build."""
    if request.config.getoption("--tuning"):
        pytest.skip("tuning run")
    maps = open("/proc/self/maps").read()
    assert "libpdht_hip_tuning.so" not in maps
