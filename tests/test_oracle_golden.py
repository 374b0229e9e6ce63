"""Pin the oracle (oracle/city_oracle.c) to the reference's own outputs.

The golden vectors were produced by the compiled reference city.c
(tests/golden/gen_golden.py); the known answers below are the ones quoted in
SURVEY.md §8c.  The reference has no tests of the hash values itself
(SURVEY.md §4), so these fixtures are the whole parity anchor.
"""
import numpy as np
import pytest

from conftest import pattern_a, pattern_b

KNOWN64 = {  # bytes k[i] = i  
    0: 0x9AE16A3B2F90404F, 1: 0x085F654E398E757C, 3: 0x34E803DC175E241F,
    4: 0xC6803D385BA50E93, 8: 0xBAB32314AB07FA4E, 9: 0xF5CB477F28A07FE7,
    16: 0x2FB0D75F94362763, 17: 0xE5AA5ED150B8E380, 32: 0x40CFEF3D008869DC,
    33: 0x532C06F602B7F406, 64: 0xF7A2ACA4D0A3FDE1, 65: 0xAC589C990483DD2E,
    128: 0x10B153630AF1F395, 256: 0x0C693049D8C2C68D,
}


def test_known_answers(oracle):
    k = pattern_a(1024)
    for L, h in KNOWN64.items():
        assert oracle.city64(k[:L]) == h, L
    assert oracle.city128(k[:64]) == (0x83D9A0502FD851D0, 0x718073343EA63F22)
    assert oracle.citycrc128(k[:64]) == (0x83D9A0502FD851D0, 0x718073343EA63F22)
    kb = pattern_b(1024)
    assert oracle.city128(kb[:900]) == (0x0BD5851D4019E72F, 0x92CEE3967DE7EFA2)
    assert oracle.citycrc128(kb[:900]) == (0x0BD5851D4019E72F, 0x92CEE3967DE7EFA2)
    assert oracle.city128(kb[:901]) == (0x8425A38F646BCA6F, 0x69245D660E939D48)
    assert oracle.citycrc128(kb[:901]) == (0x785BE23A39A70DFB, 0x471283FDE71131AF)


@pytest.mark.parametrize("tag,pat", [("A", pattern_a), ("B", pattern_b)])
def test_all_lengths_0_1024(oracle, golden, tag, pat):
    buf = pat(1024)
    c64 = golden[f"pat{tag}_city64"]
    c128 = golden[f"pat{tag}_city128"]
    crc_hi = golden[f"pat{tag}_crc128_901up"]
    for L in range(1025):
        assert oracle.city64(buf[:L]) == int(c64[L]), L
        assert oracle.city128(buf[:L]) == tuple(int(x) for x in c128[L]), L
        want_crc = c128[L] if L <= 900 else crc_hi[L - 901]
        assert oracle.citycrc128(buf[:L]) == tuple(int(x) for x in want_crc), L


def test_seeded_and_crc256(oracle, golden):
    buf = pattern_a(1024)
    s64 = int(golden["seed64"][0])
    lo, hi = (int(x) for x in golden["seed128"])
    for L in range(1025):
        assert oracle.city64_seed(buf[:L], s64) == int(golden["patA_city64_seed"][L]), L
        assert oracle.city64_seeds(buf[:L], lo, hi) == int(golden["patA_city64_seeds"][L]), L
        assert oracle.city128_seed(buf[:L], lo, hi) == tuple(int(x) for x in golden["patA_city128_seed"][L])
        want = golden["patA_city128_seed"][L] if L <= 900 else golden["patA_crc128_seed_901up"][L - 901]
        assert oracle.citycrc128_seed(buf[:L], lo, hi) == tuple(int(x) for x in want), L
        assert oracle.citycrc256(buf[:L]) == tuple(int(x) for x in golden["patA_crc256"][L]), L


def test_long_keys(oracle, golden):
    lens = [int(x) for x in golden["long_lens"]]
    buf = pattern_b(max(lens))
    for j, L in enumerate(lens):
        assert oracle.city64(buf[:L]) == int(golden["longB_city64"][j])
        assert oracle.city128(buf[:L]) == tuple(int(x) for x in golden["longB_city128"][j])
        assert oracle.citycrc128(buf[:L]) == tuple(int(x) for x in golden["longB_crc128"][j])


def test_synthetic_generator(oracle, golden):
    assert (oracle.splitmix64(oracle.SEED_KEYS, 0, 64) == golden["splitmix_head"]).all()
    assert (oracle.splitmix64(oracle.SEED_LENS, 0, 64) == golden["splitmix_lens_head"]).all()
    # random access into the stream agrees with the sequential stream
    assert (oracle.splitmix64(oracle.SEED_KEYS, 10, 20) == golden["splitmix_head"][10:30]).all()


def test_random_64B_keys(oracle, golden):
    k = oracle.fixed_keys(1024, 64)
    assert (oracle.city64_fixed(k) == golden["rand64_city64"]).all()
    assert (oracle.city128_fixed(k) == golden["rand64_city128"]).all()
    assert (oracle.city128_fixed(k, crc=True) == golden["rand64_city128"]).all()


def test_mixed_keys(oracle, golden):
    data, offs = oracle.mixed_keys(1024)
    assert (offs == golden["mixed_offsets"]).all()
    lens = np.diff(offs.astype(np.int64))
    assert lens.min() >= 16 and lens.max() <= 256
    assert (oracle.city64_var(data, offs) == golden["mixed_city64"]).all()
    assert (oracle.city128_var(data, offs) == golden["mixed_city128"]).all()
    assert (oracle.city128_var(data, offs, crc=True) == golden["mixed_city128"]).all()


def test_pdht_hash_placement(oracle, golden):
    keys = np.arange(256, dtype=np.uint64).view(np.uint8).reshape(256, 8)
    mb = golden["pdht_u64keys_mbits"]
    # keys 0..3 -> mbits, rank % 4 = 2,2,1,1
    assert [int(x) for x in mb[:4]] == [0xD7C06285B9DE677A, 0x8CC42B24AE99097E,
                                        0x2DA3830134001575, 0x2BC1BBBACD374FE1]
    for a, p in enumerate(golden["pdht_nptes"]):
        for b, r in enumerate(golden["pdht_nranks"]):
            m, pt, rk = oracle.pdht_hash_fixed(keys, int(p), int(r))
            assert (m == mb).all()
            assert (pt == golden["pdht_ptindex"][a]).all()
            assert (rk == golden["pdht_rank"][b]).all()
    m, pt, rk = oracle.pdht_hash_fixed(keys[:4], 1, 4)
    assert list(rk) == [2, 2, 1, 1]


def _crc32c_bytes(crc, data):
    for byte in data:
        crc ^= byte
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc


def test_crc32c_instruction_semantics(oracle):
    # the pure-Python CRC-32C is pinned by the standard check value
    assert _crc32c_bytes(0xFFFFFFFF, b"123456789") ^ 0xFFFFFFFF == 0xE3069283
    # _mm_crc32_u64: 8 LE bytes, low 32 bits of crc in, no inversion, zero-extended
    assert oracle.lib().oracle_crc32c_u64(0, 0) == 0
    rng = np.random.default_rng(3)
    for _ in range(200):
        c, v = (int(x) for x in rng.integers(0, 2**63, 2, dtype=np.uint64))
        c |= 0xABCD << 40  # high bits of the crc operand are ignored
        want = _crc32c_bytes(c & 0xFFFFFFFF, v.to_bytes(8, "little"))
        assert oracle.lib().oracle_crc32c_u64(c, v) == want


def test_fold(oracle):
    d = np.array([1, 2, 3], dtype=np.uint64)
    assert oracle.fold64(d) == 1 * 1 + 2 * 3 + 3 * 5
    assert oracle.fold64(d, 10) == 1 * 21 + 2 * 23 + 3 * 25


def test_oracle_matches_compiled_reference_fuzz(oracle):
    """Cross-check against oracle/_ref (the reference compiled here), if built."""
    R = oracle.ref()
    if R is None:
        pytest.skip("oracle/_ref not built (no /root/reference)")
    rng = np.random.default_rng(7)
    for L in list(range(0, 300)) + [511, 512, 513, 899, 900, 901, 902, 1199, 1200, 1201, 3000]:
        d = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        assert oracle.city64(d) == R.CityHash64(d, L)
        r = R.CityHashCrc128(d, L)
        assert oracle.citycrc128(d) == (r.first, r.second)
        r = R.CityHash128(d, L)
        assert oracle.city128(d) == (r.first, r.second)


def test_cpu_bucketing_baseline_is_the_stable_bucketing(oracle):
    """bench.py's f4 CPU baseline (oracle_time_bucket: hash, count per rank,
    stable scatter, the Meraculous count-then-ship shape) produces exactly the
    reference placement stably bucketed -- the outputs the GPU bucketing is
    checked against -- for 1 and several threads, arrays and records."""
    k = oracle.fixed_keys(50_003, 8)
    fn, _ = oracle.cpu_fn("CityHash64")
    m2, p2, r2 = oracle.pdht_hash_fixed(k, 3, 1000)
    order = np.argsort(r2, kind="stable")
    want_offs = np.concatenate([[0], np.cumsum(np.bincount(r2, minlength=1000))])
    for thr in (1, 3):
        _, b = oracle.time_bucket(fn, k, 3, 1000, threads=thr, reps=2)
        assert (b.offsets == want_offs).all() and (b.idx == order).all()
        assert (b.mbits == m2[order]).all() and (b.pt == p2[order]).all() and (b.keys == k[order]).all()
        _, b = oracle.time_bucket(fn, k, 3, 1000, threads=thr, records=True, src_rank=5, ht_index=3)
        w32 = b.rec[:, :16].copy().view(np.uint32)
        assert (w32[:, 0] == 1).all() and (w32[:, 1] == 5).all() and (w32[:, 2] == 3).all()
        assert (w32[:, 3] == order).all() and (b.rec[:, 24:32] == k[order]).all()
        assert (b.rec[:, 16:24].copy().view(np.uint64).ravel() == m2[order]).all()
