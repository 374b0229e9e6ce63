"""bench.py's parity strings: a shard is "ok" only when its digests were
compared with a reference fold and matched; a shard the golden file has no
fold for is "unchecked" (never "ok"); a mismatch is "FAILED".  Runs on CPU
tensors with no process group (world 1)."""
import sys

import torch

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pdht_amd import dist as D  # noqa: E402


def _shard(first, n, rank=0, world=1):
    return D.Shard(rank, world, first, n)


def test_shard_without_golden_fold_is_unchecked():
    out = torch.arange(1000, dtype=torch.int64)
    for cfg in ("cfg2", "cfg3", "cfg4", "cfg5", "long"):
        p = bench.check_parity(None, torch, D, cfg, _shard(0, 1000), out, None, None)
        assert p.startswith("unchecked: "), p
        assert "no reference fold" in p and not p.startswith("ok")
    # cfg3 rank 9 of a weak-scaling run: no per-rank fold committed
    p = bench.check_parity(None, torch, D, "cfg3", _shard(9 * 64 * bench.M, 64 * bench.M, rank=9), out, None, None)
    assert p.startswith("unchecked: "), p


def test_wrong_digests_fail(monkeypatch):
    out = torch.arange(16, dtype=torch.int64)
    right = D.fold_tensor(out, 0)
    folds = {"cfg5_city64_1B_x64": {"chunk_keys": 16, "chunks": [f"{(right + 1) & D.MASK64:016x}"]}}
    monkeypatch.setattr(bench, "golden_folds", lambda: folds)
    p = bench.check_parity(None, torch, D, "cfg2", _shard(0, 16), out, None, None)
    assert p.startswith("FAILED: "), p


def test_matching_digests_ok(monkeypatch):
    out = torch.arange(32, dtype=torch.int64) * 0x9E3779B97F4A7C15
    folds = {"cfg5_city64_1B_x64": {"chunk_keys": 16,
                                    "chunks": [f"{D.fold_tensor(out[:16], 0):016x}",
                                               f"{D.fold_tensor(out[16:], 16):016x}"]}}
    monkeypatch.setattr(bench, "golden_folds", lambda: folds)
    assert bench.check_parity(None, torch, D, "cfg2", _shard(0, 32), out, None, None).startswith("ok: ")
    # the second chunk alone, as rank 1 of a 2-way split would hold it
    assert bench.check_parity(None, torch, D, "cfg2", _shard(16, 16, rank=1, world=1), out[16:], None,
                              None).startswith("ok: ")


def test_committed_multirank_folds_present():
    """The per-rank folds that make cfg1/cfg3/cfg4 ranks 1..7 checkable."""
    f = bench.golden_folds()
    assert len(f["cfg3_city64_64M_mixed"]["ranks"]) == 8
    assert f["cfg3_city64_64M_mixed"]["ranks"][0]["fold"] == f["cfg3_city64_64M_mixed"]["total"]
    assert len(f["cfg4_crc128_16M_x64"]["rank_chunks"]) == 8
    assert f["cfg4_crc128_16M_x64"]["rank_chunks"][0] == f["cfg4_crc128_16M_x64"]["total"]
    r0 = f["cfg1_pdht_hash_1M_x64"]["ranks"][0]
    pl = [x for x in f["cfg1_pdht_hash_1M_x64"]["placements"] if (x["nptes"], x["nranks"]) == (1, 4)][0]
    assert r0["mbits"] == f["cfg1_pdht_hash_1M_x64"]["mbits"]
    assert (r0["ptindex"], r0["rank"], r0["hist"]) == (pl["ptindex"], pl["rank"], pl["hist"])
    for w in (2, 4, 8):
        for r in range(w):
            sh = D.weak_shard(r, w, 64 * bench.M)
            assert bench.golden_shard_fold(f, "cfg3", sh)[0] is not None
            sh = D.weak_shard(r, w, 16 * bench.M)
            assert bench.golden_shard_fold(f, "cfg4", sh)[0] is not None
            assert bench.golden_shard_fold(f, "cfg2", sh)[0] is not None


def test_committed_bucket_world_folds():
    """exchange / xrecords bucket by nranks = world size: a shard for every
    rank of N = 1, 2, 4, 8.  With one rank the bucketing is the identity:
    index is 0..n-1, offsets are {0, n}, and mbits fold as the place config's
    shard 0 (both reference CityHash64 of the same keys at index 0)."""
    f = bench.golden_folds()
    n = 16 * bench.M
    for w in (1, 2, 4, 8):
        g = f[f"bucket_8B_16M_{w}"]
        assert g["nranks"] == w and g["n"] == n and len(g["shards"]) == w
    one = f["bucket_8B_16M_1"]["shards"][0]
    ident = torch.arange(n, dtype=torch.int64)
    assert int(one["index"], 16) == D.fold_tensor(ident, 0)
    assert int(one["offsets"], 16) == D.fold_tensor(torch.tensor([0, n]), 0)
    assert one["mbits"] == f["place_8B_16M"]["shards"][0]["mbits"]


def _parity_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, ROOT)
        import bench as B
        from pdht_amd import dist as DD
        # rank 0 holds a shard with a (monkeypatched) reference fold, rank 1 a shard without one
        out = torch.arange(16, dtype=torch.int64) + rank
        folds = {"cfg5_city64_1B_x64": {"chunk_keys": 16, "chunks": [f"{DD.fold_tensor(out, 0):016x}"]}}
        B.golden_folds = lambda: folds
        sh = DD.Shard(rank, world, 0 if rank == 0 else 1000, 16)
        q.put((rank, B.check_parity(None, torch, DD, "cfg2", sh, out, None, None)))
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_unchecked_shard_makes_the_line_unchecked():
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_parity_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        assert got[r].startswith("unchecked (worst of 2 ranks): "), got[r]
        assert "[rank 0: ok]" in got[r] and "[rank 1: unchecked]" in got[r]
