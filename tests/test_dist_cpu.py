"""The N > 1 path on CPU: world_size-2 gloo processes run bench.py's sharding
and reductions (pdht_amd.dist) over a small key stream -- and the same code in
a gloo group of ONE process (what `bench.py --dist-backend` does at N = 1:
the collectives and the exchange still run, every bucket to rank 0).

Each rank hashes its weak-scaling shard with the product's scalar CityHash64
(the same city_core.h code the kernels run), folds it by global key index and
all-reduces: the sum of the rank folds must equal the oracle's fold of the
whole stream, and each rank's fold must equal the oracle's fold of its slice
-- the property bench.py relies on to check every GPU's shard independently.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

N_PER = 3000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pdht_amd as P
        from pdht_amd import dist as D
        from oracle import oracle as O
        r, lr, w = D.env_rank_world()
        sh = D.weak_shard(r, w, N_PER)
        keys = O.fixed_keys(sh.n, 64, first_key=sh.first)
        d = np.array([P.CityHash64(k.tobytes()) for k in keys], dtype=np.uint64)
        t = torch.from_numpy(d.view(np.int64))
        local = D.fold_tensor(t, sh.first)
        total = D.allreduce_fold(local)
        mx = D.allreduce_max([float(r + 1), 0.5 * r])
        ok_all = D.allreduce_min_flag(r != 1)  # rank 1 reports failure
        # f4 exchange: bucket this shard by owner rank (on a GPU pdht_amd.bucket_batch
        # does this; here the oracle's placement + a stable sort stands in) and ship
        # every bucket to its owner
        mb, _, rk = O.pdht_hash_fixed(keys[:, :8], 3, w)
        order = np.argsort(rk, kind="stable")
        offs = np.concatenate([[0], np.cumsum(np.bincount(rk, minlength=w))])
        gidx = torch.from_numpy((order + sh.first).astype(np.int64))
        k2, m2, i2, cnt = D.exchange_buckets(torch.from_numpy(keys[order, :8].copy()),
                                             torch.from_numpy(mb[order].view(np.int64)),
                                             torch.from_numpy(offs.astype(np.int64)), gidx)
        # the same bucket as wire records (the layout pdht_bucket_records_dev
        # writes on a GPU, built here with numpy) shipped in ONE all-to-all(v)
        rec = np.zeros((sh.n, P.bucket_record_bytes(8)), np.uint8)
        rec[:, 0:4] = np.frombuffer(np.uint32(P.PDHT_PUT).tobytes(), np.uint8)
        rec[:, 4:8] = np.frombuffer(np.uint32(r).tobytes(), np.uint8)
        rec[:, 12:16] = order.astype(np.uint32).view(np.uint8).reshape(-1, 4)
        rec[:, 16:24] = mb[order].view(np.uint8).reshape(-1, 8)
        rec[:, 24:32] = keys[order, :8]
        xr, xrc = D.exchange_records(torch.from_numpy(rec), torch.from_numpy(offs.astype(np.int64)))
        # the N > 1 bench line's per-rank block (bench.py per_rank): rank r
        # reports a kernel time of (r+1) ms for its n keys
        pr = D.per_rank_report(r, lr, w, 1 << 20, 72, float(r + 1), 2.0, 10, 8000.0)
        D.barrier()
        q.put({"rank": r, "first": sh.first, "n": sh.n, "local": local, "total": total, "per_rank": pr,
               "xrec": xr.numpy(), "xrcnt": xrc.numpy(),
               "max": mx, "ok_all": ok_all,
               "oracle_local": O.fold64(O.city64_fixed(keys), sh.first),
               "xkeys": k2.numpy(), "xmbits": m2.numpy().view(np.uint64), "xidx": i2.numpy(),
               "xcnt": cnt.numpy()})
    finally:
        dist.destroy_process_group()


def test_shard_helpers_single_process():
    from pdht_amd import dist as D
    assert D.weak_shard(3, 8, 100) == D.Shard(3, 8, 300, 100)
    cover = [D.strong_shard(r, 3, 10) for r in range(3)]
    assert [c.first for c in cover] == [0, 3, 6] and sum(c.n for c in cover) == 10
    # no process group: reductions are identities
    assert D.allreduce_max([1.5, 2.0]) == [1.5, 2.0]
    assert D.allreduce_fold(5) == 5
    t = torch.tensor([1, 2, 3], dtype=torch.int64)
    assert D.fold_tensor(t, 10) == 1 * 21 + 2 * 23 + 3 * 25
    big = torch.tensor([-1], dtype=torch.int64)  # 0xffff... as u64
    assert D.fold_tensor(big, 0) == (1 << 64) - 1


@pytest.mark.parametrize("WORLD", [2, 1, 3, 8])
def test_gloo_shards_and_reductions(oracle, WORLD):
    """World sizes 1 and 2, a non-power-of-two 3, and 8 -- the driver's
    scaling run -- so the exchange's 8-way splits are checked as well."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda x: x["rank"])
    whole = oracle.fixed_keys(WORLD * N_PER, 64)
    want_total = oracle.fold64(oracle.city64_fixed(whole), 0)
    for r in res:
        assert r["first"] == r["rank"] * N_PER and r["n"] == N_PER
        assert r["local"] == r["oracle_local"]          # each shard checks on its own
        assert r["total"] == want_total                 # and they add up to the whole
        assert r["max"] == [float(WORLD), 0.5 * (WORLD - 1)]
        assert r["ok_all"] is (WORLD == 1)              # one failing rank (rank 1) fails all
        pr = r["per_rank"]                              # every rank sees every rank's numbers
        assert pr["world_size"] == WORLD and pr["backend"] == "gloo"
        assert [x["rank"] for x in pr["ranks"]] == list(range(WORLD))
        assert all({"host", "device", "name", "pci", "event_ms", "keys", "Gkeys_s", "frac", "wall_Gkeys_s"} <= set(x)
                   for x in pr["ranks"])
        assert pr["Gkeys_s"] == [round((1 << 20) / (k + 1) / 1e6, 3) for k in range(WORLD)]
        assert pr["frac"] == [round(72 * (1 << 20) / (k + 1) / 1e6 / 8000, 4) for k in range(WORLD)]
        assert pr["aggregate_kernel_Gkeys_s"] == round(sum(pr["Gkeys_s"]), 3)
    # after the exchange rank r holds exactly the keys the reference places on r,
    # grouped by source rank, each group in key order
    mb, _, rk = oracle.pdht_hash_fixed(whole[:, :8], 3, WORLD)
    for r in res:
        want = np.flatnonzero(rk == r["rank"])
        assert (r["xidx"] == want).all()
        assert (r["xmbits"] == mb[want]).all()
        assert (r["xkeys"] == whole[want, :8]).all()
        assert list(r["xcnt"]) == [int(((rk == r["rank"]) & (np.arange(len(rk)) // N_PER == s)).sum())
                                   for s in range(WORLD)]
        # records: the same keys in the same order, header fields intact
        xr = r["xrec"]
        src = xr[:, 4:8].copy().view(np.uint32).ravel()
        loc = xr[:, 12:16].copy().view(np.uint32).ravel()
        assert (xr[:, 0:4].copy().view(np.uint32).ravel() == 1).all()
        assert ((src.astype(np.int64) * N_PER + loc) == want).all()
        assert (xr[:, 16:24].copy().view(np.uint64).ravel() == mb[want]).all()
        assert (xr[:, 24:32] == whole[want, :8]).all()
        assert (r["xrcnt"] == r["xcnt"]).all()
