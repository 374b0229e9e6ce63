"""Child process of tests/test_gpu_dist.py (not a test module): one rank in
an RCCL ("nccl") process group of world size 1 on cuda:0, running the N-rank
code paths of pdht_amd.dist on device tensors -- the exchange of bucketed
keys and of wire records (all_to_all_single, the one collective the path
has: libmpipdht/putget.c:80-100 ships each request to its owner), the
reductions and the per-rank report.  Started as a fresh process, before
anything in it touches the GPU; prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import pdht_amd as P  # noqa: E402
from pdht_amd import dist as D  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", sys.argv[1] if len(sys.argv) > 1 else "29533")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    n, L = 100003, 8
    keys = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, n, device=dev).view(torch.uint8).view(n, L)

    # arrays: bucket by the world size (one bucket), ship it to its owner
    ko, mb, pt, ix, offs = P.bucket_batch(keys, 3, 1)
    xk, xm, xi, recv = D.exchange_buckets(ko, mb, offs, ix)
    res["exchange_buckets"] = bool(xk.is_cuda and xm.is_cuda and xi.is_cuda and torch.equal(xk, ko)
                                   and torch.equal(xm, mb) and torch.equal(xi, ix)
                                   and recv.tolist() == [n] and torch.equal(mb, P.city64_batch(keys)))

    # wire records: one all-to-all(v) of the record bytes
    rec, roffs = P.bucket_records(keys, 1)
    xr, rrecv = D.exchange_records(rec, roffs)
    res["exchange_records"] = bool(xr.is_cuda and torch.equal(xr, rec) and rrecv.tolist() == [n])

    # reductions and the per-rank report on device tensors
    res["allreduce_max"] = D.allreduce_max([1.5, 2.25], device=dev) == [1.5, 2.25]
    f = D.fold_tensor(mb, 0)
    res["allreduce_fold"] = D.allreduce_fold(f, device=dev) == f
    res["allreduce_min_int"] = D.allreduce_min_int(2, device=dev) == 2
    rep = D.per_rank_report(0, 0, 1, n, 72.0, 1.0, 1.0, 1, 8000.0, device=dev)
    res["per_rank_report"] = rep["world_size"] == 1 and rep["backend"] == "nccl"
    D.barrier()
    torch.cuda.synchronize()
    with open("/proc/self/maps") as fm:
        maps = fm.read()
    res["rccl_mapped"] = "librccl" in maps
    res["product_mapped"] = "libpdht_hip.so" in maps
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
