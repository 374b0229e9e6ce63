"""Multi-GPU orchestration of the batch hash: independent shards, no
collective on the data path.

A key batch is split by key index into contiguous per-rank slices; each rank
hashes its slice on its own GPU.  The only collectives are the ones a
benchmark or a caller needs around the data path: a start barrier, the max
of per-rank elapsed times, and (for verification) the sum of per-rank fold
checksums, which equals the fold of the whole batch because the fold is
position-weighted by GLOBAL key index (sum_i d_i * (2i+1) mod 2^64).

Backend-agnostic: "nccl" (RCCL on ROCm) on GPUs, "gloo" in the CPU tests.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

MASK64 = (1 << 64) - 1


def _grouped() -> bool:
    """True inside an initialised process group -- of ANY size: at world size
    1 the collectives still run (through RCCL when the group is "nccl"), so
    a one-GPU run executes the same code path as an N-GPU one."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    first: int  # global index of this rank's first key
    n: int      # keys on this rank


def env_rank_world() -> tuple[int, int, int]:
    """(rank, local_rank, world) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def weak_shard(rank: int, world: int, n_per_rank: int) -> Shard:
    """Weak scaling: every rank gets n_per_rank keys, rank r the slice
    [r*n, (r+1)*n) of the global key stream."""
    return Shard(rank, world, rank * n_per_rank, n_per_rank)


def strong_shard(rank: int, world: int, n_total: int) -> Shard:
    """Strong scaling: n_total keys split as evenly as possible, contiguous."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return Shard(rank, world, lo, hi - lo)


def fold_tensor(d, first_index: int) -> int:
    """Position-weighted fold of a digest tensor (int64 view of u64 digests,
    flattened; 128-bit digests contribute 2 entries per key and the caller
    passes first_index = 2*first_key)."""
    import torch
    d = d.reshape(-1)
    acc = torch.zeros((), dtype=torch.int64, device=d.device)
    step = 1 << 24  # bounded temporaries: a 1B-key shard folds in 16M-entry pieces
    for lo in range(0, d.numel(), step):
        part = d[lo:lo + step]
        idx = torch.arange(part.numel(), device=d.device, dtype=torch.int64) + (first_index + lo)
        acc += (part * (2 * idx + 1)).sum()  # int64 arithmetic wraps mod 2^64
    return int(acc.item()) & MASK64


def _to_signed(v: int) -> int:
    v &= MASK64
    return v - (1 << 64) if v >= 1 << 63 else v


def allreduce_fold(local_fold: int, device=None) -> int:
    """Sum of per-rank folds mod 2^64 (int64 two's-complement wraparound)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([_to_signed(local_fold)], dtype=torch.int64, device=device)
    if _grouped():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item()) & MASK64


def allreduce_max(values, device=None) -> list[float]:
    """Element-wise max over ranks (the bench's elapsed / kernel times)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if _grouped():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def allreduce_min_int(v: int, device=None) -> int:
    """Min over ranks of a small integer (the bench's per-shard parity status)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(v)], dtype=torch.int64, device=device)
    if _grouped():
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def allreduce_min_flag(ok: bool, device=None) -> bool:
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=device)
    if _grouped():
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def exchange_buckets(keys_out, mbits_out, offsets, index_out=None):
    """Ship every bucket to its owner rank: bucket r of this rank (rows
    offsets[r]:offsets[r+1] of the bucketed outputs, pdht_amd.bucket_batch
    with nranks == world size) goes to rank r with one all-to-all(v) per
    payload (RCCL over xGMI on GPUs, gloo on CPU).

    Returns (keys [m, L], mbits [m], index [m] | None, recv_counts [world]):
    all keys this rank owns (mbits % world == rank), grouped by source rank in
    rank order, each group in its source's key order.  The only collective on
    the placement path: the first step that needs one.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    if offsets.numel() != world + 1:
        raise ValueError("bucket_batch must have been called with nranks == world size")
    send = (offsets[1:] - offsets[:-1]).to(torch.int64)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    s_split = [int(x) for x in send.cpu().tolist()]
    r_split = [int(x) for x in recv.cpu().tolist()]
    m = sum(r_split)

    def a2a(t):
        out = torch.empty((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_to_all_single(out, t.contiguous(), r_split, s_split)
        return out

    keys = a2a(keys_out) if keys_out is not None else None
    mbits = a2a(mbits_out)
    index = a2a(index_out) if index_out is not None else None
    return keys, mbits, index, recv


def exchange_records(records, offsets):
    """Ship wire records (pdht_amd.bucket_records with nranks == world size)
    to their owner ranks: ONE all-to-all(v) of the record bytes instead of one
    per payload (exchange_buckets).  Returns (records [m, stride] uint8,
    recv_counts [world]): every record this rank owns, grouped by source rank
    in rank order, each group in its source's key order."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    if offsets.numel() != world + 1:
        raise ValueError("bucket_records must have been called with nranks == world size")
    rb = records.shape[1]
    send = (offsets[1:] - offsets[:-1]).to(torch.int64)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    s_split = [int(x) * rb for x in send.cpu().tolist()]
    r_split = [int(x) * rb for x in recv.cpu().tolist()]
    out = torch.empty(sum(r_split), dtype=torch.uint8, device=records.device)
    dist.all_to_all_single(out, records.contiguous().view(-1), r_split, s_split)
    return out.view(-1, rb), recv


def device_info(device=None) -> dict:
    """Where this rank runs: host, device index, name and PCI address (the
    RCCL world / device map of a multi-GPU bench line)."""
    import socket
    info = {"host": socket.gethostname()}
    if device is not None and getattr(device, "type", "cpu") == "cuda":
        import torch
        p = torch.cuda.get_device_properties(device)
        info.update(device=device.index, name=p.name,
                    pci=f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                        f"{getattr(p, 'pci_device_id', 0):02x}")
    else:
        info.update(device=None, name="cpu", pci=None)
    return info


def per_rank_report(rank: int, local: int, world: int, n: int, bytes_per_key: float, kernel_ms: float,
                    elapsed_s: float, steps: int, peak_GBps: float, device=None) -> dict:
    """Every rank's own numbers, gathered to all ranks: device, kernel time,
    Gkeys/s and roofline fraction per GPU, plus the world (SURVEY.md §8e:
    per-GPU and aggregate Gkeys/s at 1/2/4/8 GPUs)."""
    import torch.distributed as dist
    mine = dict(rank=rank, local_rank=local, **device_info(device), keys=n,
                event_ms=round(kernel_ms, 4),
                Gkeys_s=round(n / (kernel_ms / 1e3) / 1e9, 3),
                frac=round(bytes_per_key * n / (kernel_ms / 1e3) / 1e9 / peak_GBps, 4),
                wall_Gkeys_s=round(n * steps / elapsed_s / 1e9, 3))
    if _grouped():
        allr = [None] * dist.get_world_size()
        dist.all_gather_object(allr, mine)
        backend = dist.get_backend()
    else:
        allr, backend = [mine], None
    return {"world_size": len(allr), "backend": backend, "ranks": allr,
            "Gkeys_s": [r["Gkeys_s"] for r in allr], "frac": [r["frac"] for r in allr],
            "aggregate_kernel_Gkeys_s": round(sum(r["Gkeys_s"] for r in allr), 3)}


def barrier():
    import torch.distributed as dist
    if _grouped():
        dist.barrier()
