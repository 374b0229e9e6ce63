#!/usr/bin/env python3
"""Interleaved A/B of kernel variants (tuning build, libpdht_hip_tuning.so):
one process, rounds interleaved across variants, HIP events on the launch
stream; every variant's output is compared with the product kernel's.

  python tools/abbench.py --work cfg2 --variants 0,7,26 [--per-cu 0,2,3,4]
  works: cfg2 (16M x 64 B City64), cfg4 (Crc128), cfg3 (64M mixed 16..256 B),
         cfg3c (64M x 136 B through the variable-length path), cfg3s<G> / cfg3sall
         (cfg3 with the lengths sorted inside groups of G keys / overall), cfg3fold (cfg3's
         window data movement: fold of the bytes; variant 40 = no LDS reads),
         varfold_<L> (64M x L-B fixed keys through the var calibration entry),
         long (1M x 1 KiB Crc128), long64 (1M x 1 KiB City64),
         place (16M x 8 B, nptes 3, nranks 1024, histogram),
         bucket (16M x 8 B, 1024 ranks, keys+mbits+ptindex+index),
         bucket_<L>_<nranks> / records_<L>_<nranks>, place<L>_<nranks>, cfg1 / cfg1nohist;
         with inputs rotated past the 256 MiB Infinity Cache (as bench.py measures):
         cfg1rot, placerot, place16rot, city8rot / city16rot / city32rot,
         bucketrot, recordsrot, bucket8krot (outputs rotated too);
         diagnostics of the bucketing count kernel: bucketgap, gaponly,
         bucketpg, bucketpg64k, bucketwarm
Variant 0 runs through the PRODUCT library; the others through the tuning
build (pdht_amd.tuning).  Numbers: median / min ms and algorithmic GB/s.
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
M = 1 << 20


def workload(name, dev):
    """(step(), result-for-equality(), algorithmic bytes per step)"""
    if name.startswith(("bucket_", "records_")):  # bucket_<L>_<nranks>, records_<L>_<nranks>
        kind, L, nr = name.split("_")
        L, nr, n = int(L), int(nr), 16 * M
        keys = P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L)
        with P.tuning(0):  # the tuning build reserves the two-pass intermediate at any nranks
            wsb = P.bucket_workspace_bytes(n, L, nr)
        ws = torch.empty(max(wsb, P.bucket_workspace_bytes(n, L, nr)), dtype=torch.uint8, device=dev)
        if kind == "records":
            outs = P.bucket_records(keys, nr, workspace=ws)
            return ((lambda: P.bucket_records(keys, nr, out=outs, workspace=ws)),
                    (lambda: torch.cat([outs[0].view(-1)[:1 << 20].long(), outs[1]])),
                    n * (L + P.bucket_record_bytes(L)))
        outs = P.bucket_batch(keys, 3, nr, workspace=ws)
        return ((lambda: P.bucket_batch(keys, 3, nr, out=outs, workspace=ws)),
                (lambda: torch.cat([outs[1], outs[3].long(), outs[4]])), n * (L + L + 8 + 4 + 4))
    if name.startswith(("place64_", "place16_", "place8_")):  # place<L>_<nranks>: 16M keys, nptes 3, + hist
        nr, n, L = int(name.split("_")[1]), 16 * M, int(name.split("_")[0][5:])
        keys = P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L)
        hist = torch.zeros(nr, dtype=torch.int64, device=dev)
        outs = P.place_batch(keys, 3, nr, hist=hist)
        return ((lambda: P.place_batch(keys, 3, nr, hist=hist, out=outs)),
                (lambda: torch.cat([outs[0], outs[1].long(), outs[2].long()])), n * (L + 16))
    if name in ("cfg1", "cfg1nohist"):  # 1M x 64 B, pdht_hash semantics (nptes 1, 4 ranks) [+ histogram]
        n, L = M, 64
        keys = P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L)
        hist = torch.zeros(4, dtype=torch.int64, device=dev) if name == "cfg1" else None
        outs = P.place_batch(keys, 1, 4, hist=hist)
        return ((lambda: P.place_batch(keys, 1, 4, hist=hist, out=outs)),
                (lambda: torch.cat([outs[0], outs[1].long(), outs[2].long()])), n * 80)
    if name in ("cfg5rot", "cfg5fix", "cfg5roto"):
        # 16M-key slices of cfg5's 128M-key buffer: rotating / always slice 3
        # (one 128 MiB digest buffer); roto: rotating keys AND digest slices
        # of a 1 GiB digest buffer
        n, L = 16 * M, 64
        keys = P.splitmix64_fill(SEED, 0, 8 * n * L // 8, device=dev).view(torch.uint8).view(8 * n, L)
        out = torch.empty(8 * n if name == "cfg5roto" else n, dtype=torch.int64, device=dev)
        turn = [0]

        def step():
            j = turn[0] % 8 if name != "cfg5fix" else 3
            turn[0] += 1
            o = out[j * n:(j + 1) * n] if name == "cfg5roto" else out
            P.city64_batch(keys[j * n:(j + 1) * n], out=o)
        return step, (lambda: out[:1].clone()), n * (L + 8)
    if name in ("long128", "long128s"):  # 2M x 512 B CityHash128 (city.c:378-400) / WithSeed (:310-376)
        n, L = 2 * M, 512
        keys = P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L)
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
        if name == "long128":
            return (lambda: P.city128_batch(keys, out=out)), (lambda: out.clone()), n * (L + 16)
        return ((lambda: P.city128_seed_batch(keys, (0x0123456789ABCDEF, 0xFEDCBA9876543210), out=out)),
                (lambda: out.clone()), n * (L + 16))
    if name in ("city8rot", "city16rot", "city32rot"):
        # CityHash64 of 16M x 8/16/32-B keys (no placement), keys rotated over 4 copies
        n, L = 16 * M, int(name[4:-3])
        ks = [P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L) for _ in range(4)]
        out = torch.empty(n, dtype=torch.int64, device=dev)
        turn = [0]

        def step():
            P.city64_batch(ks[turn[0] % 4], out=out)
            turn[0] += 1
        return step, (lambda: out.clone()), n * (L + 8)
    if name == "cfg1rot":
        # cfg1 (1M x 64 B, nptes 1, 4 ranks, histogram) with the keys rotated
        # over 8 copies (512 MiB), as bench.py measures it
        n, L = M, 64
        ks = [P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L) for _ in range(8)]
        hist = torch.zeros(4, dtype=torch.int64, device=dev)
        outs = P.place_batch(ks[0], 1, 4, hist=hist)
        turn = [0]

        def step():
            P.place_batch(ks[turn[0] % 8], 1, 4, hist=hist, out=outs)
            turn[0] += 1
        return step, (lambda: torch.cat([outs[0], outs[1].long(), outs[2].long()])), n * 80
    if name in ("placerot", "place16rot"):
        # place (16M x 8 / 16 B, nptes 3, 1024 ranks, histogram) with the KEYS
        # rotated over 4 sets (>= 512 MiB): no step finds its keys still in the
        # Infinity Cache from the step before
        n, L = 16 * M, (8 if name == "placerot" else 16)
        ks = [P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L) for _ in range(4)]
        hist = torch.zeros(1024, dtype=torch.int64, device=dev)
        outs = P.place_batch(ks[0], 3, 1024)
        turn = [0]

        def step():
            P.place_batch(ks[turn[0] % 4], 3, 1024, hist=hist, out=outs)
            turn[0] += 1
        return step, (lambda: torch.cat([outs[0], outs[1].long(), outs[2].long()])), n * (L + 16)
    if name in ("bucket2s", "bucket8k2s", "records2s"):
        # two batches per step, bucketed concurrently on two streams (each its
        # own workspace and outputs; keys and outputs rotated over 4 sets):
        # the bulk-loader shape of consecutive batches in flight together
        n = 16 * M
        nr = 8192 if name == "bucket8k2s" else 1024
        kk = [P.splitmix64_fill(SEED, 0, n, device=dev).view(torch.uint8).view(n, 8) for _ in range(4)]
        wss = [torch.empty(P.bucket_workspace_bytes(n, 8, nr), dtype=torch.uint8, device=dev) for _ in range(2)]
        rec = name == "records2s"
        sets = [P.bucket_records(k, nr, workspace=wss[0]) if rec else P.bucket_batch(k, 3, nr, workspace=wss[0])
                for k in kk]
        strs = [torch.cuda.Stream(device=dev) for _ in range(2)]
        turn = [0]

        def step():
            cur = torch.cuda.current_stream(dev)
            for s_ in strs:
                s_.wait_stream(cur)
            for q in range(2):
                j = (turn[0] + q) % 4
                with torch.cuda.stream(strs[q]):
                    if rec:
                        P.bucket_records(kk[j], nr, out=sets[j], workspace=wss[q], stream=strs[q])
                    else:
                        P.bucket_batch(kk[j], 3, nr, out=sets[j], workspace=wss[q], stream=strs[q])
            turn[0] += 2
            for s_ in strs:
                cur.wait_stream(s_)
        per = 40 if rec else 32
        return step, (lambda: sets[0][1][:1 << 20].clone()), 2 * n * per
    if name.startswith("bucketn_"):
        # bucketn_<M>_<nranks>: 8-B keys, n = M x 2^20, keys and outputs
        # rotated over 4 sets (per-key cost against n at any rank count)
        _, mm, nr = name.split("_")
        n, nr = int(mm) * M, int(nr)
        kk = [P.splitmix64_fill(SEED, 0, n, device=dev).view(torch.uint8).view(n, 8) for _ in range(4)]
        with P.tuning(0):
            wsb = P.bucket_workspace_bytes(n, 8, nr)
        ws = torch.empty(max(wsb, P.bucket_workspace_bytes(n, 8, nr)), dtype=torch.uint8, device=dev)
        sets = [P.bucket_batch(k, 3, nr, workspace=ws) for k in kk]
        turn = [0]

        def step():
            j = turn[0] % 4
            turn[0] += 1
            P.bucket_batch(kk[j], 3, nr, out=sets[j], workspace=ws)
        return step, (lambda: torch.cat([sets[0][1], sets[0][3].long(), sets[0][4]])), n * 32
    if name.startswith("bucket8kn_"):
        # bucket8krot's setup at n = <M> x 2^20 keys (per-key cost against n:
        # how much of the two-pass intermediate the Infinity Cache holds)
        n = int(name.split("_")[1]) * M
        kk = [P.splitmix64_fill(SEED, 0, n, device=dev).view(torch.uint8).view(n, 8) for _ in range(4)]
        ws = torch.empty(P.bucket_workspace_bytes(n, 8, 8192), dtype=torch.uint8, device=dev)
        sets = [P.bucket_batch(k, 3, 8192, workspace=ws) for k in kk]
        turn = [0]

        def step():
            j = turn[0] % 4
            turn[0] += 1
            P.bucket_batch(kk[j], 3, 8192, out=sets[j], workspace=ws)
        return step, (lambda: torch.cat([sets[0][1], sets[0][3].long(), sets[0][4]])), n * 32
    if name in ("bucketrot", "recordsrot", "bucket8krot"):
        # bucket / records at 1024 ranks (bucket8k: 8192 ranks, two passes)
        # with the keys rotated over 4 copies and the outputs over 4 sets, as
        # bench.py measures them: no output line can still sit in the
        # Infinity Cache when its address is written again
        n = 16 * M
        nr = 8192 if name == "bucket8krot" else 1024
        kk = [P.splitmix64_fill(SEED, 0, n, device=dev).view(torch.uint8).view(n, 8) for _ in range(4)]
        with P.tuning(0):  # the tuning / experiment builds reserve the two-pass intermediate too
            wsb = P.bucket_workspace_bytes(n, 8, nr)
        ws = torch.empty(max(wsb, P.bucket_workspace_bytes(n, 8, nr)), dtype=torch.uint8, device=dev)
        if name == "recordsrot":
            sets = [P.bucket_records(k, nr, workspace=ws) for k in kk]
        else:
            sets = [P.bucket_batch(k, 3, nr, workspace=ws) for k in kk]
        turn = [0]

        def step():
            j = turn[0] % 4
            turn[0] += 1
            if name == "recordsrot":
                P.bucket_records(kk[j], nr, out=sets[j], workspace=ws)
            else:
                P.bucket_batch(kk[j], 3, nr, out=sets[j], workspace=ws)
        if name == "recordsrot":
            return step, (lambda: torch.cat([sets[0][0].view(-1)[:1 << 20].long(), sets[0][1]])), n * 40
        return step, (lambda: torch.cat([sets[0][1], sets[0][3].long(), sets[0][4]])), n * 32
    if name in ("bucketpg", "bucketpg64k", "bucketwarm"):
        # before each bucketing step, touch the keys: one byte per 4 KiB page
        # (pg) / per 64 KiB (pg64k) -- translations warm, data not -- or read
        # them all (warm: translations and the Infinity Cache both warm)
        n = 16 * M
        keys = P.splitmix64_fill(SEED, 0, n, device=dev).view(torch.uint8).view(n, 8)
        ws = torch.empty(P.bucket_workspace_bytes(n, 8, 1024), dtype=torch.uint8, device=dev)
        outs = P.bucket_batch(keys, 3, 1024, workspace=ws)
        flat = keys.view(-1)
        gout = torch.zeros(1, dtype=torch.int64, device=dev)
        st = 4096 if name == "bucketpg" else 65536

        def step():
            if name == "bucketwarm":
                P.read_stream(flat, True, out=gout)
            else:
                gout.copy_(flat[::st].to(torch.int64).sum().view(1))
            P.bucket_batch(keys, 3, 1024, out=outs, workspace=ws)
        return step, (lambda: torch.cat([outs[1], outs[3].long(), outs[4]])), n * 32
    if name in ("bucketgap", "gaponly"):
        # diagnostics of the count kernel's "drain" (DESIGN.md §4.4): bucketing
        # steps with a 1 GiB read-only stream between them (bucketgap), and that
        # stream alone (gaponly); rocprof tells the kernels apart
        n = 16 * M
        gap = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
        gout = torch.zeros(1, dtype=torch.int64, device=dev)
        if name == "gaponly":
            return (lambda: P.read_stream(gap, True, out=gout)), (lambda: gout.clone()), 1 << 30
        keys = P.splitmix64_fill(SEED, 0, n, device=dev).view(torch.uint8).view(n, 8)
        ws = torch.empty(P.bucket_workspace_bytes(n, 8, 1024), dtype=torch.uint8, device=dev)
        outs = P.bucket_batch(keys, 3, 1024, workspace=ws)

        def step():
            P.bucket_batch(keys, 3, 1024, out=outs, workspace=ws)
            P.read_stream(gap, True, out=gout)
        return step, (lambda: torch.cat([outs[1], outs[3].long(), outs[4]])), n * 32 + (1 << 30)
    if name in ("cfg2", "cfg5", "cfg4", "long", "long64", "place", "bucket"):
        L = {"cfg2": 64, "cfg5": 64, "cfg4": 64, "long": 1024, "long64": 1024, "place": 8, "bucket": 8}[name]
        n = M if name in ("long", "long64") else 128 * M if name == "cfg5" else 16 * M
        keys = P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8).view(n, L)
        if name in ("cfg2", "cfg5", "long64"):
            out = torch.empty(n, dtype=torch.int64, device=dev)
            return (lambda: P.city64_batch(keys, out=out)), (lambda: out.clone()), n * (L + 8)
        if name in ("cfg4", "long"):
            out = torch.empty((n, 2), dtype=torch.int64, device=dev)
            return (lambda: P.citycrc128_batch(keys, out=out)), (lambda: out.clone()), n * (L + 16)
        if name == "place":
            hist = torch.zeros(1024, dtype=torch.int64, device=dev)
            outs = P.place_batch(keys, 3, 1024)
            return ((lambda: P.place_batch(keys, 3, 1024, hist=hist, out=outs)),
                    (lambda: torch.cat([outs[0], outs[1].long(), outs[2].long()])), n * 24)
        with P.tuning(0):
            wsb = P.bucket_workspace_bytes(n, 8, 1024)
        ws = torch.empty(max(wsb, P.bucket_workspace_bytes(n, 8, 1024)), dtype=torch.uint8, device=dev)
        outs = P.bucket_batch(keys, 3, 1024, workspace=ws)
        return ((lambda: P.bucket_batch(keys, 3, 1024, out=outs, workspace=ws)),
                (lambda: torch.cat([outs[1], outs[3].long(), outs[4]])), n * (8 + 8 + 8 + 4 + 4))
    if name.startswith("varfold_"):  # varfold_<L>: 64M x L-B keys through the var calibration entry
        L = int(name.split("_")[1])
        n = 64 * M if L <= 136 else 32 * M
        data = P.splitmix64_fill(SEED, 0, n * L // 8, device=dev).view(torch.uint8)
        offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=dev)
        out = torch.empty(n, dtype=torch.int64, device=dev)
        return (lambda: P.key_stream_var(data, offs, out=out, check=False)), (lambda: out[:1].clone()), n * (L + 16)
    if name not in ("cfg3", "cfg3c", "cfg3fold", "cfg3cfold", "cfg3s128", "cfg3s256", "cfg3s1024", "cfg3sall"):
        raise SystemExit(f"unknown work {name}")
    n = 64 * M
    lo, hi = (136, 136) if name in ("cfg3c", "cfg3cfold") else (16, 256)
    lens = P.mixed_lengths(0x1E575EED1E575EED, 0, n, lo, hi, device=dev)
    if name.startswith("cfg3s"):
        # cfg3's lengths sorted inside every group of G keys (sall: all of them):
        # the same bytes, but each 64-key tile holds keys of similar length --
        # what regrouping keys by length class across G/64 waves could buy
        g = n if name == "cfg3sall" else int(name[5:])
        lens = lens.view(-1, g).sort(dim=1).values.reshape(-1)
    offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    total = int(offs[-1].item())
    data = P.splitmix64_fill(SEED, 0, (total + 7) // 8, device=dev).view(torch.uint8)[:total]
    out = torch.empty(n, dtype=torch.int64, device=dev)
    if name in ("cfg3fold", "cfg3cfold"):  # the window kernel's data movement, hash replaced (40: no LDS reads)
        return (lambda: P.key_stream_var(data, offs, out=out, check=False)), (lambda: out[:1].clone()), total + 16 * n
    return (lambda: P.city64_var_batch(data, offs, out=out, check=False)), (lambda: out.clone()), total + 16 * n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work", default="cfg2")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--per-cu", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pair", action="store_true",
                    help="one event pair around each round's reps (launches queue back to back, as "
                         "bench.py times them); default: a pair per launch")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    step, result, nbytes = workload(a.work, dev)
    # "x<N>" = variant N of the compile-time experiment build (make exp EXP=...),
    # "x<N>:<tag>" = of the build made with EXP_TAG=<tag>
    combos = [(v, int(pc)) for v in a.variants.split(",") for pc in a.per_cu.split(",")]

    class Ctx:
        def __init__(self, v, pc):
            x = str(v).startswith("x")
            vv, _, tag = str(v)[1:].partition(":") if x else (str(v), "", "")
            n = int(vv)
            self.c = P.tuning(n, pc, exp=tag or True) if x else P.tuning(n, pc) if (n or pc) else None

        def __enter__(self):
            if self.c:
                self.c.__enter__()

        def __exit__(self, *e):
            if self.c:
                self.c.__exit__(*e)

    ref, stats = None, {}
    for v, pc in combos:
        with Ctx(v, pc):
            step()
            torch.cuda.synchronize()
            r = result()
            if ref is None:
                ref = r
            stats[(v, pc)] = {"ok": bool(torch.equal(r, ref)), "kernel": P.last_kernel(), "ms": []}
    for _ in range(a.rounds):
        for v, pc in combos:
            with Ctx(v, pc):
                if a.pair:
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.reps):
                        step()
                    e.record()
                    torch.cuda.synchronize()
                    stats[(v, pc)]["ms"].append(s.elapsed_time(e) / a.reps)
                    continue
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.reps)]
                for s, e in ev:
                    s.record()
                    step()
                    e.record()
                torch.cuda.synchronize()
                stats[(v, pc)]["ms"].extend(s.elapsed_time(e) for s, e in ev)
    rows = []
    for (v, pc), t in stats.items():
        med = float(np.median(t["ms"]))
        rows.append({"work": a.work, "variant": v, "per_cu": pc, "kernel": t["kernel"], "ok": t["ok"],
                     "median_ms": round(med, 4), "min_ms": round(float(np.min(t["ms"])), 4),
                     "mean_ms": round(float(np.mean(t["ms"])), 4), "max_ms": round(float(np.max(t["ms"])), 4),
                     "GBps": round(nbytes / med / 1e6, 1), "frac_8TBps": round(nbytes / med / 1e6 / 8000, 4)})
    for r in sorted(rows, key=lambda r: r["median_ms"]):
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
