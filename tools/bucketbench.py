#!/usr/bin/env python3
"""Destination-bucketing A/B: pdht_bucket_batch_dev on
packed keys, kernel variants interleaved in one process, plus the per-phase
shader-clock split of the scatter kernel (pdht_hip_set_phase_counters).

  python tools/bucketbench.py [--n 16777216] [--L 8] [--nranks 1024] [--variants 0,41]
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

PHASES = ["load+hash", "count", "scan+starts", "rank+stage", "gather+prefetch", "stores"]


def timeit(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return [s.elapsed_time(e) for s, e in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16 << 20)
    ap.add_argument("--L", type=int, default=8)
    ap.add_argument("--nranks", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0,41")
    ap.add_argument("--per-cu", default="", help="comma list of PDHT_HIP_SCATTER_PER_CU values to sweep")
    a = ap.parse_args()
    if a.per_cu:  # each (variant, blocks per CU) pair becomes its own case
        pcs = [int(x) for x in a.per_cu.split(",")]
        a.variants = ",".join(f"{v}@{p}" for v in a.variants.split(",") for p in pcs)
    dev = torch.device("cuda:0")
    n, L, nr = a.n, a.L, a.nranks
    variants = a.variants.split(",")

    def use(v):
        """'v' or 'v@blocks_per_cu'"""
        var, _, pc = v.partition("@")
        P.set_variant(int(var))
        if pc:
            os.environ["PDHT_HIP_SCATTER_PER_CU"] = pc
        else:
            os.environ.pop("PDHT_HIP_SCATTER_PER_CU", None)
    w = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, n * L // 8, device=dev)
    keys = w.view(torch.uint8).view(n, L)
    ws = torch.empty(P.bucket_workspace_bytes(n, nr), dtype=torch.uint8, device=dev)
    outs = P.bucket_batch(keys, 3, nr, workspace=ws)
    fn = lambda: P.bucket_batch(keys, 3, nr, out=outs, workspace=ws)  # noqa: E731
    bpk = L + L + 8 + 8 + 4
    ms = {v: [] for v in variants}
    kern, ref = {}, None
    for v in variants:
        use(v)
        fn()
        kern[v] = P.last_kernel()
        got = [t.clone() for t in outs]
        if ref is None:
            ref = got
        elif not all(bool(torch.equal(x, y)) for x, y in zip(got, ref)):
            print(json.dumps({"variant": v, "error": "output differs from the first variant"}), flush=True)
    for _ in range(a.rounds):
        for v in variants:
            use(v)
            ms[v].extend(timeit(fn, a.reps))
    for v in variants:
        use(v)
        ctr = torch.zeros(16, dtype=torch.int64, device=dev)
        P.set_phase_counters(ctr)
        try:
            fn()
            torch.cuda.synchronize()
        finally:
            P.set_phase_counters(None)
        c = ctr.cpu().numpy()
        tot = max(1, int(c[:6].sum()))
        med = float(np.median(ms[v]))
        print(json.dumps({"case": f"bucket L={L} nranks={nr} n={n}", "variant": v, "kernel": kern[v],
                          "median_ms": round(med, 4), "Gkeys_s": round(n / med / 1e6, 2),
                          "GBps": round(n * bpk / med / 1e6, 1),
                          "frac_8TBps": round(n * bpk / med / 1e6 / 8000, 4), "tiles": int(c[8]),
                          "cycles_per_tile": round(tot / max(1, int(c[8])), 1),
                          "phase_share": {p: round(int(c[k]) / tot, 3) for k, p in enumerate(PHASES)}}),
              flush=True)
    use("0")


if __name__ == "__main__":
    main()
