#!/usr/bin/env python3
"""Small-key A/B: fused placement (pdht_hash over a batch) and plain
CityHash64 on 8/16-byte keys, kernel variants interleaved in one process.

  python tools/placebench.py [--n 16777216] [--variants 0,16,17]
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0,16,17")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = a.n
    variants = [int(x) for x in a.variants.split(",")]
    cases = []
    for L in (8, 16):
        w = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, n * L // 8, device=dev)
        keys = w.view(torch.uint8).view(n, L)
        hist = torch.zeros(1024, dtype=torch.int64, device=dev)
        outs = P.place_batch(keys, 3, 1024, hist=hist)
        o64 = torch.empty(n, dtype=torch.int64, device=dev)
        cases.append((f"place L={L} nptes=3 nranks=1024 +hist", L + 8 + 4 + 4,
                      (lambda k=keys, h=hist, o=outs: P.place_batch(k, 3, 1024, hist=h, out=o))))
        outs2 = P.place_batch(keys, 3, 1024)
        cases.append((f"place L={L} nptes=3 nranks=1024 no-hist", L + 8 + 4 + 4,
                      (lambda k=keys, o=outs2: P.place_batch(k, 3, 1024, out=o))))
        cases.append((f"city64 L={L}", L + 8, (lambda k=keys, o=o64: P.city64_batch(k, out=o))))
    for name, bpk, fn in cases:
        ms = {v: [] for v in variants}
        kern = {}
        for v in variants:
            P.set_variant(v)
            fn()
            kern[v] = P.last_kernel()
        for _ in range(a.rounds):
            for v in variants:
                P.set_variant(v)
                ms[v].extend(timeit(fn, a.reps))
        for v in variants:
            med = float(np.median(ms[v]))
            print(json.dumps({"case": name, "variant": v, "kernel": kern[v], "median_ms": round(med, 4),
                              "Gkeys_s": round(n / med / 1e6, 2), "GBps": round(n * bpk / med / 1e6, 1),
                              "frac_8TBps": round(n * bpk / med / 1e6 / 8000, 4)}))
    P.set_variant(0)


if __name__ == "__main__":
    main()
