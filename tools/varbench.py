#!/usr/bin/env python3
"""Variable-length kernel A/B: kernel variants x length distributions, one
process, rounds interleaved (guide §5.4 rule 24), HIP events on the stream.

  python tools/varbench.py [--n 16777216] [--variants 0,3,14] [--rounds 5]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16 << 20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--cases", default="mixed16-256,const136,const64,mixed129-256")
    ap.add_argument("--max-bytes", type=int, default=3 << 30, help="cap on key bytes per case")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    data = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, a.max_bytes // 8, device=dev).view(torch.uint8)
    S = 0x1E575EED1E575EED
    cases = {  # name -> (lo, hi) uniform lengths
        "mixed16-256": (16, 256), "const136": (136, 136), "const200": (200, 200), "const64": (64, 64),
        "mixed65-128": (65, 128), "mixed129-256": (129, 256), "mixed256-768": (256, 768),
        "mixed1k-3k": (1024, 3072),
    }
    variants = [int(x) for x in a.variants.split(",")]
    for case in a.cases.split(","):
        lo, hi = cases[case]
        n = min(a.n, a.max_bytes // hi)
        lens = (torch.full((n,), lo, dtype=torch.int64, device=dev) if lo == hi
                else P.mixed_lengths(S, 0, n, lo, hi, device=dev))
        offs = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens, 0, out=offs[1:])
        total = int(offs[-1].item())
        d = data[:total]
        out = torch.empty(n, dtype=torch.int64, device=dev)
        ref = None
        ms = {v: [] for v in variants}
        kern = {}
        for v in variants:  # warm-up + parity between variants
            P.set_variant(v)
            P.city64_var_batch(d, offs, out=out)
            kern[v] = P.last_kernel()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), (case, v)
        for _ in range(a.rounds):
            for v in variants:
                P.set_variant(v)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.reps)]
                for s, e in ev:
                    s.record()
                    P.city64_var_batch(d, offs, out=out)
                    e.record()
                torch.cuda.synchronize()
                ms[v].extend(s.elapsed_time(e) for s, e in ev)
        bpk = total / n + 16
        for v in variants:
            med = float(np.median(ms[v]))
            print(json.dumps({"case": case, "variant": v, "kernel": kern[v], "mean_len": round(total / n, 1),
                              "median_ms": round(med, 4), "Gkeys_s": round(n / med / 1e6, 2),
                              "GBps": round(n * bpk / med / 1e6, 1),
                              "frac_8TBps": round(n * bpk / med / 1e6 / 8000, 4)}))
        del lens, offs, out, ref
    P.set_variant(0)


if __name__ == "__main__":
    main()
