#!/usr/bin/env python3
"""Kernel-variant A/B for the 64-byte CityHash64 path (one process, interleaved
rounds, HIP events on the launch stream; MI355X_MICROARCH / guide rule 24).

  python tools/kbench.py [--n 16777216] [--rounds 5] [--reps 10]
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

NAMES = {0: "xpose nt/nt depth 2, 3 WG/CU (default)", 1: "xpose plain", 2: "lds-dma+prefetch",
         3: "window", 4: "lds-dma nt-store", 5: "direct nt-load nt-store", 6: "direct plain",
         7: "xpose nt/nt depth 1, 4 WG/CU", 8: "xpose nt-store", 9: "direct nt-store",
         15: "xpose nt/nt depth 2, 4 WG/CU", 26: "xpose nt-load plain-store depth 2"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0,1,2,4,5,6,8,9,3")
    ap.add_argument("--per-cu", default="0")
    ap.add_argument("--algo", default="city64", choices=["city64", "crc128"])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = a.n
    words = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, n * 8, device=dev)
    keys = words.view(torch.uint8).view(n, 64)
    w = 1 if a.algo == "city64" else 2
    out = torch.empty((n,) if w == 1 else (n, 2), dtype=torch.int64, device=dev)
    fn = P.city64_batch if a.algo == "city64" else P.citycrc128_batch
    bpk = 64 + 8 * w
    variants = [int(v) for v in a.variants.split(",")]
    percus = [int(x) for x in a.per_cu.split(",")]
    # achievable read bandwidth on this box (same buffer, read-only stream)
    for nt in (False, True):
        P.read_stream(keys, nt)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.reps * a.rounds)]
        for s, e in ev:
            s.record()
            P.read_stream(keys, nt)
            e.record()
        torch.cuda.synchronize()
        med = float(np.median([s.elapsed_time(e) for s, e in ev]))
        print(json.dumps({"read_stream": "nt" if nt else "plain", "median_ms": round(med, 4),
                          "GBps": round(n * 64 / med / 1e6, 1)}))
    ref = None
    times = {}
    for v in variants:
        for pc in percus:
            os.environ["PDHT_HIP_BLOCKS_PER_CU"] = str(pc)
            P.set_variant(v)
            fn(keys, out=out)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            ok = bool(torch.equal(out, ref))
            times[(v, pc)] = {"ok": ok, "ms": [], "kernel": P.last_kernel()}
    for _ in range(a.rounds):
        for v in variants:
            for pc in percus:
                os.environ["PDHT_HIP_BLOCKS_PER_CU"] = str(pc)
                P.set_variant(v)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.reps)]
                for s, e in ev:
                    s.record()
                    fn(keys, out=out)
                    e.record()
                torch.cuda.synchronize()
                times[(v, pc)]["ms"].extend(s.elapsed_time(e) for s, e in ev)
    res = []
    for (v, pc), t in times.items():
        med = float(np.median(t["ms"]))
        mn = float(np.min(t["ms"]))
        res.append({"variant": v, "name": NAMES.get(v, str(v)), "per_cu": pc, "kernel": t["kernel"],
                    "ok": t["ok"], "median_ms": round(med, 4), "min_ms": round(mn, 4),
                    "GBps_median": round(n * bpk / med / 1e6, 1),
                    "frac_8TBps": round(n * bpk / med / 1e6 / 8000, 4)})
    for r in sorted(res, key=lambda r: r["median_ms"]):
        print(json.dumps(r))
    P.set_variant(0)


if __name__ == "__main__":
    main()
