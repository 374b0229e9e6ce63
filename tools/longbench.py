#!/usr/bin/env python3
"""Long-key throughput: CityHash64 / CityHash128 /
CityHashCrc128 over packed fixed-length keys of 256 B .. 8 KiB (1 GiB of keys
per case), HIP events on the launch stream, median of --reps.  Crc128 above
900 B runs CityHashCrc256's CRC-32C rounds (city.c:407-517).

  python tools/longbench.py [--lens 256,1024,4096] [--reps 10]
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
    ap.add_argument("--lens", default="256,901,1024,4096,8192")
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--algos", default="city64,city128,crc128")
    ap.add_argument("--variants", default="0")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    fns = {"city64": (P.city64_batch, 8), "city128": (P.city128_batch, 16),
           "crc128": (P.citycrc128_batch, 16)}
    for L in [int(x) for x in a.lens.split(",")]:
        n = a.bytes // L
        words = P.splitmix64_fill(0x5EED5EED5EED5EED, 0, (n * L + 7) // 8, device=dev)
        keys = words.view(torch.uint8)[: n * L].view(n, L)
        for name, v in [(x, int(y)) for x in a.algos.split(",") for y in a.variants.split(",")]:
            P.set_variant(v)
            fn, d = fns[name]
            out = torch.empty((n,) if d == 8 else (n, 2), dtype=torch.int64, device=dev)
            fn(keys, out=out)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.reps)]
            for s, e in ev:
                s.record()
                fn(keys, out=out)
                e.record()
            torch.cuda.synchronize()
            med = float(np.median([s.elapsed_time(e) for s, e in ev]))
            gbps = n * (L + d) / med / 1e6
            print(json.dumps({"algo": name, "variant": v, "key_bytes": L, "keys": n, "kernel": P.last_kernel(),
                              "median_ms": round(med, 4), "Gkeys_s": round(n / med / 1e6, 3),
                              "GBps": round(gbps, 1), "frac_8TBps": round(gbps / 8000, 4)}), flush=True)
        del keys, words
    P.set_variant(0)


if __name__ == "__main__":
    main()
