#!/usr/bin/env python3
"""Host-side cost of one batch call (tools only): the Python wrapper of
pdht_amd against the bare ctypes call with prebuilt arguments, on a tiny
batch (the kernel is negligible; the launch queue never runs dry of work the
CPU could not keep up with).  Prints one JSON line per form, us per call."""
import ctypes as C
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import pdht_amd as P  # noqa: E402


def per_call(fn, reps=2000):
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / reps * 1e6


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = 4096
    keys = torch.randint(0, 256, (n, 64), dtype=torch.uint8, device=dev)
    hist = torch.zeros(4, dtype=torch.int64, device=dev)
    outs = P.place_batch(keys, 1, 4, hist=hist)
    out64 = torch.empty(n, dtype=torch.int64, device=dev)
    lib = P.lib()
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (C.c_void_p(keys.data_ptr()), 64, n, 1, 4, C.c_void_p(outs[0].data_ptr()),
            C.c_void_p(outs[1].data_ptr()), C.c_void_p(outs[2].data_ptr()), 4, C.c_void_p(hist.data_ptr()), s)
    forms = {
        "place_batch (wrapper)": lambda: P.place_batch(keys, 1, 4, hist=hist, out=outs),
        "pdht_place_batch_dev (bare ctypes)": lambda: lib.pdht_place_batch_dev(*args),
        "city64_batch (wrapper)": lambda: P.city64_batch(keys, out=out64),
        "torch.cuda.current_stream()": lambda: torch.cuda.current_stream(dev).cuda_stream,
        "torch.cuda.device guard": lambda: torch.cuda.device(dev).__enter__(),
    }
    for name, fn in forms.items():
        print(json.dumps({"form": name, "us_per_call": round(per_call(fn), 2)}), flush=True)


if __name__ == "__main__":
    main()
