#!/usr/bin/env python3
"""Summarise a rocprofv3 counter-collection CSV: mean per dispatch of every
(kernel, counter) pair (kernels whose name contains `pdht`).

  python tools/pmc_summary.py gpurun_out/sq_cfg3/run_counter_collection.csv
"""
import collections
import csv
import sys


def summary(path, match="pdht"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "")
        if match not in name:
            continue
        key = (name[:110], r["Counter_Name"])
        acc[key][r["Dispatch_Id"]] += float(r["Counter_Value"])
        disp[name[:110]].add(r["Dispatch_Id"])
    out = {}
    for (k, c), d in sorted(acc.items()):
        out.setdefault(k, {})[c] = sum(d.values()) / len(d)
    return out


if __name__ == "__main__":
    for k, cs in summary(sys.argv[1], *(sys.argv[2:3])).items():
        print(k)
        for c, v in cs.items():
            print(f"   {c:28s} {v:16.0f}")
