#!/usr/bin/env python3
"""Static instruction counts of a kernel's loops from an ISA listing
(`make asm`, or hipcc --cuda-device-only -S of one unit): for every loop
(a backward branch to a label inside the kernel) the VALU / LDS / VMEM / SALU
counts, innermost first.  Used for the long-key CityHashCrc256 block loop
(DESIGN.md §4.3): the loop whose LDS count is 240 is one 240-B block (30
CRC-32C updates of 8 lookups).

  python tools/isa_counts.py build/pdht_fixed128.s 'k_globalILb0ENS_6CrcLdsINS_10AlgoCrc128ELi8EEENS_8Sink128TILb1EEELb1ELi5E'
"""
import collections
import re
import sys


def kernel_body(path, pattern):
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and pattern in l]
    if not starts:
        raise SystemExit(f"no kernel matching {pattern}")
    s = starts[0]
    e = s + 1
    while e < len(lines) and not lines[e].startswith(".Lfunc_end"):
        e += 1
    return lines[s:e]


def loops(body):
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    out = set()
    for i, l in enumerate(body):
        m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            out.add((labels[m.group(1)], i))
    return sorted(out, key=lambda x: x[1] - x[0])


def mix(body, a, b):
    c = collections.Counter()
    for l in body[a:b + 1]:
        m = re.match(r"\s+([a-z_0-9]+)", l)
        if m and not l.strip().startswith(";"):
            c[m.group(1)] += 1
    return c


def main():
    path, pattern = sys.argv[1], sys.argv[2]
    body = kernel_body(path, pattern)
    print(f"kernel {pattern}: {len(body)} lines")
    for a, b in loops(body):
        c = mix(body, a, b)
        cls = {"VALU": sum(v for k, v in c.items() if k.startswith("v_")),
               "LDS": sum(v for k, v in c.items() if k.startswith("ds_")),
               "VMEM": sum(v for k, v in c.items() if k.startswith(("global_", "buffer_"))),
               "SALU": sum(v for k, v in c.items() if k.startswith("s_") and not k.startswith("s_waitcnt"))}
        top = ", ".join(f"{k} {v}" for k, v in c.most_common(8))
        print(f"loop [{a}, {b}] {b - a} lines: " + " ".join(f"{k} {v}" for k, v in cls.items()) + f"  | {top}")


if __name__ == "__main__":
    main()
