#!/usr/bin/env python3
"""Measurement table from same-run files: for every config, the bench line
(bench.json) and the rocprofv3 kernel trace of THAT run (run_kernel_trace.csv,
tools/gpu_session.sh hyg_<cfg>).  For each config it prints

  * the bench line's own figures: Gkeys/s, roofline frac (algorithmic bytes
    over the HIP-event time per step), read-only GB/s;
  * the same frac recomputed from the trace: algorithmic bytes per step over
    the summed kernel time per step of the step's launches -- the hash
    kernel's dispatches of the timed steps (the K steps are the last K x
    launches-per-step dispatches before the parity leg; warm-up and
    calibration launches excluded);
  * their ratio, so a reader can check that the event timing and the kernel
    durations agree.

  python tools/hyg_summary.py profiles/r05/hyg [--md]
"""
import csv
import json
import os
import sys

# kernels (substrings of the rocprof symbols) that make up one bench step
STEP_KERNELS = {
    "bucket": ["k_bucket_count_reg", "k_bucket_colscan", "k_bucket_chunkscan", "k_bucket_base",
               "k_bucket_scatter"],
    "records": ["k_bucket_count_reg", "k_bucket_colscan", "k_bucket_chunkscan", "k_bucket_base",
                "k_bucket_scatter"],
    "bucket8k": ["k_bucket_count_tp", "k_bucket_colscan", "k_bucket_chunkscan2", "k_bucket_base",
                 "k_bucket_pass1", "k_bucket_pass2"],
}


def load_line(path):
    for ln in open(path):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


def step_kernel_us(cfg, trace, line):
    """Mean kernel microseconds per timed step, from the trace."""
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps, warm = line["steps"], line["warmup"]
    if cfg in STEP_KERNELS:
        pats = STEP_KERNELS[cfg]
        sel = [r for r in rows if any(p in r["Kernel_Name"] for p in pats)]
        base = [r for r in sel if "k_bucket_base" in r["Kernel_Name"]]  # one per bucketing
        # the timed bucketings: the (warmup + 1)th .. (warmup + steps)th (the first
        # bucketing of every rotation set is the set-up call before the warm-up)
        starts = [int(r["Start_Timestamp"]) for r in base]
        nsets = line["config"].get("rotation", {}).get("output_sets", 1)
        first = nsets + warm
        t0 = starts[first]
        t1 = starts[first + steps] if first + steps < len(starts) else float("inf")
        # a bucketing's count kernel starts before its base kernel: take the
        # dispatches from the count kernel that precedes the first timed base
        prev = [int(r["Start_Timestamp"]) for r in sel if int(r["Start_Timestamp"]) < t0
                and ("count" in r["Kernel_Name"])]
        lo = prev[-1] if prev else t0
        prev1 = [int(r["Start_Timestamp"]) for r in sel if int(r["Start_Timestamp"]) < t1
                 and ("count" in r["Kernel_Name"])]
        hi = prev1[-1] if t1 != float("inf") and prev1 else t1
        tim = [r for r in sel if lo <= int(r["Start_Timestamp"]) < hi]
        tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tim)
        return tot / 1e3 / steps, len(tim)
    tag = line["config"]["kernel"]
    head = tag.split("<")[0]
    sel = [r for r in rows if head in r["Kernel_Name"]]
    per = max(1, round(len(sel) / max(1, steps + warm + 1)))  # launches per step (512-MiB launches)
    # the timed steps: after the warm-up, before anything else runs
    idx = [i for i, r in enumerate(rows) if head in r["Kernel_Name"]]
    # locate the K-step block: the longest run of consecutive same-kernel dispatches
    runs, cur = [], [idx[0]]
    for a, b in zip(idx, idx[1:]):
        if b == a + 1:
            cur.append(b)
        else:
            runs.append(cur)
            cur = [b]
    runs.append(cur)
    block = max(runs, key=len)
    timed = block[-steps * per:] if len(block) >= steps * per else block
    tot = sum(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"]) for i in timed)
    return tot / 1e3 / (len(timed) / per), len(timed)


def main():
    root = sys.argv[1]
    md = "--md" in sys.argv
    out = []
    for cfg in sorted(os.listdir(root)):
        d = os.path.join(root, cfg)
        bj = os.path.join(d, "bench.json")
        tr = os.path.join(d, "run_kernel_trace.csv")
        if not (os.path.exists(bj) and os.path.exists(tr)):
            continue
        line = load_line(bj)
        if line is None:
            continue
        n = line["config"]["keys_per_gpu"]
        bpk = line["config"]["bytes_per_key"]
        ev_ms = line["roofline"]["event_ms_per_step"]
        kus, nk = step_kernel_us(cfg, tr, line)
        frac_tr = bpk * n / (kus * 1e-6) / 1e9 / 8000.0
        row = {"cfg": cfg, "Gkeys_s": line["value"], "frac_event": line["roofline"]["frac"],
               "event_ms_per_step": ev_ms, "trace_ms_per_step": round(kus / 1e3, 4), "trace_dispatches": nk,
               "frac_trace": round(frac_tr, 4), "event_over_trace": round(ev_ms / (kus / 1e3), 4),
               "read_only_GBps": line["roofline"].get("read_only_GBps"), "kernel": line["config"]["kernel"],
               "parity": line["parity"].split(":")[0], "traffic": line["roofline"].get("traffic"),
               "cpu": (line.get("cpu_baseline") or {}).get("value")}
        out.append(row)
    if md:
        print("| cfg | kernel | Gkeys/s | frac (event) | frac (trace, same run) | event / trace | parity | CPU ref Gkeys/s |")
        print("|---|---|---|---|---|---|---|---|")
        for r in out:
            print(f"| {r['cfg']} | `{r['kernel']}` | {r['Gkeys_s']} | {r['frac_event']} | {r['frac_trace']} | "
                  f"{r['event_over_trace']} | {r['parity']} | {r['cpu']} |")
    else:
        for r in out:
            print(json.dumps(r))


if __name__ == "__main__":
    main()
