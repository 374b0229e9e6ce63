#!/usr/bin/env python3
"""Measurement table from same-run files: for every config, the bench line
(bench.json) and the rocprofv3 kernel trace of THAT run (run_kernel_trace.csv,
tools/gpu_session.sh hyg_<cfg>).  For each config it prints

  * the bench line's own figures: Gkeys/s, roofline frac (algorithmic bytes
    over the HIP-event time per step), read-only GB/s;
  * the same frac recomputed from the trace: algorithmic bytes per step over
    the summed kernel time per step of the step's launches -- the step
    kernels' dispatches of the K timed steps (the first K x launches-per-step
    of them after the bench's Infinity-Cache flush; warm-up, calibration and
    parity launches excluded), and the first-start-to-last-end span of those
    dispatches per step (kernel time plus the gaps between launches);
  * their ratio, so a reader can check that the event timing and the kernel
    durations agree.

  python tools/hyg_summary.py profiles/r06/hyg [--md]
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
    "exchange": ["k_bucket_count_reg", "k_bucket_colscan", "k_bucket_chunkscan", "k_bucket_base",
                 "k_bucket_scatter"],
    "xrecords": ["k_bucket_count_reg", "k_bucket_colscan", "k_bucket_chunkscan", "k_bucket_base",
                 "k_bucket_scatter"],
    # (late r05: the two-pass count kernel scans its fine counts itself, no colscan launch)
    "bucket8k": ["k_bucket_count_tp", "k_bucket_chunkscan2", "k_bucket_base", "k_bucket_pass1",
                 "k_bucket_pass2"],
    # r06: the tile-local two passes (pass 2 forms the bucket bases: no k_bucket_base)
    "bucket8k_tl": ["k_bucket_tl_pass1", "k_bucket_chunkscan_tl", "k_bucket_tl_pass2"],
}


def load_line(path):
    for ln in open(path):
        if ln.startswith("{"):
            return json.loads(ln)
    return None


LAUNCH_BYTES = 512 << 20  # launch.h kLaunchBytes


def launches_per_step(line):
    """Launches of the hash kernel per bench step (launch.h: fixed keys in
    ~512-MiB launches of whole 4096-key blocks, k_global batches in one,
    variable keys by the batch's mean key length)."""
    c = line["config"]
    n, kern = c["keys_per_gpu"], c["kernel"]
    if kern.startswith("k_global"):
        return 1
    if kern.startswith("k_window<var"):
        mean = max(1, int(c["bytes_per_key"] - 16))
        if n * mean <= LAUNCH_BYTES:
            return 1
        step = max(4096, (LAUNCH_BYTES // mean) & ~4095)
        return -(-n // step)
    L = c["key_bytes"]
    per = max(1, LAUNCH_BYTES // L)
    if n <= per:
        return 1
    step = (per + 4095) & ~4095
    return -(-n // step)


def step_kernel_us(cfg, trace, line):
    """Mean kernel microseconds per timed step, from the trace: the timed
    steps are the first K x launches-per-step dispatches of the step's
    kernels after the Infinity-Cache flush (bench.py flush_infinity_cache,
    a 512-MiB torch fill) that follows the warm-up."""
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    steps = line["steps"]
    if cfg in STEP_KERNELS:
        pats = STEP_KERNELS[cfg + "_tl" if line["config"]["kernel"].startswith("k_bucket_tl") else cfg]
        is_step = lambda nm: any(p in nm for p in pats)  # noqa: E731
        per = len(pats)
    else:
        head = line["config"]["kernel"].split("<")[0]
        is_step = lambda nm: head in nm  # noqa: E731
        per = launches_per_step(line)
    first = next(i for i, r in enumerate(rows) if is_step(r["Kernel_Name"]))
    flush = next(i for i, r in enumerate(rows) if i > first and "vectorized_elementwise_kernel<16" in r["Kernel_Name"])
    timed = [r for r in rows[flush + 1:] if is_step(r["Kernel_Name"])][:steps * per]
    if len(timed) != steps * per:
        raise SystemExit(f"{cfg}: {len(timed)} timed dispatches, want {steps * per}")
    tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed)
    span = int(timed[-1]["End_Timestamp"]) - int(timed[0]["Start_Timestamp"])
    return tot / 1e3 / steps, len(timed), span / 1e3 / steps


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
        kus, nk, span_us = step_kernel_us(cfg, tr, line)
        frac_tr = bpk * n / (kus * 1e-6) / 1e9 / 8000.0
        row = {"cfg": cfg, "Gkeys_s": line["value"], "frac_event": line["roofline"]["frac"],
               "event_ms_per_step": ev_ms, "trace_ms_per_step": round(kus / 1e3, 4), "trace_dispatches": nk,
               "trace_span_ms_per_step": round(span_us / 1e3, 4),
               "frac_trace": round(frac_tr, 4), "event_over_trace": round(ev_ms / (kus / 1e3), 4),
               "read_only_GBps": line["roofline"].get("read_only_GBps"), "kernel": line["config"]["kernel"],
               "parity": line["parity"].split(":")[0], "traffic": line["roofline"].get("traffic"),
               "cpu": (line.get("cpu_baseline") or {}).get("value")}
        out.append(row)
    if md:
        print("| config | kernel (tag) | Gkeys/s | frac, HIP events | frac, rocprof trace of the same run | "
              "read-only frac | parity | CPU reference Gkeys/s |")
        print("|---|---|---|---|---|---|---|---|")
        for r in out:
            ro = round(r["read_only_GBps"] / 8000.0, 4) if r["read_only_GBps"] else None
            print(f"| {r['cfg']} | `{r['kernel']}` | {r['Gkeys_s']} | {r['frac_event']} | {r['frac_trace']} | "
                  f"{ro} | {r['parity']} | {r['cpu']} |")
    else:
        for r in out:
            print(json.dumps(r))


if __name__ == "__main__":
    main()
