#!/usr/bin/env python3
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, as
MI355X_MICROARCH.md §rocprofv3 requires) into HBM bytes per hash-kernel launch.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts exactly half
the bytes of a wide coalesced streaming read (16 B per lane, global_load and
LDS-DMA alike) -> x2.  WRITE_SIZE is exact for streaming stores.  Both are in
KiB.

  python tools/pmc_traffic.py --cfg cfg2 --keys 16777216 --kernel k_fixed_xpose64 \
      --algo-bytes-per-key 72 --fetch-dir gpurun_out/pmc_cfg2_1 --write-dir gpurun_out/pmc_cfg2_2 \
      --bench-log gpurun_out/pmc_cfg2_1.log --out profiles/traffic_cfg2.json
  (--kernel "a|b|c" sums several kernels of one step, e.g. the bucketing launches)
The kernel tag of the run (pdht_hip_last_kernel, from the bench line in
--bench-log) and the full rocprof kernel symbols are stored: bench.py uses
the figure only when the tag of ITS kernel is the same.
"""
import argparse
import csv
import json
import os
import statistics


def per_launch(path, kernel, counter, per_step=1):
    """Median counter value per launch; with per_step > 1 (a step is several
    launches of the kernel, e.g. 512-MiB chunks) the mean per STEP: the sum
    over every profiled launch x per_step / launches (every profiled call of
    the kernel is a whole step)."""
    rows = [r for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not rows:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    names = sorted({r["Kernel_Name"] for r in rows})
    if len(names) != 1:
        raise SystemExit(f"{kernel} matches several kernels in {path}: {names}")
    # rocprofv3 may split one dispatch's counter over several rows (dimensions)
    disp = {}
    for j, r in enumerate(rows):
        d = r.get("Dispatch_Id", j)
        disp[d] = disp.get(d, 0.0) + float(r["Counter_Value"])
    vals = list(disp.values())
    if per_step > 1:
        if len(vals) % per_step:
            raise SystemExit(f"{len(vals)} launches of {kernel} are not whole steps of {per_step}")
        return sum(vals) * per_step / len(vals), len(vals), names[0]
    return statistics.median(vals), len(vals), names[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", required=True)
    ap.add_argument("--keys", type=int, required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--algo-bytes-per-key", type=float, required=True)
    ap.add_argument("--launches-per-step", type=int, default=1,
                    help="launches of --kernel per bench step (batches split into ~512-MiB launches)")
    ap.add_argument("--dir", default="gpurun_out")
    ap.add_argument("--out", required=True)
    ap.add_argument("--fetch-dir", default=None, help="default: <dir>/pmc_FETCH_SIZE")
    ap.add_argument("--write-dir", default=None, help="default: <dir>/pmc_WRITE_SIZE")
    ap.add_argument("--bench-log", required=True, help="bench.py output of the profiled run (kernel tag)")
    a = ap.parse_args()
    fd = a.fetch_dir or os.path.join(a.dir, "pmc_FETCH_SIZE")
    wd = a.write_dir or os.path.join(a.dir, "pmc_WRITE_SIZE")
    # --kernel "a|b|c": the step launches several kernels; sum their medians
    f_kib = w_kib = 0.0
    nf = nw = 0
    symbols = []
    for k in a.kernel.split("|"):
        f, nf, name = per_launch(os.path.join(fd, "run_counter_collection.csv"), k, "FETCH_SIZE",
                                 a.launches_per_step)
        w, nw, name2 = per_launch(os.path.join(wd, "run_counter_collection.csv"), k, "WRITE_SIZE",
                                  a.launches_per_step)
        if name != name2:
            raise SystemExit(f"FETCH and WRITE passes profiled different kernels: {name} / {name2}")
        symbols.append(name)
        f_kib += f
        w_kib += w
    line = [ln for ln in open(a.bench_log) if ln.startswith("{")][-1]
    tag = json.loads(line)["config"]["kernel"]
    fetch = f_kib * 1024 * 2  # gfx950: FETCH_SIZE = half of a wide streaming read
    write = w_kib * 1024
    algo = a.algo_bytes_per_key * a.keys
    res = {"cfg": a.cfg, "kernel": a.kernel, "kernel_tag": tag, "rocprof_kernels": symbols,
           "keys_per_launch": a.keys,  # keys per bench step (one or more launches)
           "launches_per_step": a.launches_per_step,
           "fetch_size_kib_raw": f_kib, "fetch_correction": 2, "write_size_kib_raw": w_kib,
           "launches_sampled": [nf, nw],
           "hbm_bytes_per_launch": int(fetch + write),
           "algorithmic_bytes_per_launch": int(algo),
           "traffic_over_algorithmic": round((fetch + write) / algo, 4)}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
