#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs into HBM traffic per launch of the SpMV kernels.

Input: directories <root>/pmc_<workload>_<dtype>_<COUNTER>/run_counter_collection.csv produced by
tools/gpu_session.sh step `pmcw` (one counter per pass: FETCH_SIZE and WRITE_SIZE cannot share a
pass on gfx950, MI355X_MICROARCH.md §rocprofv3 PMC slots).

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE counts a wide coalesced streaming
read at exactly half its bytes (TCC_EA0_RDREQ x 64 B for 128-B requests), so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024      [FETCH_SIZE, WRITE_SIZE in KiB]
The doubling is exact for the dwordx4 entry streams; for the 8-byte x gathers that miss L2 it
can over-count (their request size is not calibrated), so the value is an upper bound for
gather-heavy kernels. Raw counter means are kept next to it.

Output: JSON {"<workload>_<dtype>": {"kernel", "nnz", "hbm_bytes_per_launch", ...}} on stdout
or into --out (bench.py reads profiles/traffic.json).
"""
import argparse
import csv
import glob
import json
import os
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=None)
    ap.add_argument("--nnz", type=json.loads, default='{"powerlaw": 160000000, "banded": 16000000}')
    a = ap.parse_args()
    res = {}
    for d in sorted(glob.glob(os.path.join(a.root, "pmc_*_*_*"))):
        if not os.path.isdir(d):
            continue
        m = re.match(r"pmc_(\w+?)_(f64|f32)_(\w+)$", os.path.basename(d))
        if not m:
            continue
        wl, dt, counter = m.groups()
        rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
        per_kernel = {}
        for r in rows:
            name = r["Kernel_Name"]
            if not any(k in name for k in ("k_spmv_tiles", "k_spmv_sweep", "k_spmv_slices", "k_fixup")):
                continue
            short = re.sub(r"\(.*", "", name).replace("void spmvhw::", "")
            per_kernel.setdefault((short, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
        entry = res.setdefault(f"{wl}_{dt}", {"nnz": a.nnz.get(wl)})
        for (k, c), vals in per_kernel.items():
            entry.setdefault("counters", {}).setdefault(k, {})[c] = statistics.mean(vals)
    for key, e in res.items():
        main_k = [k for k in e.get("counters", {}) if "fixup" not in k]
        if not main_k:
            continue
        k = main_k[0]
        c = e["counters"][k]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["kernel"] = k
            e["hbm_bytes_per_launch"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
            e["correction"] = "(2*FETCH_SIZE + WRITE_SIZE)*1024, MI355X_MICROARCH.md §HBM"
    text = json.dumps(res, indent=1, sort_keys=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
