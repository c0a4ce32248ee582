#!/usr/bin/env python3
"""HBM traffic per SpMV of the two binned passes (k_bin_mul + k_bin_acc) from rocprofv3 --pmc
runs, one counter per pass (tools/gpu_session.sh step `pmcbin`): <root>/pmcbin_<dtype>_<COUNTER>/
run_counter_collection.csv. hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch (the
gfx950 correction of MI355X_MICROARCH.md §HBM, as tools/pmc_traffic.py). Output: the structure
bench.py reads for side_configs.config5.roofline.traffic ({"f32": {"hbm_bytes_per_spmv": ...}})."""
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
    ap.add_argument("--out", required=True)
    ap.add_argument("--session", default="")
    a = ap.parse_args()
    res = {}
    for d in sorted(glob.glob(os.path.join(a.root, "pmcbin_*_*"))):
        m = re.match(r"pmcbin_(f32|f64)_(\w+)$", os.path.basename(d))
        if not m or not os.path.isdir(d):
            continue
        dt, counter = m.groups()
        vals = {}
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            for k in ("k_bin_mul", "k_bin_acc"):
                if k in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    vals.setdefault(k, []).append(float(r["Counter_Value"]))
        for k, v in vals.items():
            res.setdefault(dt, {}).setdefault(k, {})[counter] = statistics.mean(v)
    for dt, e in res.items():
        total = 0
        for k in ("k_bin_mul", "k_bin_acc"):
            c = e.get(k, {})
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                c["hbm_bytes"] = int((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
                total += c["hbm_bytes"]
        e["hbm_bytes_per_spmv"] = total
        e["design_bytes"] = 160_000_000 * (15 if dt == "f32" else 27)
    res["_note"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per pass, bench.py --dtype <dt> on the "
                    "10M x 10M / 160M power-law matrix (kernel 6 forced for f64), session " + a.session +
                    "; hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch (MI355X_MICROARCH.md gfx950 "
                    "correction); design_bytes = 15 (fp32) / 27 (fp64) B per non-zero streamed by the two passes")
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_spmv") for k, v in res.items() if k != "_note"}))


if __name__ == "__main__":
    main()
