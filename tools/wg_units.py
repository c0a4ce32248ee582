#!/usr/bin/env python3
"""Per-unit sweep times of the 10M/160M plan over several launches (measurement build): are the
slow units the same panels every launch (a property of the panel: rows, longest row) or the
same CUs (a property of the hardware)? Prints one JSON line: per launch the Pearson correlation of
unit times with launch 0, the share of units on the same CU (HW_ID) as in launch 0, and the
per-unit mean times. Measurement tool, not product code."""
import ctypes
import json
import os
import sys

import numpy as np

os.environ["SPMV_HW_ABLATIONS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import torch  # noqa: E402

import spmv_hw  # noqa: E402


def main():
    lib = spmv_hw.load(np.float64)
    n, z = 10_000_000, 160_000_000
    os.environ["SPMV_HW_KERNEL"] = "sweep"
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    U = plan.stats()["nr_tiles"]
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    times, hw = [], []
    for it in range(8):
        plan.run(x, y)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4 * U))()
        lib.L.spmv_abl_wg_times(buf, ctypes.c_uint(4 * U))
        a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).copy()
        if it >= 2:
            times.append((a[:, 1].astype(np.int64) - a[:, 0].astype(np.int64)) / 100.0)
            hw.append(a[:, 3])
    T = np.array(times)
    mean = T.mean(axis=0)
    out = {"units": U, "launches": len(T), "mean_us": round(float(mean.mean()), 2), "spread_us": round(float(mean.max() - mean.min()), 2),
           "corr_with_launch0": [round(float(np.corrcoef(T[0], T[k])[0, 1]), 3) for k in range(len(T))],
           "same_hw_id_as_launch0": [float((hw[0] == hw[k]).mean()) for k in range(len(hw))],
           "round1_vs_round2_corr": round(float(np.corrcoef(mean[:U // 2], mean[U // 2:])[0, 1]), 3) if U % 2 == 0 else None,
           "per_unit_mean_us": [round(float(v), 1) for v in mean]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
