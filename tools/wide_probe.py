#!/usr/bin/env python3
"""A matrix whose first panels are sparse (a run of empty rows at the top, 20 % empty rows
elsewhere, 6M x 6M, ~77M nnz, fp64): the sweep plan with the wide chunks in the delta side table
(product library, format bit 12) against the unpacked 14-byte sweep this matrix used to fall
back to (tools library, SPMV_SWEEP_PACKED=0). Plans timed in interleaved rounds with HIP events
(spmv_plan_get_timing), y compared. One JSON line per plan. Measurement tool, not product code."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import torch  # noqa: E402

import spmv_hw  # noqa: E402


def main():
    rng = np.random.default_rng(21)
    n = 6_000_000
    lens = rng.poisson(16, n)
    lens[rng.random(n) < 0.2] = 0
    lens[1000:50_000] = 0
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    z = int(rp[-1])
    col = rng.integers(0, n, z, dtype=np.uint32)
    val = rng.uniform(-1, 1, z)
    x = rng.uniform(0, 1, n)
    dev = lambda a: torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).cuda()  # noqa: E731
    d_rp, d_col, d_val, d_x = dev(rp.astype(np.uint32)), dev(col), dev(val), dev(x)
    os.environ["SPMV_HW_KERNEL"] = "sweep"
    plans = {"wide_delta": spmv_hw.Plan.from_device(spmv_hw.load(np.float64), d_rp, d_col, d_val, n)}
    os.environ["SPMV_SWEEP_PACKED"] = "0"
    plans["unpacked"] = spmv_hw.Plan.from_device(spmv_hw.load(np.float64, ablations=True), d_rp, d_col, d_val, n)
    ys = {k: torch.empty(n, dtype=torch.float64, device="cuda") for k in plans}
    times = {k: [] for k in plans}
    for _ in range(5):
        for k, p in plans.items():
            for _ in range(3):
                p.run(d_x, ys[k])
            torch.cuda.synchronize()
            p.set_timing(True)
            for _ in range(20):
                p.run(d_x, ys[k])
            torch.cuda.synchronize()
            times[k].append(p.timing()[0])
            p.set_timing(False)
    ref = ys["unpacked"].double()
    for k, p in plans.items():
        st = p.stats()
        diff = float(((ys[k] - ref).abs().max() / ref.abs().max()).item())
        print(json.dumps({"plan": k, "rows": n, "nnz": z, "format": st["format"], "device_bytes": st["device_bytes"],
                          "kernel_ms_median": round(float(np.median(times[k])), 5), "rounds": times[k],
                          "max_rel_diff_vs_unpacked": diff}), flush=True)
        p.destroy()


if __name__ == "__main__":
    main()
