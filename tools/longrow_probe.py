#!/usr/bin/env python3
"""Measures the "long rows in their own dense panels" lever on the headline matrix
(the reference's answer to x locality is its 2-D column
blocking, csr_hw.cpp:25-27,64-76).

The sweep's x-line requests per non-zero fall with the entries a panel holds per x line. Panels
are nnz-balanced, so every panel of the power-law matrix has the same density (~0.79 lines per
entry). Rows sorted by length would put the longest rows into panels of 20,447 rows with far more
entries; the sweep then cuts such panels into column pieces (the split-panel path). This probe
builds that split without a new kernel: the top q of rows by length become one matrix (its 20,447-
row panels are dense and get cut into pieces by the automatic plan), the other rows a second
one, and both plans are timed beside the plan of the whole matrix (interleaved rounds, HIP
events). 1 - (T_long + T_short) / T_all is the gain of the split run as two launches: it leaves
out the cost of writing the long rows' y to scattered rows (optimistic) and pays a second
launch's ramp and tail (pessimistic by at most one tail, a few us). Prints one JSON line per
threshold."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import torch  # noqa: E402

import spmv_hw  # noqa: E402


def sub_csr(rp, col, val, rows_mask):
    """CSR of the rows where rows_mask is set (in their original order)."""
    lens = (rp[1:] - rp[:-1]).long()
    ent_mask = torch.repeat_interleave(rows_mask, lens)
    sl = lens[rows_mask]
    srp = torch.zeros(sl.numel() + 1, dtype=torch.int64, device=rp.device)
    srp[1:] = torch.cumsum(sl, 0)
    return srp.int(), col[ent_mask].contiguous(), val[ent_mask].contiguous(), int(sl.numel())


def time_plan(plan, x, y, reps):
    plan.set_timing(True)
    for _ in range(reps):
        plan.run(x, y)
    ms, _, _ = plan.timing()
    plan.set_timing(False)
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--nnz", type=int, default=160_000_000)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--top", default="0.01,0.05,0.1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dtype = np.float64 if a.dtype == "f64" else np.float32
    lib = spmv_hw.load(dtype)
    os.environ["SPMV_HW_KERNEL"] = "sweep"
    n = a.rows
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, a.nnz, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    y = torch.empty(n, dtype=x.dtype, device="cuda")
    whole = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    lens = (rp[1:] - rp[:-1]).long()
    for q in [float(t) for t in a.top.split(",")]:
        k = max(1, int(q * n))
        thr = torch.topk(lens, k).values.min()
        long_mask = lens >= thr
        lrp, lcol, lval, nl = sub_csr(rp, col, val, long_mask)
        srp, scol, sval, ns = sub_csr(rp, col, val, ~long_mask)
        pl = spmv_hw.Plan.from_device(lib, lrp, lcol, lval, n)
        ps = spmv_hw.Plan.from_device(lib, srp, scol, sval, n)
        yl = torch.empty(nl, dtype=x.dtype, device="cuda")
        ys = torch.empty(ns, dtype=x.dtype, device="cuda")
        # the split must reproduce the whole matrix's y (checked on the long/short rows)
        whole.run(x, y)
        pl.run(x, yl)
        ps.run(x, ys)
        torch.cuda.synchronize()
        scale = y.abs().max().clamp_min(1e-300)
        err = max(float(((y[long_mask] - yl).abs().max() / scale).item()),
                  float(((y[~long_mask] - ys).abs().max() / scale).item()))
        t = {"all": [], "long": [], "short": []}
        for _ in range(a.rounds):
            t["all"].append(time_plan(whole, x, y, a.reps))
            t["long"].append(time_plan(pl, x, yl, a.reps))
            t["short"].append(time_plan(ps, x, ys, a.reps))
        med = {kk: float(np.median(v)) for kk, v in t.items()}
        stl, sts = pl.stats(), ps.stats()
        out = {"dtype": a.dtype, "rows": n, "nnz": a.nnz, "top_frac": q, "min_len_long": int(thr.item()),
               "long_rows": nl, "long_nnz": stl["nr_nzeros"], "long_units": stl["nr_tiles"],
               "short_units": sts["nr_tiles"], "max_rel_diff": err,
               "ms_all": round(med["all"], 5), "ms_long": round(med["long"], 5), "ms_short": round(med["short"], 5),
               "ms_split_sum": round(med["long"] + med["short"], 5),
               "gain_two_launches": round(1.0 - (med["long"] + med["short"]) / med["all"], 4)}
        print(json.dumps(out), flush=True)
        pl.destroy()
        ps.destroy()
        del lrp, lcol, lval, srp, scol, sval, yl, ys
        torch.cuda.empty_cache()
    whole.destroy()


if __name__ == "__main__":
    main()
