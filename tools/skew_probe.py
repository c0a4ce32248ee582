#!/usr/bin/env python3
"""Ragged extremes: a matrix whose rows are ~16 long except for a few dense rows (one row of
`--dense` entries every `--every` rows). Times every kernel on it and checks each against the
oracle (scaled error). Prints one JSON line. Usage: skew_probe.py [--rows N] [--dense L]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spmv-fpga_amd"), os.path.join(ROOT, "oracle")]
import torch  # noqa: E402

import oracle  # noqa: E402
import spmv_hw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--cols", type=int, default=2_000_000)
    ap.add_argument("--dense", type=int, default=2_000_000)
    ap.add_argument("--ndense", type=int, default=2)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--kernels", default="tiles,sweep,gold")
    a = ap.parse_args()
    dtype = np.float64 if a.dtype == "f64" else np.float32
    rng = np.random.default_rng(5)
    n, m = a.rows, a.cols
    lens = rng.poisson(16, n).astype(np.int64)
    dense_rows = rng.choice(n, a.ndense, replace=False)
    lens[dense_rows] = a.dense
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    z = int(rp[-1])
    col = np.empty(z, np.uint32)
    for r in range(n):  # sorted unique columns per row
        k = int(lens[r])
        if k == 0:
            continue
        if k > m // 4:
            c = np.sort(rng.choice(m, k, replace=False))
        else:
            c = np.unique(rng.integers(0, m, k))
            while len(c) < k:
                c = np.unique(np.concatenate([c, rng.integers(0, m, k - len(c))]))
        col[rp[r]:rp[r + 1]] = c
    val = rng.uniform(-1, 1, z).astype(dtype)
    x = rng.uniform(0, 1, m).astype(dtype)
    rp = rp.astype(np.uint32)
    ref = oracle.spmv_gold(rp, col, val, x)
    lib = spmv_hw.load(dtype)
    d = lambda t: torch.from_numpy(t.view(np.int32) if t.dtype == np.uint32 else t).cuda()
    drp, dcol, dval, dx = d(rp), d(col), d(val), d(x)
    out = {"rows": n, "cols": m, "nnz": z, "dense_rows": a.ndense, "dense_len": a.dense, "dtype": a.dtype}
    for kern in a.kernels.split(","):
        os.environ["SPMV_HW_KERNEL"] = kern  # "auto": the automatic choice
        plan = spmv_hw.Plan.from_device(lib, drp, dcol, dval, m)
        y = torch.empty(n, dtype=dx.dtype, device="cuda")
        plan.run(dx, y)
        torch.cuda.synchronize()
        err = oracle.scaled_error(rp, col, val, x, ref, y.cpu().numpy())
        plan.set_timing(True)
        for _ in range(a.reps):
            plan.run(dx, y)
        ms, _, _ = plan.timing()
        st = plan.stats()
        out[kern] = {"ms": round(ms, 4), "scaled_err": err, "units": st["nr_tiles"], "kernel": st["kernel"]}
        plan.destroy()
    os.environ.pop("SPMV_HW_KERNEL", None)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
