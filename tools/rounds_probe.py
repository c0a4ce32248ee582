#!/usr/bin/env python3
"""The drop-in's streamed copy-back against the number of rounds of panels the sweep runs: one
create_csr_hw_matrix of the 10M/160M fp64 matrix per setting of the tools build's
SPMV_SWEEP_ROUNDS (0 = the plan's own two rounds of full-LDS panels; k = at least k rounds of
smaller panels, so the first panels -- and the first copies -- finish earlier while the kernel
itself slows on the thinner x reuse), then interleaved rounds of spmv_hw calls on each; the
library's printed Hardware / Total times are captured. One JSON line per setting (medians).
Measurement tool, not product code."""
import argparse
import ctypes
import json
import os
import re
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import dropin_main  # noqa: E402
import spmv_hw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds-list", default="0,3,4,6,8")
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--pieces", default="", help="tools SPMV_HW_PIECES for every call (default: 8)")
    a = ap.parse_args()
    os.environ["SPMV_HW_MERGE"] = "host"
    if a.pieces:
        os.environ["SPMV_HW_PIECES"] = a.pieces
    lib = spmv_hw.load(np.float64, ablations=True)
    args = dropin_main.parse(["--ref", "unused"])
    h_rp, h_col, h_val, h_x = dropin_main.host_matrix(lib, args)
    n = len(h_rp) - 1
    flows = {}
    for r in [int(v) for v in a.rounds_list.split(",")]:
        os.environ["SPMV_SWEEP_ROUNDS"] = str(r)
        hw, bm = lib.create_csr_hw_matrix(lib.make_csr_matrix(h_rp, h_col, h_val, n))
        hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(h_x), hw[0].contents.blocks, hw[0].contents.nr_cols)
        yv = lib.make_csr_vector(np.zeros(n))
        flows[r] = (hw, bm, hx, yv)
    os.environ.pop("SPMV_SWEEP_ROUNDS", None)
    libc = ctypes.CDLL(None)
    res = {r: {"hw": [], "tot": []} for r in flows}
    saved = os.dup(1)
    with tempfile.TemporaryFile(mode="w+") as f:
        for _ in range(a.iters):
            for r, (hw, bm, hx, yv) in flows.items():
                sys.stdout.flush()
                os.dup2(f.fileno(), 1)
                for _ in range(a.calls):
                    lib.spmv_hw(hw, hx, yv, bm)
                libc.fflush(None)
                os.dup2(saved, 1)
                f.seek(0)
                txt = f.read()
                f.seek(0)
                f.truncate()
                res[r]["hw"] += [float(v) for v in re.findall(r"Hardware execution time\s*:\s*([0-9.]+)", txt)]
                res[r]["tot"] += [float(v) for v in re.findall(r"Total time\s*:\s*([0-9.]+)", txt)]
    ref = None
    for r, (hw, bm, hx, yv) in flows.items():
        y = np.ctypeslib.as_array(yv.values, shape=(n,)).copy()
        calls = len(res[r]["tot"])
        y1 = y / calls  # every call added A x once
        if ref is None:
            ref = y1
        diff = float(np.abs(y1 - ref).max() / np.abs(ref).max())
        print(json.dumps({"rounds": r, "calls": calls,
                          "hardware_ms_median": round(float(np.median(res[r]["hw"])), 4),
                          "total_ms_median": round(float(np.median(res[r]["tot"])), 4),
                          "total_ms_min": min(res[r]["tot"]), "max_rel_diff_vs_first": diff}), flush=True)
        lib.delete_csr_hw_matrix(hw)
        lib.free_bitmap(bm)
        lib.delete_csr_hw_x_vector(hx)


if __name__ == "__main__":
    main()
