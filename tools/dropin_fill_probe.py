#!/usr/bin/env python3
"""Does the caller's zeroing of y_fpga right before spmv_hw (what spmv-fpga_amd/dropin_main.py
does per call, main.cpp:74's fresh vector) cost the streamed copy-back's adds? The drop-in flow on
the 10M/160M matrix, spmv_hw timed by its own printed Total under three caller forms, interleaved:
zero y with numpy right before the call, zero it and then evict it from the caches (a 512 MB
sweep), or do not zero it (y accumulates). One JSON line per form. Measurement tool, not product
code."""
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
    os.environ["SPMV_HW_MERGE"] = "host"
    args = dropin_main.parse(["--ref", "unused"])
    lib = spmv_hw.load(np.float64)
    h_rp, h_col, h_val, h_x = dropin_main.host_matrix(lib, args)
    n = len(h_rp) - 1
    hw, bm = lib.create_csr_hw_matrix(lib.make_csr_matrix(h_rp, h_col, h_val, n))
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(h_x), hw[0].contents.blocks, hw[0].contents.nr_cols)
    yv = lib.make_csr_vector(np.zeros(n))
    y = np.ctypeslib.as_array(yv.values, shape=(n,))
    junk = np.ones(64 << 20)  # 512 MB
    libc = ctypes.CDLL(None)
    forms = {"zero_then_call": lambda: y.fill(0), "zero_evict_then_call": lambda: (y.fill(0), junk.sum()),
             "no_zero": lambda: None}
    tot = {k: [] for k in forms}
    saved = os.dup(1)
    with tempfile.TemporaryFile(mode="w+") as f:
        for _ in range(8):
            for k, prep in forms.items():
                for _ in range(3):
                    prep()
                    sys.stdout.flush()
                    os.dup2(f.fileno(), 1)
                    lib.spmv_hw(hw, hx, yv, bm)
                    libc.fflush(None)
                    os.dup2(saved, 1)
                    f.seek(0)
                    t = [float(v) for v in re.findall(r"Total time\s*:\s*([0-9.]+)", f.read())]
                    f.seek(0)
                    f.truncate()
                    tot[k].append(t[-1])
    for k, v in tot.items():
        print(json.dumps({"form": k, "calls": len(v), "total_ms_median": round(float(np.median(v)), 4),
                          "total_ms_min": min(v)}), flush=True)
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)


if __name__ == "__main__":
    main()
