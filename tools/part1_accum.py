"""Part 1 (`spmv_hw`) timing probe: the reference's three timing lines for a fresh,
calloc-backed y_fpga (first touch of its pages inside the accumulation, as in main.cpp:74)
and for a reused one. Banded matrix, `--rows` rows x 16, fp64; `--units` sets SPMV_NGPUS.
Run with SPMV_HW_TRACE=1 for the per-phase breakdown on stderr."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spmv-fpga_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--units", type=int, default=1)
    ap.add_argument("--calls", type=int, default=3)
    a = ap.parse_args()
    os.environ["SPMV_NGPUS"] = str(a.units)
    import spmv_hw
    lib = spmv_hw.load(np.float64)
    n, w = a.rows, 16
    rp = (np.arange(n + 1, dtype=np.int64) * w).astype(np.uint32)
    start = np.clip(np.arange(n) - w // 2, 0, n - w)
    col = (start[:, None] + np.arange(w)[None, :]).ravel().astype(np.uint32)
    val = np.random.default_rng(1).uniform(-1, 1, n * w)
    x = np.random.default_rng(2).uniform(0, 1, n)
    m = lib.make_csr_matrix(rp, col, val, n)
    hw, bm = lib.create_csr_hw_matrix(m)
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), hw[0].contents.blocks, hw[0].contents.nr_cols)
    ref = None
    for c in range(a.calls):
        y = lib.make_csr_vector(np.zeros(n))  # numpy zeros: calloc, pages untouched
        print(f"-- call {c}: fresh y_fpga", flush=True)
        lib.spmv_hw(hw, hx, y, bm)
        out = np.ctypeslib.as_array(y.values, (n,)).copy()
        if ref is None:
            ref = out
        assert np.array_equal(out, ref)
    print("-- reused y_fpga (second call adds: 2y)", flush=True)
    lib.spmv_hw(hw, hx, y, bm)
    out = np.ctypeslib.as_array(y.values, (n,))
    assert np.array_equal(out, 2 * ref)
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)
    print("ok", flush=True)


if __name__ == "__main__":
    main()
