#!/usr/bin/env python3
"""The reference's run.elf flow (euroexa/spmv-fpga src/main.cpp:46-97) through the Part-1 C-ABI of
libspmv_hw (include/csr_hw_wrapper.h), on the bench's synthetic matrix instead of a .mtx file.

    create_csr_hw_matrix + create_csr_hw_x_vector   -> "Matrix read time"        (main.cpp:67-72)
    spmv_hw                                         -> "Hardware execution time", "Result
                                                       accumulation time", "Total time"
                                                       (csr_hw_wrapper.cpp:272-285, printed by
                                                       the library itself)
    verification(y, y_fpga)                         -> "Verification PASSED!"   (main.cpp:77-82)
    storage_overhead per unit                       -> the storage line         (main.cpp:84-88)

bench.py runs it as a child process (so the library's fail-fast exit(1) or a stuck RCCL clique
cannot take the bench line with it) with the software result y -- the oracle's spmv_gold of the
same matrix, computed by the bench -- in a .npy file, as main.cpp computes y before the hardware
path. Units ("ComputeUnits") and the merge form come from the command line (spmv_hw_set_units,
env SPMV_HW_MERGE): at N > 1 the bench asks for N units, one per GPU, merged by the library's RCCL
reduce over xGMI (the north star's mapping of accum_results). spmv_hw is called --reps times, each
into a zeroed y_fpga (it accumulates, csr.cpp:1555), and every call is verified.

stdout: the reference's lines, then one line "DROPIN_JSON {...}" with the per-call results.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=["powerlaw", "banded"], default="powerlaw")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--nnz", type=int, default=160_000_000)
    ap.add_argument("--units", type=int, default=1)
    ap.add_argument("--merge", choices=["host", "gather", "reduce"], default="host")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ref", required=True, help=".npy of the software y (spmv_gold of the same matrix)")
    ap.add_argument("--ab-unstreamed", type=int, default=0,
                    help="then this many more calls with SPMV_HW_STREAM=0 (the copy after the kernel), "
                         "printed after a line DROPIN_AB_UNSTREAMED")
    return ap.parse_args(argv)


def host_matrix(lib, args):
    """The bench's matrix (bench.py build_workload, rank 0 / the whole matrix) and x, in host memory."""
    import torch
    import spmv_hw
    n = args.rows
    if args.workload == "banded":
        rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
        x = spmv_hw.gen_vector(lib, n, seed=3)
    else:
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, args.nnz, seed=4)
        x = spmv_hw.gen_vector(lib, n, seed=6)
    h = (rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32), val.cpu().numpy(), x.cpu().numpy())
    del rp, col, val, x
    torch.cuda.empty_cache()
    return h


def _die_with_parent():
    """This process is SIGKILLed when the bench rank that started it dies (Linux prctl
    PR_SET_PDEATHSIG, set from here: the rank has threads, so no preexec hook there), so a rank
    killed at a deadline leaves no drop-in run holding the node's GPUs."""
    parent = os.getppid()
    try:
        import signal
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGKILL, 0, 0, 0)
    except Exception:
        return
    if os.getppid() != parent:  # the parent was already gone
        os._exit(1)


def main(argv=None):
    _die_with_parent()
    args = parse(argv)
    os.environ["SPMV_HW_MERGE"] = args.merge  # read by create_csr_hw_matrix
    import spmv_hw
    dtype = np.float64 if args.dtype == "f64" else np.float32
    lib = spmv_hw.load(dtype)
    libc = ctypes.CDLL(None)
    h_rp, h_col, h_val, h_x = host_matrix(lib, args)
    n = len(h_rp) - 1
    y_sw = np.load(args.ref, allow_pickle=False)
    if y_sw.shape != (n,) or y_sw.dtype != dtype:
        raise SystemExit(f"--ref holds {y_sw.dtype}{y_sw.shape}, the matrix has {n} rows of {np.dtype(dtype)}")
    lib.set_units(args.units)  # the caller's ComputeUnits
    matrix = lib.make_csr_matrix(h_rp, h_col, h_val, n)
    x = lib.make_csr_vector(h_x)

    def flush():  # the library prints through C stdio; keep its lines in order with ours
        sys.stdout.flush()
        libc.fflush(None)

    mr_s = time.perf_counter()
    hw, bm = lib.create_csr_hw_matrix(matrix)
    hx = lib.create_csr_hw_x_vector(x, hw[0].contents.blocks, hw[0].contents.nr_cols)
    mr_ms = (time.perf_counter() - mr_s) * 1e3
    flush()
    print(f"Matrix read time        : {mr_ms:.6f} ms elapsed", flush=True)

    y_fpga = lib.make_csr_vector(np.zeros(n, dtype))
    y_view = np.ctypeslib.as_array(y_fpga.values, shape=(n,))
    calls = []
    for k in range(max(1, args.reps)):
        y_view.fill(0)  # main.cpp:74 hands spmv_hw a zeroed vector; spmv_hw accumulates
        t0 = time.perf_counter()
        lib.spmv_hw(hw, hx, y_fpga, bm)
        wall_ms = (time.perf_counter() - t0) * 1e3
        flush()
        status = lib.verification(y_sw, y_view, 0)
        print("Verification PASSED!" if status == 0 else "Verification FAILED!", flush=True)
        ref = y_sw.astype(np.float64)
        scale = max(float(np.abs(ref).max()), 1e-300) if n else 1.0
        diff = float(np.abs(y_view.astype(np.float64) - ref).max() / scale) if n else 0.0
        calls.append({"wall_ms": round(wall_ms, 4), "verification": status, "max_rel_diff": diff})

    if args.ab_unstreamed > 0:  # the same calls with the copy-back after the kernel
        os.environ["SPMV_HW_STREAM"] = "0"  # (read per call)
        flush()
        print("DROPIN_AB_UNSTREAMED", flush=True)
        for _ in range(args.ab_unstreamed):
            y_view.fill(0)
            lib.spmv_hw(hw, hx, y_fpga, bm)
            flush()
        os.environ.pop("SPMV_HW_STREAM", None)

    units = lib.units()
    mem = sum(lib.storage_overhead(hw[u]) for u in range(units))
    csr_mem = ((n + 1) * 32 + int(h_rp[-1]) * (32 + 8 * np.dtype(dtype).itemsize)) / (8.0 * 1024 * 1024)
    print(f"CSR representation : {csr_mem:g} MB. Our representation : {mem:g} MB. "
          f"Storage Overhead : {(mem - csr_mem) / csr_mem * 100 if csr_mem else 0.0:g} %", flush=True)
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)
    flush()
    print("DROPIN_JSON " + json.dumps({"units": units, "merge": args.merge, "rows": n, "nnz": int(h_rp[-1]),
                                       "matrix_read_ms": round(mr_ms, 3), "calls": calls,
                                       "storage_mb": round(mem, 3), "csr_mb": round(csr_mem, 3)}), flush=True)
    return 0  # (the caller judges the calls' verification and differences)


if __name__ == "__main__":
    sys.exit(main())
