#!/usr/bin/env python3
"""Interleaved A/B timing of kernel variants on one plan, in one process (methodology rule 24 of
cdna_hip_programming.md §5.4): N variants x M rounds, median and min of the main kernel's HIP-event
duration. Prints one JSON line per workload."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import torch  # noqa: E402

import spmv_hw  # noqa: E402


def stencil(rows, points, dtype):
    """3-D Laplacian-shaped matrix on a g^3 grid (g = rows^(1/3)): 7- or 27-point
    neighbourhoods, columns sorted within rows, random values. Local columns, but the first two
    columns of a row lie a grid plane apart."""
    g = int(round(rows ** (1 / 3)))
    n = g ** 3
    idx = np.arange(n, dtype=np.int64)
    z, y, xx = idx // (g * g), (idx // g) % g, idx % g
    offs = [(dz, dy, dx) for dz in (-1, 0, 1) for dy in (-1, 0, 1) for dx in (-1, 0, 1)
            if points == 27 or abs(dz) + abs(dy) + abs(dx) <= 1]
    cols = np.full((n, len(offs)), -1, np.int64)
    for k, (dz, dy, dx) in enumerate(offs):  # offsets in increasing column order
        ok = (z + dz >= 0) & (z + dz < g) & (y + dy >= 0) & (y + dy < g) & (xx + dx >= 0) & (xx + dx < g)
        cols[ok, k] = idx[ok] + dz * g * g + dy * g + dx
    lens = (cols >= 0).sum(axis=1)
    c = cols[cols >= 0].astype(np.uint32)
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    v = np.random.default_rng(2).uniform(-1, 1, len(c)).astype(dtype)
    t = lambda h: torch.from_numpy(h.view(np.int32) if h.dtype == np.uint32 else h).cuda()
    return t(rp.astype(np.uint32)), t(c), t(v), n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="powerlaw,banded")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--variants", default="tiles:0,tiles:1,sweep:0",
                    help="comma list of kernel:variant (kernel = tiles | sweep)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--nnz", type=int, default=None)
    ap.add_argument("--cols", type=int, default=None, help="power-law: columns (default = rows)")
    a = ap.parse_args()
    # every variant but the default lives in the tools library (spmv-fpga_amd Makefile target
    # `ablations`: the same kernels plus the measurement variants and layout switches); the
    # product library refuses them
    os.environ["SPMV_HW_ABLATIONS"] = "1"
    dtype = np.float64 if a.dtype == "f64" else np.float32
    lib = spmv_hw.load(dtype)
    variants = [v if ":" in v else f"tiles:{v}" for v in a.variants.split(",")]
    for wl in a.workload.split(","):
        mcols = None
        if wl == "banded":
            n = a.rows or 1_000_000
            rp, col, val = spmv_hw.gen_banded(lib, n, 16)
            x = spmv_hw.gen_vector(lib, n, seed=3)
        elif wl in ("stencil7", "stencil27"):
            rp, col, val, n = stencil(a.rows or 8_000_000, 7 if wl == "stencil7" else 27, dtype)
            x = spmv_hw.gen_vector(lib, n, seed=3)
        else:
            n = a.rows or 10_000_000
            mcols = a.cols or n
            rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, mcols, a.nnz or 16 * n)
            x = spmv_hw.gen_vector(lib, mcols, seed=6)
        mcols = mcols or n
        plans = {}
        for v in variants:
            k, var = v.split(":")
            if k not in plans:  # "sweep@512" = 512-thread workgroups, "sweepU" = unpacked entries
                kern = k.partition("#")[0]  # "binned#2": a second plan of the same layout (duplicate)
                kern, _, threads = kern.partition("@")
                kern, _, pskew = kern.partition("^")  # "binned^4096": SPMV_BIN_PROD_SKEW=4096
                if pskew:
                    os.environ["SPMV_BIN_PROD_SKEW"] = pskew
                kern, _, xbias = kern.partition("~")  # "sweep~0.012": SPMV_SWEEP_XCC_BIAS=0.012
                if xbias:  # "binned~0.025": SPMV_BIN_XCC_BIAS (pass-1 window widths)
                    os.environ["SPMV_BIN_XCC_BIAS" if kern.startswith("binned") else "SPMV_SWEEP_XCC_BIAS"] = xbias
                if kern.endswith("U"):
                    kern = kern[:-1]
                    os.environ["SPMV_SWEEP_PACKED"] = "0"
                if kern.endswith("S"):  # sweep without split panels (smaller panels instead)
                    kern = kern[:-1]
                    os.environ["SPMV_SWEEP_SPLIT"] = "0"
                if kern.endswith("F"):  # sweep with split panels whenever they fit
                    kern = kern[:-1]
                    os.environ["SPMV_SWEEP_SPLIT"] = "2"
                if kern.endswith("X"):  # tile kernel with XCD-contiguous (not round-robin) tiles
                    kern = kern[:-1]
                    os.environ["SPMV_TILE_XCD"] = "1"
                if kern.endswith("H"):  # tile kernel with at most 16-bit column offsets
                    kern = kern[:-1]
                    os.environ["SPMV_TILE_NARROW"] = "16"
                if kern.endswith("W"):  # tile kernel with 32-bit columns (no narrow form)
                    kern = kern[:-1]
                    os.environ["SPMV_TILE_NARROW"] = "0"
                if kern.endswith("L"):  # packed, without the lane-order permutation
                    kern = kern[:-1]
                    os.environ["SPMV_SWEEP_LANE_ORDER"] = "0"
                if kern.endswith("D"):  # deterministic sweep (one row segment per wave)
                    kern = kern[:-1]
                    os.environ["SPMV_SWEEP_DETERMINISTIC"] = "1"
                if kern.endswith("F32"):  # sweep with the fp32 (CAS) LDS accumulator for fp32 matrices
                    kern = kern[:-3]
                    os.environ["SPMV_SWEEP_ACC"] = "32"
                if kern.endswith("A32"):  # slices with the fp32 row accumulator (fp32 matrices)
                    kern = kern[:-3]
                    os.environ["SPMV_SLICE_ACC"] = "32"
                if kern.startswith("blocked") and kern[7:].isdigit():  # blockedW: W-column blocks
                    os.environ["SPMV_FPGA_BLOCK"] = kern[7:]
                    kern = "blocked"
                os.environ["SPMV_HW_KERNEL"] = kern
                if threads:
                    os.environ["SPMV_SWEEP_THREADS"] = threads
                plans[k] = spmv_hw.Plan.from_device(lib, rp, col, val, mcols)
                os.environ.pop("SPMV_SWEEP_THREADS", None)
                os.environ.pop("SPMV_SWEEP_PACKED", None)
                os.environ.pop("SPMV_SWEEP_LANE_ORDER", None)
                os.environ.pop("SPMV_TILE_NARROW", None)
                os.environ.pop("SPMV_SWEEP_SPLIT", None)
                os.environ.pop("SPMV_TILE_XCD", None)
                os.environ.pop("SPMV_FPGA_BLOCK", None)
                os.environ.pop("SPMV_SWEEP_ACC", None)
                os.environ.pop("SPMV_SLICE_ACC", None)
                os.environ.pop("SPMV_SWEEP_DETERMINISTIC", None)
                os.environ.pop("SPMV_SWEEP_XCC_BIAS", None)
                os.environ.pop("SPMV_BIN_XCC_BIAS", None)
                os.environ.pop("SPMV_BIN_PROD_SKEW", None)
        os.environ.pop("SPMV_HW_KERNEL", None)
        st = next(iter(plans.values())).stats()
        del rp, col, val
        y = torch.empty(n, dtype=x.dtype, device="cuda")
        res = {v: [] for v in variants}
        ref = None
        for r in range(a.rounds):
            for v in variants:
                k, var = v.split(":")
                plan = plans[k]
                plan.set_variant(int(var))
                plan.run(x, y)
                torch.cuda.synchronize()
                if ref is None:
                    ref = y.clone()
                elif int(var) not in (50, 51, 52, 53, 54, 55, 60, 61, 62, 63) and not (k.startswith("blocked") and var == "1"):  # measurement-only ablations (wrong y)
                    err = float(((ref - y).abs().max() / ref.abs().max().clamp_min(1e-300)).item())
                    assert err < (1e-9 if a.dtype == "f64" else 1e-5), f"{v} changed the result ({err})"
                plan.set_timing(True)
                for _ in range(a.reps):
                    plan.run(x, y)
                ms, _, _ = plan.timing()
                plan.set_timing(False)
                res[v].append(ms)
        out = {"workload": wl, "dtype": a.dtype, "nnz": st["nr_nzeros"], "alg_bytes": st["algorithmic_bytes"],
               "library": os.path.basename(os.path.dirname(lib.path)),
               "plans": {k: {kk: p.stats()[kk] for kk in ("kernel", "nr_tiles", "device_bytes")} for k, p in plans.items()}}
        # (device_bytes tells packed 12-B entries from unpacked 14-B ones)
        for v in variants:
            med = float(np.median(res[v]))
            out[v] = {"median_ms": round(med, 5), "min_ms": round(min(res[v]), 5),
                      "alg_GBps": round(st["algorithmic_bytes"] / (med * 1e-3) / 1e9, 1)}
        print(json.dumps(out), flush=True)
        for p in plans.values():
            p.destroy()


if __name__ == "__main__":
    main()
