#!/usr/bin/env python3
"""Config 4 (strong scaling) rehearsed on ONE GPU: for N in 1,2,4,8 the rank slices of the
10M x 10M / 160M-nnz power-law matrix (nnz-balanced, exactly as bench.py --scaling strong cuts
them) are built and timed one after another; the slowest slice is the compute-only step time of
an N-GPU run. Prints one JSON line per N (kernel ms of the slowest slice, implied aggregate
GFLOP/s and speed-up vs N=1). The y exchange is not included (bench.py reports it per mode).
Usage: strong_slices.py [--ns 1,2,4,8] [--slices all|ends] [--dtype f64|f32]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spmv-fpga_amd")]
import torch  # noqa: E402

import spmv_dist  # noqa: E402
import spmv_hw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--nnz", type=int, default=160_000_000)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--slices", default="ends", help="'all' slices, or first+last only")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default=None, help="recorded as _setting in every line (e.g. the env under test)")
    ap.add_argument("--variants", default=None,
                    help="comma list of spmv_plan_set_variant values timed interleaved on each slice's plan "
                         "(e.g. 28,36: the split sweep with and without work stealing)")
    ap.add_argument("--rounds", type=int, default=5, help="with --variants / --graph-ab: interleaved rounds")
    ap.add_argument("--graph-ab", type=int, default=0,
                    help="K > 0: per slice, K SpMVs replayed from one hipGraph (spmv_plan_run_graph) in "
                         "each capture form of --graph-modes (tools build), interleaved; ms per step")
    ap.add_argument("--graph-modes", default="product,dag,serial",
                    help="with --graph-ab: the captures compared -- product (the library's choice), or "
                         "SPMV_GRAPH_FORM=serial|dag|behind, with _rN (SPMV_BEHIND_ROWS) / _bN (SPMV_BEHIND_BLOCKS)")
    a = ap.parse_args()
    dtype = np.float64 if a.dtype == "f64" else np.float32
    lib = spmv_hw.load(dtype, ablations=bool(a.graph_ab or a.variants) or None)
    n, z = a.rows, a.nnz
    rp_full, _ = lib.powerlaw_row_ptr(n, z, 65536, 4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    base = None
    for N in [int(v) for v in a.ns.split(",")]:
        b = lib.partition_rows(rp_full, N)
        ranks = range(N) if a.slices == "all" or N <= 2 else (0, N - 1)
        worst, per, worst_v = 0.0, {}, {}
        for r in ranks:
            r0, r1 = spmv_dist.row_slice(b, r)
            rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4, row_begin=r0, row_end=r1)
            plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
            del rp, col, val
            y = torch.empty(r1 - r0, dtype=x.dtype, device="cuda")
            for _ in range(3):
                plan.run(x, y)
            st = plan.stats()
            if a.graph_ab:  # overlapped vs serial graph capture, interleaved (median ms per step)
                times = {m: [] for m in a.graph_modes.split(",")}
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(a.rounds):
                    for mode in times:
                        for k in ("SPMV_GRAPH_FORM", "SPMV_BEHIND_ROWS", "SPMV_BEHIND_BLOCKS"):
                            os.environ.pop(k, None)
                        form, *knobs = mode.split("_")  # e.g. behind_r2048_b512
                        if form != "product":
                            os.environ["SPMV_GRAPH_FORM"] = form
                        for kn in knobs:
                            os.environ["SPMV_BEHIND_ROWS" if kn[0] == "r" else "SPMV_BEHIND_BLOCKS"] = kn[1:]
                        plan.set_variant(28)  # drops the captured graph: the next call re-captures
                        plan.run_graph(x, y, a.graph_ab)
                        torch.cuda.synchronize()
                        ev0.record()
                        plan.run_graph(x, y, a.graph_ab)
                        ev1.record()
                        torch.cuda.synchronize()
                        times[mode].append(ev0.elapsed_time(ev1) / a.graph_ab)
                for k in ("SPMV_GRAPH_FORM", "SPMV_BEHIND_ROWS", "SPMV_BEHIND_BLOCKS"):
                    os.environ.pop(k, None)
                med = {m: float(np.median(t)) for m, t in times.items()}
                per[r] = {"rows": r1 - r0, "nnz": st["nr_nzeros"], "kernel": st["kernel"], "panels": st["nr_tiles"],
                          "xcc_lighter": "even" if st["format"] & 1024 else "odd" if st["format"] & 2048 else "none",
                          "graph_ms_per_step": {m: round(v, 5) for m, v in med.items()},
                          "graph_min_ms": {m: round(min(t), 5) for m, t in times.items()}}
                ms = med.get("product", min(med.values()))
                for m in med:
                    worst_v[m] = max(worst_v.get(m, 0.0), med[m])
            elif a.variants:  # interleaved A/B of plan variants on this slice (median per variant)
                vs = [int(v) for v in a.variants.split(",")]
                times = {v: [] for v in vs}
                for _ in range(a.rounds):
                    for v in vs:
                        plan.set_variant(v)
                        plan.run(x, y)
                        plan.set_timing(True)
                        for _ in range(a.reps):
                            plan.run(x, y)
                        times[v].append(plan.timing()[0])
                        plan.set_timing(False)
                med = {v: float(np.median(t)) for v, t in times.items()}
                per[r] = {"rows": r1 - r0, "nnz": st["nr_nzeros"], "kernel": st["kernel"], "panels": st["nr_tiles"],
                          "format": st["format"], "variants_ms": {str(v): round(m, 5) for v, m in med.items()},
                          "variants_min_ms": {str(v): round(min(t), 5) for v, t in times.items()}}
                ms = med[vs[0]]
                for v in vs:
                    worst_v[v] = max(worst_v.get(v, 0.0), med[v])
            else:
                plan.set_timing(True)
                for _ in range(a.reps):
                    plan.run(x, y)
                ms, _, _ = plan.timing()
                per[r] = {"rows": r1 - r0, "nnz": st["nr_nzeros"], "kernel": st["kernel"], "ms": round(ms, 5),
                          "panels": st["nr_tiles"]}
            worst = max(worst, ms)
            plan.destroy()
            torch.cuda.empty_cache()
        gflops = 2.0 * z / (worst * 1e-3) / 1e9
        if base is None:
            base = worst
        print(json.dumps({"n_gpus": N, "dtype": a.dtype, "slowest_slice_ms": round(worst, 5),
                          "aggregate_GFLOPs": round(gflops, 1), "speedup_vs_1": round(base / worst, 3),
                          "slices": per, **({"slowest_by_variant_ms": {str(v): round(t, 5) for v, t in worst_v.items()}}
                                            if worst_v else {}),
                          **({"_setting": a.tag} if a.tag else {})}), flush=True)


if __name__ == "__main__":
    main()
