"""How do the steps of a split plan's replay sit on the GPU? Reads a `rocprofv3 --kernel-trace
--output-format csv` kernel trace (tools/gpu_session.sh tracegraph: strong_slices.py --graph-ab
under the profiler) and prints one line per run of sweep launches (a replay, or the eager
warm-up): launches, HW queues, grid sizes (the "behind" form's launches carry extra blocks), the
median period from one sweep launch's start to the next, the idle gap between them, the median
sweep launch and the median separate combine launch. Measurement tool only.

usage: python tools/graph_overlap.py gpurun_out/<tag>/trace_graph/run_kernel_trace.csv
"""
import csv
import json
import statistics
import sys


def segments(path, split_ns=1_000_000):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        kind = "sweep" if "k_spmv_sweep" in name else "combine" if "k_sweep_combine" in name else None
        if kind:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r["Queue_Id"],
                         int(r["Grid_Size_X"])))
    rows.sort()
    sweeps = [r for r in rows if r[2] == "sweep"]
    if not sweeps:
        return []
    segs = [[sweeps[0]]]
    for a, b in zip(sweeps, sweeps[1:]):
        if b[0] - a[0] > split_ns:  # a new replay (or the warm-up) starts
            segs.append([])
        segs[-1].append(b)
    out = []
    for g in segs:
        lo, hi = g[0][0], g[-1][1]
        comb = [(c[1] - c[0]) / 1e3 for c in rows if c[2] == "combine" and lo <= c[0] <= hi]
        med = lambda v: round(statistics.median(v), 2) if v else None  # noqa: E731
        out.append({"launches": len(g), "queues": sorted({x[3] for x in g}), "grids": sorted({x[4] for x in g}),
                    "period_us": med([(b[0] - a[0]) / 1e3 for a, b in zip(g, g[1:])]),
                    "gap_us": med([(b[0] - a[1]) / 1e3 for a, b in zip(g, g[1:])]),
                    "sweep_us": med([(x[1] - x[0]) / 1e3 for x in g]), "combine_us": med(comb)})
    return out


if __name__ == "__main__":
    for s in segments(sys.argv[1]):
        print(json.dumps(s))
