"""Does a split plan's graph replay run the combine of step k beside the sweep of step k + 1?
Reads a `rocprofv3 --kernel-trace --output-format csv` kernel trace (tools/gpu_session.sh
tracegraph) and, for every run of consecutive split-sweep / combine launches, prints how long each
combine overlaps the next sweep, the queue each ran on, and the gap from one sweep's end to the
next sweep's start. Measurement tool only.

usage: python tools/graph_overlap.py gpurun_out/<tag>/trace_graph/.../run_kernel_trace.csv
"""
import csv
import json
import statistics
import sys


def main(path):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        kind = "sweep" if "k_spmv_sweep" in name else "combine" if "k_sweep_combine" in name else None
        if kind:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r["Queue_Id"], r["Stream_Id"]))
    rows.sort()
    sweeps = [r for r in rows if r[2] == "sweep"]
    combines = [r for r in rows if r[2] == "combine"]
    overlaps, gaps, pairs = [], [], 0
    for i in range(len(sweeps) - 1):
        s0, s1 = sweeps[i], sweeps[i + 1]
        gaps.append((s1[0] - s0[1]) / 1e3)
        # the combine that started after sweep i ended and before sweep i + 1 ended
        c = next((c for c in combines if s0[1] <= c[0] <= s1[1]), None)
        if c is None:
            continue
        pairs += 1
        overlaps.append(max(0, min(c[1], s1[1]) - max(c[0], s1[0])) / 1e3)
    out = {
        "trace": path, "sweeps": len(sweeps), "combines": len(combines), "pairs": pairs,
        "combine_us_median": statistics.median([(c[1] - c[0]) / 1e3 for c in combines]) if combines else None,
        "overlap_us_median": statistics.median(overlaps) if overlaps else None,
        "pairs_overlapping": sum(o > 0 for o in overlaps),
        "sweep_to_sweep_gap_us_median": statistics.median(gaps) if gaps else None,
        "queues": sorted({(r[2], r[3], r[4]) for r in rows}),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
