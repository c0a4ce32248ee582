#!/usr/bin/env python3
"""Workgroup timeline of one k_spmv_sweep_packed launch (measurement build, SPMV_HW_ABLATIONS=1):
where the time of a strong-scaling slice goes (the N = 8 slice costs ~5.6 ps per
non-zero against 4.8 in the whole matrix).

For each workgroup the kernel records the 100 MHz real-time clock at its start, at the end of its
sweep and after its y / partial-sum store, plus its XCC id. After a few warm runs of the plan this
prints, for the last launch: the start spread (dispatch ramp), the distribution of sweep end times
(the tail: how long the first-finished CUs sit idle), the store phase, and per-XCC means. One JSON
line per matrix. Rows [r0, r1) of the 10M/160M power-law matrix (--slice k/N: slice k of N).
--binned: the fp32 10M/160M matrix on the binned kernel, per pass the workgroup durations and
their even- / odd-XCC means.
Measurement tool, not product code."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

os.environ["SPMV_HW_ABLATIONS"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import torch  # noqa: E402

import spmv_hw  # noqa: E402


def pct(a, q):
    return round(float(np.percentile(a, q)), 2)


def read_stamps(lib, units, binned_pass=None):
    n = 4 * min(units, 4096)
    buf = (ctypes.c_ulonglong * n)()
    rc = (lib.L.spmv_abl_wg_times(buf, ctypes.c_uint(n)) if binned_pass is None
          else lib.L.spmv_abl_bin_times(ctypes.c_int(binned_pass), buf, ctypes.c_uint(n)))
    if rc:
        raise RuntimeError("reading the workgroup stamps failed")
    return np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4).copy()


def bin_pass(a):
    """start / end clocks of one binned pass (slots 0, 1) and the XCC id (slot 3)."""
    t = a[:, :2].astype(np.int64)
    us = (t - t[:, 0].min()) / 100.0
    xcc = (a[:, 3] >> np.uint64(32)).astype(np.int64)
    dur = us[:, 1] - us[:, 0]
    return {"units": int(len(a)), "dur_us": {"min": pct(dur, 0), "p50": pct(dur, 50), "max": pct(dur, 100)},
            "end_us": {"p10": pct(us[:, 1], 10), "p50": pct(us[:, 1], 50), "max": pct(us[:, 1], 100)},
            "even_xcc_dur_us": round(float(dur[xcc % 2 == 0].mean()), 2),
            "odd_xcc_dur_us": round(float(dur[xcc % 2 == 1].mean()), 2),
            "per_xcc_dur_us": {int(k): round(float(dur[xcc == k].mean()), 2) for k in np.unique(xcc)}}


def timeline(lib, plan, x, y, units):
    for _ in range(5):
        plan.run(x, y)
    torch.cuda.synchronize()
    a = read_stamps(lib, units)
    t = a[:, :3].astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # 100 MHz ticks -> microseconds
    xcc = (a[:, 3] >> np.uint64(32)).astype(np.int64)
    start, sweep_end, done = us[:, 0], us[:, 1], us[:, 2]
    per_xcc = {int(k): {"n": int((xcc == k).sum()), "sweep_us": round(float((sweep_end - start)[xcc == k].mean()), 2),
                        "end_us": round(float(done[xcc == k].mean()), 2)} for k in np.unique(xcc)}
    return {"units": int(units), "start_us": {"p50": pct(start, 50), "max": pct(start, 100)},
            "sweep_us": {"min": pct(sweep_end - start, 0), "p50": pct(sweep_end - start, 50),
                         "max": pct(sweep_end - start, 100)},
            "sweep_end_us": {"min": pct(sweep_end, 0), "p10": pct(sweep_end, 10), "p50": pct(sweep_end, 50),
                             "p90": pct(sweep_end, 90), "max": pct(sweep_end, 100)},
            "store_us": {"p50": pct(done - sweep_end, 50), "max": pct(done - sweep_end, 100)},
            "last_done_us": pct(done, 100),
            "idle_frac": round(float(1.0 - (done - start).sum() / (len(done) * done.max())), 4),
            "per_xcc": per_xcc}


def consistency(lib, plan, x, y, units, launches):
    """Is a unit's sweep time a property of the unit? Per-unit sweep durations over `launches`
    launches: the correlation of two launches' durations, the spread of the per-unit means (the
    part a one-time re-cut of the units could remove) and of the residuals (the part it could
    not), and the longest sweep if every unit's mean were brought to the median."""
    durs = []
    for _ in range(launches):
        plan.run(x, y)
        torch.cuda.synchronize()
        a = read_stamps(lib, units)
        t = a[:, :2].astype(np.int64)
        durs.append((t[:, 1] - t[:, 0]) / 100.0)
    d = np.array(durs)  # launches x units
    mean = d.mean(axis=0)
    resid = d - mean
    cc = [float(np.corrcoef(d[i], d[i + 1])[0, 1]) for i in range(launches - 1)]
    med = float(np.median(mean))
    return {"launches": launches, "corr_consecutive_p50": round(float(np.median(cc)), 3),
            "unit_mean_us": {"min": pct(mean, 0), "p50": pct(mean, 50), "max": pct(mean, 100)},
            "resid_us": {"p5": pct(resid, 5), "p95": pct(resid, 95), "max": pct(resid, 100)},
            "max_sweep_us_p50": round(float(np.median(d.max(axis=1))), 2),
            "max_sweep_us_if_rebalanced_p50": round(float(np.median((med + resid).max(axis=1))), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--consistency", type=int, default=0,
                    help="K > 1: per-unit sweep durations over K launches (is the tail systematic?)")
    ap.add_argument("--slices", default="0/8,0/4,0/1", help="k/N: rows of slice k of N (nnz-balanced)")
    ap.add_argument("--binned", action="store_true",
                    help="the fp32 10M/160M matrix on the binned kernel instead: both passes' timelines")
    a = ap.parse_args()
    if a.binned:
        os.environ["SPMV_HW_KERNEL"] = "binned"
        lib = spmv_hw.load(np.float32)
        n, z = 10_000_000, 160_000_000
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
        x = spmv_hw.gen_vector(lib, n, seed=6)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
        y = torch.empty(n, dtype=torch.float32, device="cuda")
        for _ in range(5):
            plan.run(x, y)
        torch.cuda.synchronize()
        st = plan.stats()
        out = {"matrix": "powerlaw 10M/160M fp32", "kernel": st["kernel"]}
        for k in (0, 1):  # every slot, trimmed to the workgroups that ran (unused slots stay 0)
            raw = read_stamps(lib, 4096, k)
            out["pass%d" % (k + 1)] = bin_pass(raw[raw[:, 1] > 0])
        print(json.dumps(out), flush=True)
        return
    lib = spmv_hw.load(np.float64)
    n, z = 10_000_000, 160_000_000
    rp_full, _ = lib.powerlaw_row_ptr(n, z, n, 4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    for sl in a.slices.split(","):
        k, N = (int(v) for v in sl.split("/"))
        cuts = np.searchsorted(rp_full, [z * i // N for i in range(N + 1)])
        cuts[0], cuts[-1] = 0, n
        r0, r1 = int(cuts[k]), int(cuts[k + 1])
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4, row_begin=r0, row_end=r1)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
        st = plan.stats()
        y = torch.empty(r1 - r0, dtype=torch.float64, device="cuda")
        out = {"slice": sl, "rows": r1 - r0, "nnz": st["nr_nzeros"], "kernel": st["kernel"], "format": st["format"]}
        if st["kernel"] == 2:
            out.update(timeline(lib, plan, x, y, st["nr_tiles"]))
            if a.consistency > 1:
                out["consistency"] = consistency(lib, plan, x, y, st["nr_tiles"], a.consistency)
        print(json.dumps(out), flush=True)
        plan.destroy()
        del rp, col, val, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
