#!/usr/bin/env python3
"""Times the drop-in spmv_hw (csr_hw_wrapper.cpp:193-288) under each y merge (VERDICT r2 item 3:
"keep the per-GPU PCIe merge behind an env switch and report both timings").

One process, the Part-1 API as the reference's main.cpp drives it: create_csr_hw_matrix on host
CSR arrays (SPMV_NGPUS units, one per visible GPU), create_csr_hw_x_vector, then spmv_hw into a
host y. One matrix per merge (SPMV_HW_MERGE = host, gather, reduce, read at create), each timed
under every --variants entry (sets of the merge knobs spmv_hw reads per call: pieced copy on/off,
pieces, add split, add threads), all in interleaved rounds. The library's own printed lines
("Hardware execution time", "Result accumulation time", "Total time", csr_hw_wrapper.cpp:272-285)
are captured from fd 1; their medians are reported beside the wall time of one call, the bare
device-to-pinned-host copy of y (the floor of the accumulation) and y's max relative difference
against the first merge. With one GPU the RCCL forms are one-rank collectives (the cost of the
branch itself); on a node with G GPUs the same command compares the G-link PCIe merge with the
xGMI gather/reduce plus one D2H copy. Prints one JSON line per (merge, variant).
Measurement tool, not product code."""
import argparse
import json
import os
import re
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import torch  # noqa: E402

import spmv_hw  # noqa: E402

KNOBS = {"pipe": "SPMV_HW_PIPELINE", "pieces": "SPMV_HW_PIECES", "split": "SPMV_HW_ADD_SPLIT",
         "threads": "SPMV_HW_ADD_THREADS", "stream": "SPMV_HW_STREAM", "direct": "SPMV_HW_DIRECT",
         "shape": "SPMV_HW_PIECE_SHAPE"}
LINES = {"hw_ms": "Hardware execution time", "accum_ms": "Result accumulation time", "total_ms": "Total time"}


class Flow:
    """One create_csr_hw_matrix under SPMV_HW_MERGE=merge (read at create), with its x and y."""

    def __init__(self, lib, merge, rp, col, val, x, ncols, dtype):
        os.environ["SPMV_HW_MERGE"] = merge
        self.lib, self.r = lib, len(rp) - 1
        self.hw, self.bm = lib.create_csr_hw_matrix(lib.make_csr_matrix(rp, col, val, ncols))
        self.hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), 1, self.hw[0].contents.nr_cols)
        self.yv = lib.make_csr_vector(np.zeros(self.r, dtype))
        self.lib.spmv_hw(self.hw, self.hx, self.yv, self.bm)  # warms the pinned staging and RCCL
        self.y_one = np.ctypeslib.as_array(self.yv.values, shape=(self.r,)).copy()

    def time(self, env, calls):
        """printed times and wall ms of `calls` spmv_hw calls under `env` (the merge knobs
        SPMV_HW_PIPELINE / _PIECES / _ADD_SPLIT / _ADD_THREADS are read per call)."""
        for k in KNOBS.values():
            os.environ.pop(k, None)
        os.environ.update(env)
        wall = []
        sys.stdout.flush()
        saved = os.dup(1)
        with tempfile.TemporaryFile(mode="w+") as f:
            os.dup2(f.fileno(), 1)
            try:
                for _ in range(calls):
                    t0 = time.perf_counter()
                    self.lib.spmv_hw(self.hw, self.hx, self.yv, self.bm)
                    wall.append((time.perf_counter() - t0) * 1e3)
            finally:
                os.dup2(saved, 1)
                os.close(saved)
            f.seek(0)
            text = f.read()
        out = {"wall_ms": wall}
        for key, label in LINES.items():
            out[key] = [float(v) for v in re.findall(re.escape(label) + r"\s*:\s*([0-9.eE+-]+) ms", text)]
        return out

    def close(self):
        self.lib.delete_csr_hw_matrix(self.hw)
        self.lib.free_bitmap(self.bm)
        self.lib.delete_csr_hw_x_vector(self.hx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--nnz", type=int, default=160_000_000)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--calls", type=int, default=5, help="calls per mode per round")
    ap.add_argument("--rounds", type=int, default=5, help="interleaved rounds over the modes")
    ap.add_argument("--merges", default="host,gather,reduce")
    ap.add_argument("--variants", default="default;pipe=0",
                    help="';'-separated knob sets, e.g. 'default;pipe=0;pieces=8,split=0' (knobs: %s)" % ", ".join(KNOBS))
    ap.add_argument("--tools", action="store_true",
                    help="load the tools build (lib/ablations), where the pieces / split / threads knobs apply")
    a = ap.parse_args()
    dtype = np.float64 if a.dtype == "f64" else np.float32
    ndev = torch.cuda.device_count()
    os.environ["SPMV_NGPUS"] = str(ndev)
    lib = spmv_hw.load(dtype, ablations=a.tools)
    n = a.rows
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, a.nnz, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    h_rp, h_col = rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32)
    h_val, h_x = val.cpu().numpy(), x.cpu().numpy()
    del rp, col, val, x
    # the bare PCIe copy of y (device -> pinned host), the floor of every merge's accumulation
    yd = torch.empty(n, dtype=torch.float64 if a.dtype == "f64" else torch.float32, device="cuda")
    yh = torch.empty(yd.shape, dtype=yd.dtype, pin_memory=True)
    d2h = []
    for _ in range(a.calls + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        yh.copy_(yd, non_blocking=True)
        torch.cuda.synchronize()
        d2h.append((time.perf_counter() - t0) * 1e3)
    del yd, yh
    torch.cuda.empty_cache()
    flows = {m: Flow(lib, m, h_rp, h_col, h_val, h_x, n, dtype) for m in a.merges.split(",")}
    variants = []
    for v in a.variants.split(";"):
        env = {} if v == "default" else {KNOBS[k]: val for k, _, val in (kv.partition("=") for kv in v.split(","))}
        variants.append((v, env))
    modes = [(m, v) for m in flows for v in range(len(variants))]
    acc = {md: {} for md in modes}
    for _ in range(a.rounds):
        for md in modes:
            for k, v in flows[md[0]].time(variants[md[1]][1], a.calls).items():
                acc[md].setdefault(k, []).extend(v)
    y_ref = next(iter(flows.values())).y_one.astype(np.float64)
    for (m, vi), t in acc.items():
        y = flows[m].y_one
        diff = float(np.max(np.abs(y - y_ref)) / max(float(np.max(np.abs(y_ref))), 1e-300))
        print(json.dumps({"merge": m, "variant": variants[vi][0], "gpus": ndev, "units": ndev, "dtype": a.dtype,
                          "rows": n, "nnz": a.nnz, "calls": len(t["wall_ms"]),
                          **{k: round(float(np.median(v)), 4) for k, v in t.items()},
                          "d2h_only_ms": round(float(np.median(d2h[1:])), 4),
                          "max_rel_diff_vs_first": diff}), flush=True)
    for f in flows.values():
        f.close()


if __name__ == "__main__":
    main()
