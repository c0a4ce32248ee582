#!/usr/bin/env python3
"""Reader throughput: spmv_read_csr (Part 3, parallel mmap + from_chars) vs the oracle's
restatement of the reference reader (fgets + sscanf, csr.cpp:87-136) on one generated file in
the reference format. Prints one JSON line. Host only (no GPU).
Usage: bench_reader.py [--nnz Z] [--rows N] [--threads T,...] [--dir D]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spmv-fpga_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
import spmv_hw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--nnz", type=int, default=16_000_000)
    ap.add_argument("--threads", default="1,4,8,16")
    ap.add_argument("--dir", default="/tmp")
    a = ap.parse_args()
    path = os.path.join(a.dir, f"reader_{a.rows}_{a.nnz}.mtx")
    if not os.path.exists(path):
        rng = np.random.default_rng(2)
        rows = np.sort(rng.integers(1, a.rows + 1, a.nnz))
        rows[-1] = a.rows
        cols = rng.integers(1, a.rows + 1, a.nnz)
        vals = rng.uniform(-1, 1, a.nnz)
        with open(path, "w") as f:
            f.write(f"{a.rows} {a.rows} {a.nnz}\n")
            for s in range(0, a.nnz, 1_000_000):
                e = min(a.nnz, s + 1_000_000)
                np.savetxt(f, np.column_stack([rows[s:e], cols[s:e], vals[s:e]]), fmt=["%d", "%d", "%.17g"])
    size = os.path.getsize(path)
    lib = spmv_hw.load(np.float64)
    out = {"file_bytes": size, "nnz": a.nnz, "rows": a.rows, "cpu_count": os.cpu_count()}
    t0 = time.perf_counter()
    ref = oracle.read_csr(path, np.float64)
    out["oracle_s"] = round(time.perf_counter() - t0, 3)
    res = {}
    for t in [int(v) for v in a.threads.split(",")]:
        os.environ["SPMV_READ_THREADS"] = str(t)
        t0 = time.perf_counter()
        rp, col, val, _ = lib.read_csr(path)
        dt = time.perf_counter() - t0
        same = (np.array_equal(rp, ref[2]) and np.array_equal(col, ref[3])
                and np.array_equal(val.view(np.uint64), ref[4].view(np.uint64)))
        res[str(t)] = {"s": round(dt, 3), "MB_per_s": round(size / dt / 1e6, 1), "bitwise_equal": bool(same)}
        del rp, col, val
    out["spmv_read_csr"] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
