#!/usr/bin/env python3
"""Conjugate gradient on the GPU with the MI355X SpMV plan as its operator — the iterative use
of the path: A stays resident in HBM as a plan, each iteration is one
spmv_plan_run plus a few vector updates, and the whole iteration is captured once in a CUDA/HIP
graph and replayed (no host round trip per iteration).

    python examples/cg.py [--grid 1000] [--iters 200] [--graph]

Matrix: the 2-D 5-point Laplacian on a grid x grid mesh plus a diagonal shift (SPD).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import torch  # noqa: E402

import spmv_hw  # noqa: E402


def laplacian_2d(g: int, shift: float = 0.1):
    """CSR of the 5-point Laplacian on a g x g grid plus shift * I (columns sorted per row)."""
    n = g * g
    idx = np.arange(n, dtype=np.int64)
    r, c = idx // g, idx % g
    offs = [(-g, r > 0), (-1, c > 0), (0, np.ones(n, bool)), (1, c < g - 1), (g, r < g - 1)]
    cols = np.full((n, 5), -1, np.int64)
    vals = np.zeros((n, 5))
    for k, (o, ok) in enumerate(offs):
        cols[ok, k] = idx[ok] + o
        vals[ok, k] = 4.0 + shift if o == 0 else -1.0
    keep = cols >= 0
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(keep.sum(axis=1))
    return rp.astype(np.uint32), cols[keep].astype(np.uint32), vals[keep], n


def cg(plan, b, iters: int, use_graph: bool):
    """Unpreconditioned CG, fixed iteration count, all state on the GPU."""
    x = torch.zeros_like(b)
    r = b.clone()
    p = r.clone()
    ap = torch.empty_like(b)
    rr = torch.dot(r, r)

    def step():
        nonlocal rr
        plan.run(p, ap)
        alpha = rr / torch.dot(p, ap)
        x.add_(alpha * p)
        r.sub_(alpha * ap)
        rr_new = torch.dot(r, r)
        p.mul_(rr_new / rr).add_(r)
        rr.copy_(rr_new)

    if not use_graph:
        for _ in range(iters):
            step()
        return x
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm up outside the capture (one real iteration)
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(iters - 1):
        g.replay()
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1000)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    lib = spmv_hw.load(np.float64)
    rp, col, val, n = laplacian_2d(a.grid)
    dev = lambda h: torch.from_numpy(h.view(np.int32) if h.dtype == np.uint32 else h).cuda()
    plan = spmv_hw.Plan.from_device(lib, dev(rp), dev(col), dev(val), n)
    b = torch.ones(n, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x = cg(plan, b, a.iters, a.graph)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ax = torch.empty_like(b)
    plan.run(x, ax)
    res = float(torch.linalg.norm(b - ax) / torch.linalg.norm(b))
    print(f"n={n} nnz={int(rp[-1])} iters={a.iters} graph={a.graph} time={dt * 1e3:.2f} ms "
          f"({dt * 1e6 / a.iters:.1f} us/iter) relative residual {res:.3e} kernel={plan.stats()['kernel']}")
    plan.destroy()
    return res


if __name__ == "__main__":
    main()
