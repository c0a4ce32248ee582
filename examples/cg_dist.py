#!/usr/bin/env python3
"""Conjugate gradient over N GPUs, one process per GPU: the multi-GPU iterative use of the path
(SURVEY.md §8e + §8f rank 3). Each rank holds a plan for its nnz-balanced row slice of A
(spmv_partition_rows, the reference's per-CU split, csr_hw.cpp:459-468), its slices of x, r and
p, and a full-length copy of p, which is the operand of its SpMV. One iteration is:

    ap = A[rows] p                      spmv_plan_run on the rank's slice
    alpha = rr / allreduce(p[rows].ap)  the two dot products are all-reduces
    x[rows] += alpha p[rows];  r[rows] -= alpha ap
    rr' = allreduce(r[rows].r[rows]);  p[rows] = r[rows] + (rr' / rr) p[rows]
    p = allgather(p[rows])              the y -> x exchange of the dependent form

so every step depends on the previous one's exchange (the form bench.py reports as
`step_forms.dependent`). torch.distributed over RCCL ('nccl', one rank per GPU) or gloo (ranks
may share a GPU: the one-GPU rehearsal).

    python examples/cg_dist.py --gpus 2 [--backend gloo] [--grid 1000] [--iters 200]

Matrix: the 2-D 5-point Laplacian plus a diagonal shift (examples/cg.py). Rank 0 gathers x and
prints the relative residual ||b - A x|| / ||b|| computed with a single-GPU plan of the whole A.
"""
from __future__ import annotations

import argparse
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
sys.path.insert(0, os.path.join(ROOT, "examples"))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=2, help="ranks (one process each)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None,
                    help="default: nccl when every rank has its own GPU, else gloo")
    ap.add_argument("--grid", type=int, default=1000)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--tol", type=float, default=1e-8,
                    help="exit status 2 when the final relative residual is above this")
    ap.add_argument("--timeout", type=float, default=300.0,
                    help="seconds the whole run may take: every collective gives up after it, and the "
                         "parent kills ranks still running then (exit status 124)")
    return ap.parse_args(argv)


def _die_with_parent():
    """A rank is SIGKILLed when the parent dies (Linux prctl PR_SET_PDEATHSIG): a parent killed by
    a test's timeout leaves no rank on the GPU."""
    try:
        import ctypes
        import signal
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGKILL, 0, 0, 0)
    except Exception:
        pass


def rank_main(rank, world, port, args, out_q=None):
    _die_with_parent()
    import datetime

    import torch
    import torch.distributed as dist

    import spmv_dist
    import spmv_hw
    from cg import laplacian_2d

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(rank % ndev)
    dev = torch.device("cuda", rank % ndev)
    tmo = datetime.timedelta(seconds=args.timeout)  # every collective gives up, none waits forever
    if args.backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, timeout=tmo)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=tmo)
    res = None
    try:
        lib = spmv_hw.load(np.float64)
        rp, col, val, n = laplacian_2d(args.grid)
        bounds = lib.partition_rows(rp, world)
        counts = spmv_dist.slice_counts(bounds)
        r0, r1 = spmv_dist.row_slice(bounds, rank)
        e0, e1 = int(rp[r0]), int(rp[r1])
        to = lambda h: torch.from_numpy(np.ascontiguousarray(h).view(np.int32) if h.dtype == np.uint32 else h).to(dev)  # noqa: E731
        plan = spmv_hw.Plan.from_device(lib, to((rp[r0:r1 + 1] - rp[r0]).astype(np.uint32)),
                                        to(col[e0:e1] if e1 > e0 else np.zeros(1, np.uint32)),
                                        to(val[e0:e1] if e1 > e0 else np.zeros(1)), n, device=dev.index)

        def allreduce(t):
            s = spmv_dist._staged(t)
            dist.all_reduce(s)
            return s.to(dev) if s is not t else s

        b = torch.ones(r1 - r0, dtype=torch.float64, device=dev)
        x = torch.zeros_like(b)
        r = b.clone()
        p_full = torch.zeros(n, dtype=torch.float64, device=dev)
        spmv_dist.exchange_allgather(r, counts, out=p_full)  # p = r = b
        ap = torch.empty_like(b)
        rr = allreduce(torch.dot(r, r).reshape(1))
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            plan.run(p_full, ap)
            p = p_full[r0:r1]
            alpha = rr / allreduce(torch.dot(p, ap).reshape(1))
            x.add_(alpha * p)
            r.sub_(alpha * ap)
            rr_new = allreduce(torch.dot(r, r).reshape(1))
            p_new = r + (rr_new / rr) * p
            rr = rr_new
            spmv_dist.exchange_allgather(p_new, counts, out=p_full)
        torch.cuda.synchronize()
        dist.barrier()
        dt = time.perf_counter() - t0
        x_full = spmv_dist.exchange_gather(x, counts)
        if rank == 0:
            x_full = x_full.to(dev)
            whole = spmv_hw.Plan.from_device(lib, to(rp), to(col), to(val), n, device=dev.index)
            ax = torch.empty(n, dtype=torch.float64, device=dev)
            whole.run(x_full, ax)
            bf = torch.ones(n, dtype=torch.float64, device=dev)
            res = float(torch.linalg.norm(bf - ax) / torch.linalg.norm(bf))
            whole.destroy()
            line = (f"n={n} nnz={int(rp[-1])} ranks={world} backend={dist.get_backend()} iters={args.iters} "
                    f"time={dt * 1e3:.2f} ms ({dt * 1e6 / args.iters:.1f} us/iter) relative residual {res:.3e} "
                    f"rows/rank={list(map(int, counts))}")
            print(line, flush=True)
            if out_q is not None:
                out_q.put(res)
        plan.destroy()
    finally:
        dist.destroy_process_group()
    if rank == 0 and not res <= args.tol:  # (NaN included)
        print(f"relative residual {res:.3e} above --tol {args.tol:g}", file=sys.stderr, flush=True)
        sys.exit(2)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def main(argv=None):
    args = parse(argv)
    import torch  # noqa: F401  (device_count does not initialise the GPU on this image)
    import torch.multiprocessing as mp
    if args.backend is None:
        args.backend = "nccl" if args.gpus <= torch.cuda.device_count() else "gloo"
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=rank_main, args=(r, args.gpus, port, args), daemon=True) for r in range(args.gpus)]
    for p in procs:
        p.start()
    deadline = time.monotonic() + args.timeout
    for p in procs:  # one deadline for the whole run, not one per rank
        p.join(timeout=max(0.0, deadline - time.monotonic()))
    hung = [r for r, p in enumerate(procs) if p.is_alive()]
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    if hung:
        print(f"cg_dist: ranks {hung} still running after {args.timeout:g} s, killed", file=sys.stderr, flush=True)
        return 124
    codes = [p.exitcode for p in procs]
    return 0 if all(c == 0 for c in codes) else max((c for c in codes if c and c > 0), default=1)


if __name__ == "__main__":
    sys.exit(main())
