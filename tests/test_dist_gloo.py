"""World-size-2 (and 3) gloo runs of the multi-GPU layout on CPU: nnz-balanced row slices per
rank, x replicated, and the three RCCL exchange forms (reduce of full-length partials = the
accum_results '+=' mapping; gather of disjoint slices to rank 0; all-gather of padded slices to
every rank, the iterative-solver form) rebuilding the full y.
The per-rank product here is the CPU oracle standing in for the GPU kernel (test only)."""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _store(tmp_path):
    """Rendezvous through a file (torch FileStore) in the test's own directory: no TCP port to
    pick, so parallel test workers cannot collide on one."""
    return str(tmp_path / "pg_store")


def _worker(rank, world, store, mode, q):
    for p in (ROOT, os.path.join(ROOT, "spmv-fpga_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import spmv_dist as sdist
    import oracle
    import spmv_hw

    dist.init_process_group("gloo", init_method="file://" + store, rank=rank, world_size=world)
    try:
        lib = spmv_hw.load(np.float64)
        rng = np.random.default_rng(5)
        n = 20_000
        lens = np.minimum(np.floor(8 * rng.random(n) ** -0.5), 3000).astype(np.int64)
        lens[rng.random(n) < 0.05] = 0
        row_ptr = np.zeros(n + 1, np.int64)
        row_ptr[1:] = np.cumsum(lens)
        z = int(row_ptr[-1])
        col = rng.integers(0, n, z).astype(np.uint32)
        val = rng.uniform(-1, 1, z)
        x = rng.uniform(0, 1, n)
        row_ptr = row_ptr.astype(np.uint32)
        bounds = lib.partition_rows(row_ptr, world)
        r0, r1 = sdist.row_slice(bounds, rank)
        rp = row_ptr[r0:r1 + 1]
        y_local = oracle.spmv_gold((rp - rp[0]).astype(np.uint32), col[rp[0]:rp[-1]], val[rp[0]:rp[-1]], x)
        y_t = torch.from_numpy(y_local)
        if mode == "pipelined":
            # 5 SpMVs, each of a different x (x scaled by k + 1), their gathers overlapping the
            # next SpMV; the last step's y reaches rank 0 whole
            counts = sdist.slice_counts(bounds)
            sub = ((rp - rp[0]).astype(np.uint32), col[rp[0]:rp[-1]], val[rp[0]:rp[-1]])
            bufs = [torch.zeros(int(max(counts)), dtype=torch.float64) for _ in range(2)]

            def step(k, yb):
                yb[:r1 - r0] = torch.from_numpy(oracle.spmv_gold(*sub, x * (k + 1)))

            full = sdist.pipelined_gather(step, bufs, counts, 5)
        elif mode == "dependent":
            # bench.py's dependent form (x <- A x): each rank's slice of A x_k, all-gathered into a
            # preallocated next-x buffer (a view, as bench passes it), three steps
            counts = sdist.slice_counts(bounds)
            sub = ((rp - rp[0]).astype(np.uint32), col[rp[0]:rp[-1]], val[rp[0]:rp[-1]])
            bufs = [torch.from_numpy(x.copy()), torch.zeros(n + 7, dtype=torch.float64)]
            for k in range(3):
                src, dst = bufs[k % 2], bufs[(k + 1) % 2]
                ys = torch.from_numpy(oracle.spmv_gold(*sub, src[:n].numpy()))
                sdist.exchange_allgather(ys, counts, out=dst[:n])
            full = bufs[1][:n]
            ref = x
            for _ in range(3):
                ref = oracle.spmv_gold(row_ptr, col, val, ref)
            assert np.array_equal(full.numpy(), ref)  # every rank holds A^3 x
        elif mode == "reduce":
            full = sdist.exchange_reduce(y_t, r0, n)
        elif mode == "gather":
            full = sdist.exchange_gather(y_t, sdist.slice_counts(bounds))
        else:  # every rank receives the whole y (next x of an iterative solver)
            full = sdist.exchange_allgather(y_t, sdist.slice_counts(bounds))
            assert np.array_equal(full.numpy(), oracle.spmv_gold(row_ptr, col, val, x))
        xb = torch.from_numpy(x.copy() if rank == 0 else np.zeros_like(x))
        sdist.broadcast_x(xb)
        assert np.array_equal(xb.numpy(), x)
        m = sdist.max_over_ranks(float(rank), torch.device("cpu"))
        if rank == 0:
            if mode == "dependent":
                y_ref = ref
            else:
                y_ref = oracle.spmv_gold(row_ptr, col, val, x * 5 if mode == "pipelined" else x)  # last step: x * 5
            q.put((np.array_equal(full.numpy(), y_ref), m, list(sdist.slice_counts(bounds))))
        elif mode not in ("allgather", "dependent"):
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("mode", ["reduce", "gather", "allgather", "pipelined", "dependent"])
def test_row_sliced_exchange_rebuilds_y(world, mode, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = _store(tmp_path)
    procs = [ctx.Process(target=_worker, args=(r, world, store, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, m, counts = q.get(timeout=10)
    assert ok, "exchanged y differs from the single-process oracle"
    assert m == world - 1
    assert sum(counts) == 20_000 and min(counts) > 0


def _rank0_worker(rank, world, store, q):
    for p in (ROOT, os.path.join(ROOT, "spmv-fpga_amd")):
        sys.path.insert(0, p)
    import time

    import torch.distributed as dist

    import spmv_dist as sdist

    dist.init_process_group("gloo", init_method="file://" + store, rank=rank, world_size=world)
    try:
        got = []

        def work(result):
            def fn():
                time.sleep(0.5)  # the waiting ranks block on the store meanwhile
                if result is None:
                    raise RuntimeError("boom")
                return result
            return fn

        for result in ({"pass": True}, {"pass": False}, None):
            got.append(sdist.rank0_only(work(result), 30, passed=lambda r: r.get("pass") is not False))
        # rank 0 never answers a fourth call: the other ranks give up after their timeout
        if rank == 0:
            got.append((None, "skipped"))
        else:
            got.append(sdist.rank0_only(lambda: None, 1))
        dist.barrier()
        q.put((rank, got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_rank0_only_waits_on_the_store(world, tmp_path):
    """bench.py's N-unit drop-in run at N > 1: rank 0 alone runs the child (every GPU of the node)
    while the other ranks wait on the process group's store, not in a GPU collective; every rank
    learns whether rank 0's result passed, and a waiting rank gives up after its timeout."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = _store(tmp_path)
    procs = [ctx.Process(target=_rank0_worker, args=(r, world, store, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = dict(q.get(timeout=10) for _ in range(world))
    assert [s for _, s in res[0]] == ["ok", "fail", "error", "skipped"]
    assert res[0][0][0] == {"pass": True} and "boom" in res[0][2][0]["error"]
    for r in range(1, world):
        assert res[r] == [(None, "ok"), (None, "fail"), (None, "error"), (None, "timeout")]
