"""The multi-GPU merge as data: spmv_mgpu_schedule (host.cpp) lists what
every rank issues for one SpMV step, and mgpu.cpp's RCCL calls iterate over that list. These CPU
tests execute the same arithmetic without a GPU:

  * the lists themselves, for 1..8 ranks with uneven, empty and zero-row slices: every row of y
    is written exactly once (gather), every send has its matching receive, every rank lists the
    same collectives in the same order (reduce, all-gather) -- the conditions under which the
    RCCL group cannot deadlock or drop rows;
  * a torch.distributed (gloo) replay of the SAME lists (spmv_dist.execute_schedule), world
    sizes 2, 3, 5 and 8, both slots of the pipelined double buffer: rank 0's y (gather, reduce)
    and every rank's next x (all-gather) equal the oracle's spmv_gold bit for bit. This is the
    reference's accum_results loop (csr_hw.cpp:1531-1565 over the CUs of
    csr_hw_wrapper.cpp:276-281) on slices of rows.
The per-rank product here is the CPU oracle standing in for the GPU kernel (test only)."""
import os
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))
import spmv_hw  # noqa: E402

GATHER, REDUCE, ALLGATHER = spmv_hw.MGPU_GATHER, spmv_hw.MGPU_REDUCE, spmv_hw.MGPU_ALLGATHER


@pytest.fixture(scope="module")
def lib():
    return spmv_hw.load(np.float64)


def _bounds_cases():
    rng = np.random.default_rng(11)
    out = []
    for nr in range(1, 9):
        n = 1000
        cuts = np.sort(rng.integers(0, n + 1, nr - 1))
        out.append((nr, [0, *cuts.tolist(), n]))  # uneven (may repeat: empty slices)
        if nr >= 2:
            b = np.linspace(0, n, nr + 1).astype(int).tolist()
            b[1] = 0  # rank 0 empty
            out.append((nr, b))
            b = np.linspace(0, n, nr + 1).astype(int).tolist()
            b[-2] = n  # last rank empty
            out.append((nr, b))
        out.append((nr, [0] * (nr + 1)))  # a matrix with no rows
    return out


@pytest.mark.parametrize("nr,bounds", _bounds_cases())
def test_schedule_covers_every_row_once(lib, nr, bounds):
    n = bounds[-1]
    rows = [bounds[r + 1] - bounds[r] for r in range(nr)]
    sch = {ex: [lib.mgpu_schedule(ex, r, nr, bounds) for r in range(nr)] for ex in (GATHER, REDUCE, ALLGATHER)}
    for ex, per_rank in sch.items():
        for r, ops in enumerate(per_rank):
            kinds = [o["kind"] for o in ops]
            # local ops first, then the exchange (one RCCL group)
            assert kinds == sorted(kinds, key=lambda k: k >= spmv_hw.XOP_SEND), kinds
            comp = [o for o in ops if o["kind"] == spmv_hw.XOP_COMPUTE]
            assert len(comp) == (1 if rows[r] else 0)  # empty slices compute nothing
            for o in comp:
                assert o["count"] == rows[r]
                assert o["offset"] == (0 if o["buf"] == spmv_hw.XBUF_SLICE else bounds[r])
            for o in ops:
                assert o["count"] > 0
    # gather: rank 0's y written exactly once (its own rows + one receive per non-empty slice)
    cover = np.zeros(n, np.int64)
    for o in sch[GATHER][0]:
        assert o["buf"] == spmv_hw.XBUF_Y
        cover[o["offset"]:o["offset"] + o["count"]] += 1
    assert np.all(cover == 1)
    sends = {r: [o for o in sch[GATHER][r] if o["kind"] == spmv_hw.XOP_SEND] for r in range(1, nr)}
    recvs = [o for o in sch[GATHER][0] if o["kind"] == spmv_hw.XOP_RECV]
    assert sorted((o["peer"], o["count"]) for o in recvs) == sorted(
        (r, s["count"]) for r, ss in sends.items() for s in ss)
    for r, ss in sends.items():
        assert all(s["peer"] == 0 and s["buf"] == spmv_hw.XBUF_SLICE and s["offset"] == 0 for s in ss)
        assert len(ss) == (1 if rows[r] else 0)
    for o in recvs:
        assert o["offset"] == bounds[o["peer"]] and o["count"] == rows[o["peer"]]
    # reduce: zero the whole partial, one identical reduce on every rank, sum lands in rank 0's y
    for r, ops in enumerate(sch[REDUCE]):
        if n == 0:
            assert ops == []
            continue
        assert ops[0] == {"kind": spmv_hw.XOP_ZERO, "buf": spmv_hw.XBUF_PART, "peer": -1, "out": -1, "offset": 0, "count": n}
        red = [o for o in ops if o["kind"] == spmv_hw.XOP_REDUCE]
        assert red == [{"kind": spmv_hw.XOP_REDUCE, "buf": spmv_hw.XBUF_PART, "peer": 0,
                        "out": spmv_hw.XBUF_Y if r == 0 else -1, "offset": 0, "count": n}]
    # all-gather: every rank lists the same broadcasts in the same order, covering x once
    coll = [[o for o in ops if o["kind"] == spmv_hw.XOP_BCAST] for ops in sch[ALLGATHER]]
    assert all(c == coll[0] for c in coll)
    if nr > 1:
        cover = np.zeros(n, np.int64)
        for o in coll[0]:
            assert o["offset"] == bounds[o["peer"]] and o["count"] == rows[o["peer"]]
            cover[o["offset"]:o["offset"] + o["count"]] += 1
        assert np.all(cover == 1)
    else:
        assert coll[0] == []


def test_schedule_known_lists(lib):
    """The exact lists for 3 ranks with an empty middle slice, bounds [0, 5, 5, 9]."""
    b = [0, 5, 5, 9]
    s = lambda ex, r: [(o["kind"], o["buf"], o["peer"], o["out"], o["offset"], o["count"])  # noqa: E731
                       for o in lib.mgpu_schedule(ex, r, 3, b)]
    C, S, R, RED, BC, Z = (spmv_hw.XOP_COMPUTE, spmv_hw.XOP_SEND, spmv_hw.XOP_RECV, spmv_hw.XOP_REDUCE,
                           spmv_hw.XOP_BCAST, spmv_hw.XOP_ZERO)
    Y, SL, P, XN = spmv_hw.XBUF_Y, spmv_hw.XBUF_SLICE, spmv_hw.XBUF_PART, spmv_hw.XBUF_XNEXT
    assert s(GATHER, 0) == [(C, Y, -1, -1, 0, 5), (R, Y, 2, -1, 5, 4)]
    assert s(GATHER, 1) == []
    assert s(GATHER, 2) == [(C, SL, -1, -1, 0, 4), (S, SL, 0, -1, 0, 4)]
    assert s(REDUCE, 0) == [(Z, P, -1, -1, 0, 9), (C, P, -1, -1, 0, 5), (RED, P, 0, Y, 0, 9)]
    assert s(REDUCE, 1) == [(Z, P, -1, -1, 0, 9), (RED, P, 0, -1, 0, 9)]
    assert s(ALLGATHER, 1) == [(BC, XN, 0, -1, 0, 5), (BC, XN, 2, -1, 5, 4)]
    # one rank: a gather exchanges nothing, a reduce still goes through RCCL (copies the partial)
    assert lib.mgpu_schedule(GATHER, 0, 1, [0, 9]) == [
        {"kind": C, "buf": Y, "peer": -1, "out": -1, "offset": 0, "count": 9}]
    assert [o["kind"] for o in lib.mgpu_schedule(REDUCE, 0, 1, [0, 9])] == [Z, C, RED]


def test_schedule_rejects_bad_arguments(lib):
    L = lib.L
    b = np.array([0, 5, 3], np.uint32)  # decreasing
    bp = b.ctypes.data_as(spmv_hw.ctypes.POINTER(spmv_hw.IndexType))
    assert L.spmv_mgpu_schedule(GATHER, 0, 2, bp, None, 0) == -1
    b = np.array([0, 5, 9], np.uint32)
    bp = b.ctypes.data_as(spmv_hw.ctypes.POINTER(spmv_hw.IndexType))
    assert L.spmv_mgpu_schedule(3, 0, 2, bp, None, 0) == -1   # no such exchange
    assert L.spmv_mgpu_schedule(GATHER, 2, 2, bp, None, 0) == -1  # rank out of range
    assert L.spmv_mgpu_schedule(GATHER, 0, 2, bp, None, 0) == 2  # count only


def _store(tmp_path):
    """Rendezvous through a file (torch FileStore) in the test's own directory: no TCP port to
    pick, so parallel test workers cannot collide on one."""
    return str(tmp_path / "pg_store")


def _worker(rank, world, store, pattern, q):
    for p in (ROOT, os.path.join(ROOT, "spmv-fpga_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import torch
    import torch.distributed as dist

    import oracle
    import spmv_dist as sdist
    import spmv_hw as hw

    dist.init_process_group("gloo", init_method="file://" + store, rank=rank, world_size=world)
    try:
        lib = hw.load(np.float64)
        rng = np.random.default_rng(7)
        n = 6000
        lens = np.minimum(np.floor(6 * rng.random(n) ** -0.5), 2000).astype(np.int64)
        lens[rng.random(n) < 0.05] = 0
        row_ptr = np.zeros(n + 1, np.int64)
        row_ptr[1:] = np.cumsum(lens)
        row_ptr = row_ptr.astype(np.uint32)
        z = int(row_ptr[-1])
        col = rng.integers(0, n, z).astype(np.uint32)
        val = rng.uniform(-1, 1, z)
        x = rng.uniform(0, 1, n)
        bounds = lib.partition_rows(row_ptr, world).astype(np.int64)
        if pattern == "empty":  # rank 0 empty, and (world >= 3) the last rank too
            bounds[1] = 0
            if world >= 3:
                bounds[world - 1] = n
        r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
        bounds = bounds.astype(np.uint32)

        def compute_with(xv):
            def compute(view):
                oracle.spmv_gold_rows(row_ptr, col, val, xv, r0, r1, out=view.numpy())
            return compute

        results = {}
        # single steps of the three forms
        for ex in (hw.MGPU_GATHER, hw.MGPU_REDUCE, hw.MGPU_ALLGATHER):
            ops = lib.mgpu_schedule(ex, rank, world, bounds)
            nan = float("nan")  # unwritten rows must not survive into the result
            bufs = {hw.XBUF_Y: torch.full((n,), nan, dtype=torch.float64),
                    hw.XBUF_SLICE: torch.full((max(r1 - r0, 1),), nan, dtype=torch.float64),
                    hw.XBUF_PART: torch.full((n,), nan, dtype=torch.float64),
                    hw.XBUF_XNEXT: torch.full((n,), nan, dtype=torch.float64)}
            sdist.execute_schedule(ops, bufs, compute_with(x))
            out = bufs[hw.XBUF_XNEXT] if ex == hw.MGPU_ALLGATHER else bufs[hw.XBUF_Y]
            results[ex] = out.numpy().copy()
        # the pipelined form: 5 steps, step k of x * (k + 1) into buffer set k & 1
        piped = {}
        for ex in (hw.MGPU_GATHER, hw.MGPU_REDUCE):
            ops = lib.mgpu_schedule(ex, rank, world, bounds)
            sets = [{b: torch.full((n if b != hw.XBUF_SLICE else max(r1 - r0, 1),), float("nan"), dtype=torch.float64)
                     for b in (hw.XBUF_Y, hw.XBUF_SLICE, hw.XBUF_PART)} for _ in range(2)]
            per_step = []
            for k in range(5):
                sdist.execute_schedule(ops, sets[k & 1], compute_with(x * (k + 1)))
                per_step.append(sets[k & 1][hw.XBUF_Y].numpy().copy())
            piped[ex] = per_step
        y_ref = oracle.spmv_gold(row_ptr, col, val, x)
        ok = {"allgather": bool(np.array_equal(results[hw.MGPU_ALLGATHER], y_ref))}
        if rank == 0:
            ok["gather"] = bool(np.array_equal(results[hw.MGPU_GATHER], y_ref))
            ok["reduce"] = bool(np.array_equal(results[hw.MGPU_REDUCE], y_ref))
            for ex, name in ((hw.MGPU_GATHER, "pipe_gather"), (hw.MGPU_REDUCE, "pipe_reduce")):
                ok[name] = all(np.array_equal(piped[ex][k], oracle.spmv_gold(row_ptr, col, val, x * (k + 1)))
                               for k in range(5))
        q.put((rank, ok, [int(b) for b in bounds]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pattern", ["balanced", "empty"])
@pytest.mark.parametrize("world", [2, 3, 5, 8])
def test_gloo_replay_of_schedule_matches_oracle(world, pattern, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    store = _store(tmp_path)
    procs = [ctx.Process(target=_worker, args=(r, world, store, pattern, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    got = dict((r, (ok, b)) for r, ok, b in (q.get(timeout=10) for _ in range(world)))
    bounds = got[0][1]
    if pattern == "empty":
        assert bounds[1] == 0 and (world < 3 or bounds[world - 1] == bounds[world])
    for r in range(world):
        ok = got[r][0]
        assert all(ok.values()), (r, ok)
    assert set(got[0][0]) == {"allgather", "gather", "reduce", "pipe_gather", "pipe_reduce"}
