"""Iterative / persistent mode: spmv_plan_run_graph replays a captured
hipGraph of SpMVs, and spmv_plan_run is capturable into a caller's graph. Same parity bar as
tests/test_gpu_parity.py (componentwise-scaled error vs the oracle); the tile kernel is also
bitwise equal to its eager launch."""
import numpy as np
import pytest

import oracle
import spmv_hw
from test_gpu_parity import TIGHT, kernel, torch  # noqa: F401  (fixtures)

pytestmark = pytest.mark.gpu


def _problem(lib, n=200_000, z=3_200_000):
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    return rp, col, val, x


def _host(*ts):
    return [t.cpu().numpy() for t in ts]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_run_graph_matches_eager_and_oracle(torch, kernel, dtype):
    lib = spmv_hw.load(dtype)
    rp, col, val, x = _problem(lib)
    n = x.numel()
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    y_eager = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y_eager)
    y_g = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    for iters in (1, 4, 4):  # capture, re-capture (iters changed), replay
        y_g.fill_(float("nan"))
        plan.run_graph(x, y_g, iters)
    torch.cuda.synchronize()
    rp_h, c_h, v_h, x_h, ye, yg = _host(rp, col, val, x, y_eager, y_g)
    rp_h, c_h = rp_h.view(np.uint32), c_h.view(np.uint32)
    ref = oracle.spmv_gold(rp_h, c_h, v_h, x_h)
    assert oracle.scaled_error(rp_h, c_h, v_h, x_h, ref, yg) <= TIGHT[np.dtype(dtype)]
    if kernel.startswith("tiles"):
        assert np.array_equal(ye.view(np.uint8), yg.view(np.uint8))
    plan.destroy()


def test_run_graph_recaptures_on_new_buffers(torch):
    lib = spmv_hw.load(np.float64)
    rp, col, val, x = _problem(lib, 50_000, 800_000)
    n = x.numel()
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    y1 = torch.zeros(n, dtype=x.dtype, device="cuda")
    y2 = torch.zeros(n, dtype=x.dtype, device="cuda")
    x2 = 2 * x
    plan.run_graph(x, y1, 2)
    plan.run_graph(x2, y2, 2)  # different x and y: must not replay the first graph
    torch.cuda.synchronize()
    assert torch.allclose(2 * y1, y2, rtol=1e-12, atol=0)
    plan.destroy()


def test_run_graph_timing_counts_graph_launches(torch):
    lib = spmv_hw.load(np.float64)
    rp, col, val, x = _problem(lib, 50_000, 800_000)
    n = x.numel()
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    y = torch.empty(n, dtype=x.dtype, device="cuda")
    plan.run_graph(x, y, 8)
    plan.set_timing(True)
    for _ in range(3):
        plan.run_graph(x, y, 8)
    mean_ms, total_ms, launches = plan.timing()
    assert launches == 3 and mean_ms > 0 and abs(total_ms - 3 * mean_ms) < 1e-9 + 1e-6 * total_ms
    plan.destroy()


def test_plan_run_is_capturable_into_a_torch_graph(torch, kernel):
    """A caller's own graph: SpMV followed by an update of x, replayed (an iterative solver's
    step; here x <- y / ||y||_inf, a power iteration on a square matrix)."""
    lib = spmv_hw.load(np.float64)
    rp, col, val, x = _problem(lib, 50_000, 800_000)
    n = x.numel()
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    y = torch.empty(n, dtype=x.dtype, device="cuda")
    x_ref = x.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up outside the capture
        plan.run(x, y)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    x.copy_(x_ref)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        plan.run(x, y)
        x.copy_(y / y.abs().max())
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    # the same three steps eagerly, checked against the oracle step by step
    rp_h, c_h, v_h = _host(rp, col, val)
    rp_h, c_h = rp_h.view(np.uint32), c_h.view(np.uint32)
    xh = x_ref.cpu().numpy()
    for _ in range(3):
        yh = oracle.spmv_gold(rp_h, c_h, v_h, xh)
        xh = yh / np.abs(yh).max()
    err = np.abs(x.cpu().numpy() - xh).max()
    assert err <= 1e-12, err
    plan.destroy()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_distinct_plans_run_concurrently_on_two_streams(torch, dtype):
    """Plan-owned scratch (the split sweep's partial sums, the binned kernel's products) belongs
    to one plan: two plans of the same matrix -- the sweep and the binned kernel -- launched on
    two streams at once, repeatedly, each give the oracle's y."""
    import os
    lib = spmv_hw.load(dtype)
    rp, col, val, x = _problem(lib, 1_000_000, 16_000_000)
    n = x.numel()
    plans = []
    for kern in ("sweep", "binned"):
        os.environ["SPMV_HW_KERNEL"] = kern
        try:
            plans.append(spmv_hw.Plan.from_device(lib, rp, col, val, n))
        finally:
            os.environ.pop("SPMV_HW_KERNEL", None)
    assert [p.stats()["kernel"] for p in plans] == [2, 6]
    ys = [torch.full((n,), float("nan"), dtype=x.dtype, device="cuda") for _ in plans]
    streams = [torch.cuda.Stream() for _ in plans]
    torch.cuda.synchronize()
    for _ in range(10):
        for p, y, s in zip(plans, ys, streams):
            p.run(x, y, s)
    torch.cuda.synchronize()
    rp_h, c_h, v_h, x_h = _host(rp, col, val, x)
    rp_h, c_h = rp_h.view(np.uint32), c_h.view(np.uint32)
    ref = oracle.spmv_gold(rp_h, c_h, v_h, x_h)
    for p, y in zip(plans, ys):
        err = oracle.scaled_error(rp_h, c_h, v_h, x_h, ref, y.cpu().numpy())
        assert err <= TIGHT[np.dtype(dtype)], (p.stats()["kernel"], err)
        p.destroy()


@pytest.mark.parametrize("iters", [1, 2, 3, 6])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_run_graph_overlaps_the_split_combine(torch, monkeypatch, dtype, iters):
    """A split sweep plan (rank 0 of the N = 8 cut of the 10M/160M matrix: panels cut into
    pieces, partial sums added by k_sweep_combine) replays with the combine of step k carried by
    step k + 1's sweep launch (the "behind" form: extra blocks behind the units, two partial
    buffers, a last combine kernel). y after the replay (and after a second replay, and a fresh x
    through a re-capture) matches the oracle, as with the tools build's other capture forms
    (SPMV_GRAPH_FORM=serial: one chain; dag: the combine on a second stream)."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    n = 10_000_000
    for ablations, env in ((False, None), (True, "SPMV_GRAPH_FORM=serial"), (True, "SPMV_GRAPH_FORM=dag")):
        monkeypatch.delenv("SPMV_GRAPH_FORM", raising=False)
        if env:
            monkeypatch.setenv(*env.split("="))
        lib = spmv_hw.load(dtype, ablations=ablations)
        rp_full, _ = lib.powerlaw_row_ptr(n, 160_000_000, 65536, 4)
        b = lib.partition_rows(rp_full, 8)
        r0, r1 = int(b[0]), int(b[1])
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 160_000_000, seed=4, row_begin=r0, row_end=r1)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
        assert plan.stats()["nr_tiles"] > 200  # split: ~62 panels in ~4 pieces each
        form = plan.stats()["format"] & (256 | 512)  # the capture form run_graph will use
        assert form == {None: 256, "SPMV_GRAPH_FORM=serial": 0, "SPMV_GRAPH_FORM=dag": 512}[env], (env, form)
        h = _host(rp, col, val)
        r, c = h[0].view(np.uint32), h[1].view(np.uint32)
        for seed in (6, 7):  # a new x buffer re-captures the graph
            x = spmv_hw.gen_vector(lib, n, seed=seed, lo=-1.0 if seed == 7 else 0.0)
            ref = (oracle.spmv_fp64acc if dtype == np.float32 else oracle.spmv_gold)(r, c, h[2], x.cpu().numpy())
            y = torch.full((r1 - r0,), float("nan"), dtype=x.dtype, device="cuda")
            for _ in range(2):  # capture + replay, then a second replay
                plan.run_graph(x, y, iters)
                torch.cuda.synchronize()
                err = oracle.scaled_error(r, c, h[2], x.cpu().numpy(), ref, y.cpu().numpy())
                assert err <= TIGHT[np.dtype(dtype)], (env, seed, err)
        plan.destroy()


@pytest.mark.parametrize("iters", [2, 5])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_run_graph_behind_two_pieces(torch, monkeypatch, dtype, iters):
    """The behind form on a panel cut into two pieces (rank 1 of the N = 4 cut: ~126 panels x 2),
    an odd step count (the last combine reads the second partial buffer), then eager runs of the
    same plan after the replay (the launch's extra blocks and counters leave nothing behind)."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    n = 10_000_000
    lib = spmv_hw.load(dtype)
    rp_full, _ = lib.powerlaw_row_ptr(n, 160_000_000, 65536, 4)
    b = lib.partition_rows(rp_full, 4)
    r0, r1 = int(b[1]), int(b[2])
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 160_000_000, seed=4, row_begin=r0, row_end=r1)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    assert plan.stats()["nr_tiles"] > 200
    h = _host(rp, col, val)
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    x = spmv_hw.gen_vector(lib, n, seed=9, lo=-1.0)
    ref = (oracle.spmv_fp64acc if dtype == np.float32 else oracle.spmv_gold)(r, c, h[2], x.cpu().numpy())
    for run in ("graph", "graph", "eager"):
        y = torch.full((r1 - r0,), float("nan"), dtype=x.dtype, device="cuda")
        if run == "graph":
            plan.run_graph(x, y, iters)
        else:
            plan.run(x, y)
        torch.cuda.synchronize()
        err = oracle.scaled_error(r, c, h[2], x.cpu().numpy(), ref, y.cpu().numpy())
        assert err <= TIGHT[np.dtype(dtype)], (run, err)
    plan.destroy()
