"""Part 4 of the C-ABI (spmv_mgpu_*): one process drives the visible GPUs through one RCCL clique
(ncclCommInitAll) -- nnz-balanced row slices per device (csr_hw.cpp:459-468), x replicated by an
RCCL broadcast (spmv.cpp:280-294), y exchanged on the devices: send/recv gather of the slices,
reduce of full-length partials (accum_results' +=, csr_hw.cpp:1531-1565) and the all-gather that
makes y the next x. Runs with every GPU the box has (1 on the test box; the driver's 8-GPU node
runs the same code with 8). y is checked against the oracle's spmv_gold (csr.cpp:184-194)."""
import numpy as np
import pytest

import oracle
import spmv_hw
from conftest import GOLDEN, manifest

pytestmark = pytest.mark.gpu

TOL = {np.dtype(np.float64): 1e-12, np.dtype(np.float32): 2e-6}


def _ndev():
    import torch
    return torch.cuda.device_count()


def _powerlaw_host(lib, n, z):
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    return (rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32), val.cpu().numpy(),
            x.cpu().numpy())


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("exchange", [spmv_hw.MGPU_GATHER, spmv_hw.MGPU_REDUCE])
@pytest.mark.parametrize("kern", ["auto", "binned"])
def test_mgpu_gather_and_reduce_match_oracle(monkeypatch, dtype, exchange, kern):
    if kern != "auto":  # every device's plan on that kernel
        monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    lib = spmv_hw.load(dtype)
    n, z = 300_000, 4_800_000
    rp, col, val, x = _powerlaw_host(lib, n, z)
    m = lib.make_csr_matrix(rp, col, val, n)
    mg = spmv_hw.MultiGpu(lib, m, ndev=_ndev())
    slices = [mg.slice(d) for d in range(mg.ndev)]
    assert slices[0][0] == 0 and slices[-1][1] == n
    assert all(slices[d][1] == slices[d + 1][0] for d in range(mg.ndev - 1))
    mg.set_x(x)
    ref = oracle.spmv_gold(rp, col, val, x)
    for _ in range(2):  # the second run reuses the exchange buffers
        mg.run(exchange)
        y = mg.y(exchange)
        assert oracle.scaled_error(rp, col, val, x, ref, y) <= TOL[np.dtype(dtype)]
    c, e = mg.timing()
    assert c > 0 and e >= 0
    mg.destroy()


def test_mgpu_allgather_iterates_y_into_x():
    """Two all-gather runs compute A(Ax): the first y becomes every device's next x."""
    lib = spmv_hw.load(np.float64)
    n, z = 200_000, 3_200_000
    rp, col, val, x = _powerlaw_host(lib, n, z)
    m = lib.make_csr_matrix(rp, col, val, n)
    mg = spmv_hw.MultiGpu(lib, m, ndev=_ndev())
    mg.set_x(x)
    mg.run(spmv_hw.MGPU_ALLGATHER)
    y1 = mg.y(spmv_hw.MGPU_ALLGATHER)
    ref1 = oracle.spmv_gold(rp, col, val, x)
    assert oracle.scaled_error(rp, col, val, x, ref1, y1) <= 1e-12
    mg.run(spmv_hw.MGPU_ALLGATHER)
    y2 = mg.y(spmv_hw.MGPU_ALLGATHER)
    ref2 = oracle.spmv_gold(rp, col, val, y1)
    assert oracle.scaled_error(rp, col, val, y1, ref2, y2) <= 1e-12
    mg.destroy()


@pytest.mark.parametrize("name", sorted(manifest().keys()))
def test_mgpu_on_golden_fixtures(name):
    import os
    lib = spmv_hw.load(np.float64)
    _, c, rp, col, val, _ = oracle.read_csr(os.path.join(GOLDEN, manifest()[name]["file"]), np.float64)
    x = np.load(os.path.join(GOLDEN, f"{name}.x.f64.npy"), allow_pickle=False)
    y_gold = np.load(os.path.join(GOLDEN, f"{name}.y_gold.f64.npy"), allow_pickle=False)
    mg = spmv_hw.MultiGpu(lib, lib.make_csr_matrix(rp, col, val, c), ndev=_ndev())
    mg.set_x(x)
    for ex in (spmv_hw.MGPU_GATHER, spmv_hw.MGPU_REDUCE):
        mg.run(ex)
        assert oracle.scaled_error(rp, col, val, x, y_gold, mg.y(ex)) <= 1e-12
    mg.destroy()


def test_mgpu_rejects_bad_devices():
    lib = spmv_hw.load(np.float64)
    rp = np.array([0, 1], np.uint32)
    m = lib.make_csr_matrix(rp, np.zeros(1, np.uint32), np.ones(1), 1)
    with pytest.raises(RuntimeError, match="does not exist"):
        spmv_hw.MultiGpu(lib, m, devices=[_ndev()])
    with pytest.raises(RuntimeError, match="appears twice"):
        spmv_hw.MultiGpu(lib, m, devices=[0, 0])


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_mgpu_rank_mode_single_rank(dtype):
    """The one-process-per-GPU form (spmv_mgpu_create_rank: RCCL id from spmv_mgpu_unique_id,
    ncclCommInitRank, the caller's own plan) as rank 0 of 1: all three exchanges, x from a device
    tensor, y read back on the host and as a device address. bench.py --gpus N uses the same
    calls on every rank."""
    import torch
    lib = spmv_hw.load(dtype)
    n, z = 200_000, 3_200_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    uid = spmv_hw.mgpu_unique_id(lib)
    assert len(uid) == 128
    mg = spmv_hw.MultiGpu.rank(lib, 0, 1, uid, 0, [0, n], n, plan)
    assert mg.slice(0) == (0, n, 0)
    mg.set_x_device(x)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    for ex in (spmv_hw.MGPU_GATHER, spmv_hw.MGPU_REDUCE):
        mg.run(ex)
        assert oracle.scaled_error(r, c, h[2], h[3], ref, mg.y(ex)) <= TOL[np.dtype(dtype)]
        assert mg.y_device_ptr(ex) != 0
    mg.run(spmv_hw.MGPU_ALLGATHER)
    y1 = mg.y(spmv_hw.MGPU_ALLGATHER)
    assert oracle.scaled_error(r, c, h[2], h[3], ref, y1) <= TOL[np.dtype(dtype)]
    mg.destroy()
    plan.destroy()


def test_mgpu_rank_mode_rejects_a_foreign_plan():
    lib = spmv_hw.load(np.float64)
    n = 10_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 160_000, seed=4)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    uid = spmv_hw.mgpu_unique_id(lib)
    with pytest.raises(RuntimeError, match="not this rank's slice"):
        spmv_hw.MultiGpu.rank(lib, 0, 1, uid, 0, [0, n - 1], n, plan)
    plan.destroy()


@pytest.mark.parametrize("form", ["on_stream", "whole_device"])
def test_mgpu_set_x_device_waits_for_the_producer(form):
    """x written on a side stream behind a long GPU sleep: the copy into the clique's x must wait
    for it (the handle's streams are non-blocking). `on_stream` orders it after the
    producer stream by an event, `whole_device` (the C call without a stream) after everything
    queued on the device."""
    import ctypes
    import torch
    lib = spmv_hw.load(np.float64)
    n, z = 200_000, 3_200_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    mg = spmv_hw.MultiGpu.rank(lib, 0, 1, spmv_hw.mgpu_unique_id(lib), 0, [0, n], n, plan)
    xs = torch.full_like(x, float("nan"))
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)  # ~0.1 s of GPU time before x lands
        xs.copy_(x)
    if form == "on_stream":
        mg.set_x_device(xs, stream=side)
    else:
        lib._ok(lib.L.spmv_mgpu_set_x_device(mg.h, ctypes.c_void_p(xs.data_ptr())), "spmv_mgpu_set_x_device")
    mg.run(spmv_hw.MGPU_GATHER)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    y = mg.y(spmv_hw.MGPU_GATHER)
    assert np.isfinite(y).all()
    assert oracle.scaled_error(r, c, h[2], h[3], ref, y) <= 1e-12
    mg.destroy()
    plan.destroy()


@pytest.mark.parametrize("exchange", [spmv_hw.MGPU_GATHER, spmv_hw.MGPU_REDUCE])
@pytest.mark.parametrize("steps", [1, 4, 5])
def test_mgpu_run_pipelined(exchange, steps):
    """spmv_mgpu_run_pipelined: `steps` SpMVs whose exchanges overlap the next SpMV's kernels
    (double-buffered y; an even step count leaves the result in the second buffer, which is then
    copied into rank 0's y: its device address does not change). The result equals the oracle and
    a plain run afterwards still works."""
    lib = spmv_hw.load(np.float64)
    n, z = 300_000, 4_800_000
    rp, col, val, x = _powerlaw_host(lib, n, z)
    mg = spmv_hw.MultiGpu(lib, lib.make_csr_matrix(rp, col, val, n), ndev=_ndev())
    mg.set_x(x)
    ref = oracle.spmv_gold(rp, col, val, x)
    p0 = mg.y_device_ptr(exchange)
    ms = mg.run_pipelined(exchange, steps)
    assert ms > 0
    assert mg.y_device_ptr(exchange) == p0
    assert oracle.scaled_error(rp, col, val, x, ref, mg.y(exchange)) <= 1e-12
    mg.run(exchange)
    assert oracle.scaled_error(rp, col, val, x, ref, mg.y(exchange)) <= 1e-12
    with pytest.raises(RuntimeError, match="gather or reduce"):
        mg.run_pipelined(spmv_hw.MGPU_ALLGATHER, 2)
    mg.destroy()


@pytest.mark.parametrize("iters", [1, 2, 3])
def test_mgpu_run_graph(iters):
    """spmv_mgpu_run_graph: kernels + RCCL exchange captured into one hipGraph and replayed (one
    device per handle: the one-process-per-GPU form). The all-gather iterates x <- A x, so after
    `iters` steps x = A^iters x0; odd counts swap the buffers, which re-captures on the next call.
    Gather and reduce repeat y = A x. Checked against the oracle applied step by step."""
    import torch
    lib = spmv_hw.load(np.float64)
    n, z = 200_000, 3_200_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    mg = spmv_hw.MultiGpu.rank(lib, 0, 1, spmv_hw.mgpu_unique_id(lib), 0, [0, n], n, plan)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref1 = oracle.spmv_gold(r, c, h[2], h[3])
    for ex in (spmv_hw.MGPU_GATHER, spmv_hw.MGPU_REDUCE):
        mg.set_x_device(x)
        for _ in range(2):  # capture, then replay
            assert mg.run_graph(ex, iters) > 0
            assert oracle.scaled_error(r, c, h[2], h[3], ref1, mg.y(ex)) <= 1e-12
    for rep in range(2):  # second round: re-captured (odd) or replayed (even) from A^iters x0
        if rep == 0:
            mg.set_x_device(x)
            xs = h[3]
        mg.run_graph(spmv_hw.MGPU_ALLGATHER, iters)
        ref = xs
        for _ in range(iters):
            prev = ref
            ref = oracle.spmv_gold(r, c, h[2], prev)
        got = mg.y(spmv_hw.MGPU_ALLGATHER)
        assert oracle.scaled_error(r, c, h[2], prev, ref, got) <= 1e-12
        xs = got
    torch.cuda.synchronize()
    mg.destroy()
    plan.destroy()


@pytest.mark.parametrize("exchange", [spmv_hw.MGPU_GATHER, spmv_hw.MGPU_REDUCE])
def test_mgpu_graph_after_pipelined_sees_new_x(exchange):
    """a graph captured before an even-step pipelined run must still write the y that
    spmv_mgpu_get_y / _y_device read. graph(x1) -> pipelined(2 steps) -> x2 -> graph (replayed,
    same x buffer): y = A x2, at the address y_device gave before."""
    import torch
    lib = spmv_hw.load(np.float64)
    n, z = 200_000, 3_200_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x1 = spmv_hw.gen_vector(lib, n, seed=6)
    x2 = spmv_hw.gen_vector(lib, n, seed=7, lo=-1.0)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    mg = spmv_hw.MultiGpu.rank(lib, 0, 1, spmv_hw.mgpu_unique_id(lib), 0, [0, n], n, plan)
    h = [t.cpu().numpy() for t in (rp, col, val, x1, x2)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    mg.set_x_device(x1)
    p0 = mg.y_device_ptr(exchange)
    mg.run_graph(exchange, 2)
    mg.run_pipelined(exchange, 2)
    mg.set_x_device(x2)
    mg.run_graph(exchange, 2)
    assert mg.y_device_ptr(exchange) == p0
    ref2 = oracle.spmv_gold(r, c, h[2], h[4])
    assert oracle.scaled_error(r, c, h[2], h[4], ref2, mg.y(exchange)) <= 1e-12
    torch.cuda.synchronize()
    mg.destroy()
    plan.destroy()


def test_mgpu_set_x_device_rejects_x_on_another_device():
    """the producer event is recorded on rank 0's device, so x must live there."""
    import torch
    if _ndev() < 2:
        pytest.skip("needs a second GPU")
    lib = spmv_hw.load(np.float64)
    n = 10_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 160_000, seed=4)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    mg = spmv_hw.MultiGpu.rank(lib, 0, 1, spmv_hw.mgpu_unique_id(lib), 0, [0, n], n, plan)
    x = torch.ones(n, dtype=torch.float64, device="cuda:1")
    with pytest.raises(ValueError, match="rank 0 of this handle"):
        mg.set_x_device(x)
    mg.destroy()
    plan.destroy()
