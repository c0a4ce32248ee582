"""Parity at BASELINE.json's full sizes, through the automatically chosen
kernel, against the CPU oracle's restatement of spmv_gold (csr.cpp:184-194):

  config 2: banded 1,000,000 x 1,000,000, 16 nnz/row, fp64        -> flagged tiles (kernel 0)
  config 3: power-law 10M x 10M, 160M nnz, fp64                   -> panel sweep (kernel 2)
  config 5: the config-3 matrix in fp32                            -> two-pass binned (kernel 6)

Componentwise-scaled error max_i |dy_i| / (|A||x|)_i <= 1e-6 (fp64) / 1e-4 (fp32), the
north_star tolerance; fp64 is also held to 1e-12, fp32 to 2e-6 against oracle.spmv_fp64acc. The matrices are the bench's (same generator,
seeds and sizes); every row of y is poisoned with NaN before the run."""
import numpy as np
import pytest

import oracle
import spmv_hw

pytestmark = pytest.mark.gpu

TOL = {np.dtype(np.float64): 1e-6, np.dtype(np.float32): 1e-4}
FP32_TIGHT = 2e-6  # fp32 y against oracle.spmv_fp64acc (fp32 products, fp64 sums)


def _run(lib, rp, col, val, x, n, expect_kernel):
    import torch
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    st = plan.stats()
    assert st["kernel"] == expect_kernel, st
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    plan.destroy()
    h_rp = rp.cpu().numpy().view(np.uint32)
    h_col = col.cpu().numpy().view(np.uint32)
    h_val, h_x, h_y = val.cpu().numpy(), x.cpu().numpy(), y.cpu().numpy()
    del y
    torch.cuda.empty_cache()
    assert not np.isnan(h_y).any(), "a row was not written"
    ref = oracle.spmv_gold(h_rp, h_col, h_val, h_x)
    err = oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, h_y)
    if h_val.dtype == np.float32:
        # the fp32 kernels accumulate in fp64, so against spmv_gold's products
        # summed in fp64 (oracle.spmv_fp64acc) their error is reassociation plus, for the sweep,
        # the unrounded product: a tight bound that the 1e-4 gate beside it cannot see
        ref64 = oracle.spmv_fp64acc(h_rp, h_col, h_val, h_x)
        err64 = oracle.scaled_error(h_rp, h_col, h_val, h_x, ref64, h_y)
        assert err64 <= FP32_TIGHT, err64
    return err, st


@pytest.mark.timeout(600)
def test_config2_banded_1m_x16_fp64_auto_tiles():
    lib = spmv_hw.load(np.float64)
    n = 1_000_000
    rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    x = spmv_hw.gen_vector(lib, n, seed=3)
    err, st = _run(lib, rp, col, val, x, n, expect_kernel=0)
    assert st["nr_nzeros"] == 16 * n
    assert err <= 1e-12, err


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=["config3_fp64", "config5_fp32"])
def test_config3_and_5_powerlaw_10m_160m_auto(dtype):
    lib = spmv_hw.load(dtype)
    n, z = 10_000_000, 160_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    err, st = _run(lib, rp, col, val, x, n, expect_kernel=2 if np.dtype(dtype) == np.float64 else 6)
    assert st["nr_nzeros"] == z and st["nr_rows"] == n
    assert err <= TOL[np.dtype(dtype)], err
    if np.dtype(dtype) == np.float64:
        assert err <= 1e-12, err


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_config3_and_5_binned_forced(monkeypatch, dtype):
    """The binned kernel (kernel 6) on the headline matrix in both precisions (fp64 forced: the
    automatic choice keeps the sweep there)."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "binned")
    lib = spmv_hw.load(dtype)
    n, z = 10_000_000, 160_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    err, st = _run(lib, rp, col, val, x, n, expect_kernel=6)
    assert st["format"] & 32  # dense segments: the 1-byte row-delta form is chosen
    assert err <= (1e-12 if np.dtype(dtype) == np.float64 else 1e-4), err


@pytest.mark.timeout(600)
def test_config3_deterministic_sweep_bitwise_over_runs(monkeypatch):
    """SPMV_SWEEP_DETERMINISTIC=1 on the headline matrix: ten runs and a second plan give the
    same bits (adds in a fixed (iteration, wave, lane) order, k_spmv_sweep_turn), within the
    fp64 tolerance of the oracle, and within 1e-13 of the default (timing-order) sweep."""
    import torch
    lib = spmv_hw.load(np.float64)
    n, z = 10_000_000, 160_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    monkeypatch.setenv("SPMV_SWEEP_DETERMINISTIC", "1")
    plans = [spmv_hw.Plan.from_device(lib, rp, col, val, n) for _ in range(2)]
    monkeypatch.delenv("SPMV_SWEEP_DETERMINISTIC")
    fast = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    y0 = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plans[0].run(x, y0)
    y = torch.empty_like(y0)
    for k in range(10):
        y.fill_(float("nan"))
        plans[k % 2].run(x, y)
        assert torch.equal(y.view(torch.int64), y0.view(torch.int64)), f"run {k} differs"
    fast.run(x, y)
    torch.cuda.synchronize()
    rel = float(((y - y0).abs().max() / y0.abs().max()).item())
    assert rel < 1e-13, rel
    for p in plans + [fast]:
        p.destroy()
    h_rp = rp.cpu().numpy().view(np.uint32)
    h_col = col.cpu().numpy().view(np.uint32)
    h_val, h_x, h_y = val.cpu().numpy(), x.cpu().numpy(), y0.cpu().numpy()
    ref = oracle.spmv_gold(h_rp, h_col, h_val, h_x)
    assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, h_y) <= 1e-12


@pytest.mark.timeout(900)
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_config4_through_the_dropin_with_8_units(monkeypatch, dtype):
    """Config 4 the reference's own way: the 10M/160M matrix through Part 1 (create_csr_hw_matrix
    / spmv_hw, csr_hw_wrapper.cpp:3-80, :193-288) with 8 units ("ComputeUnits", here virtual
    units sharing the box's GPU), each holding its nnz-balanced row slice (csr_hw.cpp:459-468, the
    cut bench.py --gpus 8 makes), and the host merge of the slices into the caller's y
    (accum_results' +=, csr_hw.cpp:1531-1565). y matches spmv_gold of the whole matrix, the
    reference's verification (abs 1e-5) passes, a second call adds A x once more, and every
    unit's slice is the 8-way strong-scaling cut."""
    monkeypatch.setenv("SPMV_NGPUS", "8")
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    lib = spmv_hw.load(dtype)
    n, z = 10_000_000, 160_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    h_rp, h_col = rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32)
    h_val, h_x = val.cpu().numpy(), x.cpu().numpy()
    del rp, col, val, x
    m = lib.make_csr_matrix(h_rp, h_col, h_val, n)
    hw, bm = lib.create_csr_hw_matrix(m)
    bounds = lib.partition_rows(h_rp, 8)
    for u in range(8):  # the units' slices: the strong-scaling cut, row for row (every row is
        # non-empty here, so the compact row count is the slice's); nr_nzeros counts the stored,
        # chunk-padded entries of the unit's representation
        assert hw[u].contents.nr_rows[0] == bounds[u + 1] - bounds[u]
        z_u = int(h_rp[bounds[u + 1]]) - int(h_rp[bounds[u]])
        assert z_u <= hw[u].contents.nr_nzeros[0] <= 1.01 * z_u
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(h_x), 1, hw[0].contents.nr_cols)
    yv = lib.make_csr_vector(np.zeros(n, dtype))
    lib.spmv_hw(hw, hx, yv, bm)
    y1 = np.ctypeslib.as_array(yv.values, shape=(n,)).copy()
    lib.spmv_hw(hw, hx, yv, bm)
    y2 = np.ctypeslib.as_array(yv.values, shape=(n,)).copy()
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)
    ref = oracle.spmv_gold(h_rp, h_col, h_val, h_x)
    if np.dtype(dtype) == np.float64:
        assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, y1) <= 1e-12
        assert lib.verification(ref, y1) == 0
        assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, y2 - y1) <= 1e-12
    else:  # fp32: the north-star gate against spmv_gold, the tight bound against fp64 sums
        assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, y1) <= TOL[np.dtype(np.float32)]
        ref64 = oracle.spmv_fp64acc(h_rp, h_col, h_val, h_x)
        assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref64, y1) <= FP32_TIGHT
        # the second call's y is y1 + A x rounded in fp32 (the += happens in fp32 on the host)
        assert oracle.scaled_error(h_rp, h_col, h_val, h_x, 2 * ref64.astype(np.float64),
                                   y2.astype(np.float64)) <= 4 * FP32_TIGHT
