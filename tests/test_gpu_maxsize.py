"""Maximum sizes: slices with more than 2^31 non-zeros (the reference's 32-bit `int` entry
counters, csr_hw.cpp:377-429, overflow there; here row_ptr/col are uint32 and every layout
indexes entries in 64 bits or declines the matrix).

The oracle cannot run 2.2e9 non-zeros in seconds, so parity at this size is checked by
size-independent properties:
  * a weighted checksum  sum_i w_i y_i  ==  sum_k val_k x[col_k] w[row_k]  (computed in fp64 by
    torch in row chunks), tolerance 1e-12 * sum |.| — one lost or doubled row of this matrix
    moves it by ~1e-9 relative;
  * y starts as NaN, so an unwritten row poisons the checksum;
  * the oracle (spmv_gold) on a sample of rows: the first and last rows, the rows around the
    entry index 2^31 and 500 random rows, each with the scaled-error bound of test_gpu_parity.
Layouts that cannot hold such a slice (the sweep: hipcub item counts are int) refuse it with
an error when forced, and the automatic choice falls back to the tiles.
"""
import numpy as np
import pytest

import oracle
import spmv_hw

pytestmark = pytest.mark.gpu

TOL = {np.dtype(np.float64): 1e-12, np.dtype(np.float32): 2e-6}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def _u32(t):
    return t.long() & 0xFFFFFFFF


def _sample_rows(rp64, n, rng):
    # rows whose entries straddle index 2^31 (and the row just before/after)
    k = int(np.searchsorted(rp64.cpu().numpy(), 1 << 31, side="right")) - 1
    rows = {0, 1, 2, n - 3, n - 2, n - 1} | {r for r in range(k - 2, k + 3) if 0 <= r < n}
    rows |= set(rng.integers(0, n, 500).tolist())
    return np.array(sorted(rows), np.int64)


def _check_sample(torch, rp64, col, val, x, y, rows, dtype, tol=None):
    """spmv_gold on the sampled rows, columns remapped into a compact x."""
    b = rp64[torch.from_numpy(rows).cuda()].cpu().numpy()
    e = rp64[torch.from_numpy(rows + 1).cuda()].cpu().numpy()
    idx = torch.cat([torch.arange(int(s), int(t), device="cuda") for s, t in zip(b, e)])
    c = _u32(col[idx]).cpu().numpy()
    v = val[idx].cpu().numpy()
    uc, inv = np.unique(c, return_inverse=True)
    xs = x[torch.from_numpy(uc.astype(np.int64)).cuda()].cpu().numpy()
    sub_rp = np.zeros(len(rows) + 1, np.uint32)
    sub_rp[1:] = np.cumsum(e - b)
    sub_col = inv.astype(np.uint32)
    ref = oracle.spmv_gold(sub_rp, sub_col, v, xs)
    got = y[torch.from_numpy(rows).cuda()].cpu().numpy()
    assert not np.any(np.isnan(got)), "a sampled row was not written"
    err = oracle.scaled_error(sub_rp, sub_col, v, xs, ref, got)
    assert err <= (tol if tol is not None else TOL[np.dtype(dtype)]), err


def _checksum(torch, rp64, col, val, x, y, n, chunk_rows, tol=1e-12):
    w = torch.rand(n, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(7))
    lhs = float((w * y.double()).sum())
    s = a = 0.0
    for r0 in range(0, n, chunk_rows):
        r1 = min(n, r0 + chunk_rows)
        e0, e1 = int(rp64[r0]), int(rp64[r1])
        lens = rp64[r0 + 1:r1 + 1] - rp64[r0:r1]
        rows = torch.repeat_interleave(torch.arange(r0, r1, device="cuda"), lens)
        prod = val[e0:e1].double() * x[col[e0:e1].long()].double() * w[rows]
        s += float(prod.sum())
        a += float(prod.abs().sum())
        del lens, rows, prod
    assert np.isfinite(lhs), "y holds NaN: a row was not written"
    # |sum_i w_i (y_i - exact_i)| <= tol * sum_i w_i (|A||x|)_i for a per-row scaled error <= tol
    assert abs(lhs - s) <= tol * a, (lhs, s, a)


def _run(torch, lib, rp, col, val, x, n, ncols):
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, ncols)
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    st = plan.stats()
    plan.destroy()
    return y, st


@pytest.fixture(scope="module")
def banded64(torch):
    lib = spmv_hw.load(np.float64)
    n = 140_000_000  # 2.24e9 non-zeros
    rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    x = spmv_hw.gen_vector(lib, n, seed=3)
    rp64 = _u32(rp)
    assert int(rp64[-1]) == n * 16 > (1 << 31)
    yield lib, rp, col, val, x, rp64, n
    del rp, col, val, x, rp64
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kern,want", [("auto", 0), ("slices", 5), ("gold", 1)])
def test_banded_above_2_31_nonzeros(torch, monkeypatch, banded64, kern, want):
    lib, rp, col, val, x, rp64, n = banded64
    if kern != "auto":
        monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    y, st = _run(torch, lib, rp, col, val, x, n, n)
    assert st["kernel"] == want
    _check_sample(torch, rp64, col, val, x, y, _sample_rows(rp64, n, np.random.default_rng(1)), np.float64)
    _checksum(torch, rp64, col, val, x, y, n, 16_000_000)
    del y
    torch.cuda.empty_cache()


def test_sweep_above_2_31_nonzeros(torch, monkeypatch, banded64):
    """the sweep's radix sort takes a 64-bit item count, so a slice past 2^31
    entries stays on the sweep (kernel 2)."""
    lib, rp, col, val, x, rp64, n = banded64
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    y, st = _run(torch, lib, rp, col, val, x, n, n)
    assert st["kernel"] == 2
    _check_sample(torch, rp64, col, val, x, y, _sample_rows(rp64, n, np.random.default_rng(4)), np.float64)
    _checksum(torch, rp64, col, val, x, y, n, 16_000_000)
    del y
    torch.cuda.empty_cache()


def test_powerlaw_above_2_31_nonzeros_stays_on_the_sweep(torch):
    """A 20M-row power-law slice with 2.2e9 non-zeros: x of 160 MB and random columns, so the
    automatic choice is the panel sweep (kernel 2), whose build now sorts 2.2e9 entries."""
    lib = spmv_hw.load(np.float64)
    n, z = 20_000_000, 2_200_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    rp64 = _u32(rp)
    assert int(rp64[-1]) == z
    y, st = _run(torch, lib, rp, col, val, x, n, n)
    assert st["kernel"] == 2
    _check_sample(torch, rp64, col, val, x, y, _sample_rows(rp64, n, np.random.default_rng(2)), np.float64)
    _checksum(torch, rp64, col, val, x, y, n, 2_000_000)
    del rp, col, val, x, rp64, y
    torch.cuda.empty_cache()


def test_powerlaw_fp32_above_2_31_nonzeros_binned(torch):
    """The same 20M-row slice in fp32: the automatic choice is the two-pass binned kernel
    (kernel 6), whose segment offsets and pass-1 units are 64-bit."""
    lib = spmv_hw.load(np.float32)
    n, z = 20_000_000, 2_200_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    rp64 = _u32(rp)
    assert int(rp64[-1]) == z
    y, st = _run(torch, lib, rp, col, val, x, n, n)
    assert st["kernel"] == 6
    # against spmv_gold's own fp32 running sum over rows of ~110 (up to thousands of) entries:
    # the north_star fp32 tolerance; the checksum below holds y to the exact sums at 2e-6
    _check_sample(torch, rp64, col, val, x, y, _sample_rows(rp64, n, np.random.default_rng(5)), np.float32, tol=1e-4)
    _checksum(torch, rp64, col, val, x, y, n, 2_000_000, tol=TOL[np.dtype(np.float32)])
    del rp, col, val, x, rp64, y
    torch.cuda.empty_cache()


def test_banded_fp32_above_2_31_nonzeros(torch):
    lib = spmv_hw.load(np.float32)
    n = 140_000_000
    rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    x = spmv_hw.gen_vector(lib, n, seed=3)
    rp64 = _u32(rp)
    y, st = _run(torch, lib, rp, col, val, x, n, n)
    assert st["kernel"] in (0, 5)
    _check_sample(torch, rp64, col, val, x, y, _sample_rows(rp64, n, np.random.default_rng(3)), np.float32)
    _checksum(torch, rp64, col, val, x, y, n, 16_000_000, tol=TOL[np.dtype(np.float32)])
    del rp, col, val, x, rp64, y
    torch.cuda.empty_cache()
