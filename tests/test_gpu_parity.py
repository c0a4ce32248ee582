"""Parity of the MI355X HIP path (through the C-ABI) with the CPU oracle.

Tolerances (BASELINE.json north_star): componentwise-scaled error max_i |dy_i| / (|A||x|)_i
<= 1e-6 for fp64 and <= 1e-4 for fp32. The HIP kernels add in a different order than spmv_gold
(segmented wave scan, tile partials), so results are not bitwise equal to the oracle; fp64 is
additionally held to 1e-12, which any wrong row or lost partial would exceed by many orders.
"""
import os
import sys

import numpy as np
import pytest

import oracle
import spmv_hw
from conftest import DTYPES, FIXTURES, GOLDEN, golden_arrays, manifest, tools_env

pytestmark = pytest.mark.gpu

TOL = {np.dtype(np.float64): 1e-6, np.dtype(np.float32): 1e-4}
TIGHT = {np.dtype(np.float64): 1e-12, np.dtype(np.float32): 2e-6}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


KERNELS = ["tiles", "tiles_wide", "sweep", "sweep_rc", "sweep_unpacked", "sweep_det", "gold", "blocked", "slices", "slices_wide",
           "binned", "binned_delta", "binned_u16"]
KERNEL_ID = {"tiles": 0, "tiles_wide": 0, "sweep": 2, "sweep_rc": 2, "sweep_unpacked": 2, "sweep_det": 2, "gold": 1, "blocked": 4,
             "slices": 5, "slices_wide": 5, "binned": 6, "binned_delta": 6, "binned_u16": 6}


@pytest.fixture(params=KERNELS)
def kernel(request, monkeypatch):
    """Plans are built with SPMV_HW_KERNEL forced to each kernel in turn ("blocked" with its
    defaults VF = 1, 32768-column blocks); "tiles_wide" is the
    tile kernel with 32-bit columns (SPMV_TILE_NARROW=0) instead of per-tile offsets and
    "sweep_rc" the packed sweep on its 12-byte words without delta-coded columns
    (SPMV_SWEEP_DELTA=0); "sweep_unpacked" the sweep on 14-byte entries (SPMV_SWEEP_PACKED=0), the layout used when a
    chunk of a panel spans >= 65536 columns; "sweep_det" the deterministic sweep
    (SPMV_SWEEP_DETERMINISTIC=1); "slices_wide" the slice kernel with 32-bit columns
    (SPMV_SLICE_NARROW=0); "binned" the two-pass propagation-blocking kernel (binned.hip) with its
    automatic row-offset form, "binned_delta" / "binned_u16" with 1-byte deltas / u16 offsets
    forced (SPMV_BIN_DELTA=1 / 0)."""
    monkeypatch.setenv("SPMV_HW_KERNEL", request.param.split("_")[0])
    if request.param == "tiles_wide":
        tools_env(monkeypatch, "SPMV_TILE_NARROW", "0")
    if request.param == "sweep_unpacked":
        tools_env(monkeypatch, "SPMV_SWEEP_PACKED", "0")
    if request.param == "sweep_rc":  # packed 12-byte words without the delta-coded columns
        monkeypatch.setenv("SPMV_SWEEP_DELTA", "0")
    if request.param == "sweep_det":  # deterministic sweep: LDS adds in a fixed (iteration, wave) order
        monkeypatch.setenv("SPMV_SWEEP_DETERMINISTIC", "1")
    if request.param == "slices_wide":
        tools_env(monkeypatch, "SPMV_SLICE_NARROW", "0")
    if request.param == "binned_delta":  # row-sorted segments with 1-byte deltas, escapes and all
        tools_env(monkeypatch, "SPMV_BIN_DELTA", "1")
    if request.param == "binned_u16":  # u16 row offsets
        tools_env(monkeypatch, "SPMV_BIN_DELTA", "0")
    return request.param


def to_dev(torch, a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a).cuda()


def run_device(torch, lib, row_ptr, col, val, x, nr_cols, poison=True, expect_kernel=None):
    plan = spmv_hw.Plan.from_device(lib, to_dev(torch, row_ptr), to_dev(torch, col if len(col) else np.zeros(1, np.uint32)),
                                    to_dev(torch, val if len(val) else np.zeros(1, lib.dtype)), nr_cols)
    n = len(row_ptr) - 1
    y = torch.full((max(n, 1),), float("nan") if poison else 0.0, dtype=spmv_hw._torch_dtype(lib.dtype), device="cuda")
    plan.run(to_dev(torch, x if len(x) else np.zeros(1, lib.dtype)), y)
    torch.cuda.synchronize()
    out = y.cpu().numpy()[:n]
    stats = plan.stats()
    plan.destroy()
    if expect_kernel is not None:
        assert stats["kernel"] == KERNEL_ID[expect_kernel]
        if expect_kernel == "tiles_wide":
            assert not stats["format"] & 1
        if expect_kernel == "sweep_unpacked":
            assert not stats["format"] & 2
        if expect_kernel == "sweep_rc":
            assert not stats["format"] & 64
        if expect_kernel in ("binned_delta", "binned_u16"):
            assert bool(stats["format"] & 32) == (expect_kernel == "binned_delta")
    return out, stats


def check(row_ptr, col, val, x, y_ref, y, dtype):
    assert not np.any(np.isnan(y) & ~np.isnan(y_ref)), "a row was not written"
    err = oracle.scaled_error(row_ptr, col, val, x, y_ref, y)
    assert err <= TOL[np.dtype(dtype)], err
    assert err <= TIGHT[np.dtype(dtype)], err
    return err


def random_csr(rng, n, m, lens, dtype):
    lens = np.asarray(lens, np.int64)
    row_ptr = np.zeros(n + 1, np.int64)
    row_ptr[1:] = np.cumsum(lens)
    z = int(row_ptr[-1])
    col = np.empty(z, np.uint32)
    for i in range(n):
        k = int(lens[i])
        if k:
            col[row_ptr[i]:row_ptr[i + 1]] = np.sort(rng.choice(m, size=min(k, m), replace=k > m))
    val = rng.uniform(-1, 1, size=z).astype(dtype)
    x = rng.uniform(0, 1, size=m).astype(dtype)
    return row_ptr.astype(np.uint32), col, val, x


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
def test_golden_fixtures_device_plan(torch, kernel, name, dtype, tag):
    lib = spmv_hw.load(dtype)
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    _, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
    x, y_gold = golden_arrays(name, tag)
    y, _ = run_device(torch, lib, row_ptr, col, val, x, c, expect_kernel=kernel)
    check(row_ptr, col, val, x, y_gold, y, dtype)
    if kernel.startswith("slices") and np.dtype(dtype) == np.float64:
        _bitwise(y, y_gold)  # kernel 5 in fp64: spmv_gold's arithmetic, bit for bit


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
@pytest.mark.parametrize("units", [1, 2, 3])
def test_reference_api_flow(torch, monkeypatch, kernel, name, dtype, tag, units):
    """main.cpp:46-97 through the drop-in API: create_csr_hw_matrix -> create_csr_hw_x_vector ->
    spmv_hw (accumulates into a zeroed y_fpga) -> verification -> delete_*; units = virtual
    "Compute Units" sharing the one GPU of the box."""
    monkeypatch.setenv("SPMV_NGPUS", str(units))
    lib = spmv_hw.load(dtype)
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    r, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
    x, y_gold = golden_arrays(name, tag)
    m = lib.make_csr_matrix(row_ptr, col, val, c)
    hw_matrix, bitmap = lib.create_csr_hw_matrix(m)
    assert hw_matrix[0].contents.blocks == 1
    assert hw_matrix[0].contents.nr_cols[0] == c
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), hw_matrix[0].contents.blocks,
                                    hw_matrix[0].contents.nr_cols)
    y_fpga = np.zeros(r, dtype)
    yv = lib.make_csr_vector(y_fpga)
    lib.spmv_hw(hw_matrix, hx, yv, bitmap)
    y = np.ctypeslib.as_array(yv.values, shape=(r,)).copy()
    check(row_ptr, col, val, x, y_gold, y, dtype)
    if dtype == np.float64:
        assert lib.verification(y_gold, y) == 0
    # bitmap[0][row] == row is empty (csr_hw.cpp:340-347)
    empty = np.diff(row_ptr.astype(np.int64)) == 0
    assert np.array_equal(np.ctypeslib.as_array(bitmap[0], shape=(r,)), empty)
    total_mb = sum(lib.storage_overhead(hw_matrix[u]) for u in range(units))
    assert total_mb > 0
    # spmv_hw accumulates (+=): the second call adds another A*x on top of the first
    lib.spmv_hw(hw_matrix, hx, yv, bitmap)
    y2 = np.ctypeslib.as_array(yv.values, shape=(r,)).astype(np.float64)
    second = y2 - y.astype(np.float64)
    assert oracle.scaled_error(row_ptr, col, val, x, y.astype(np.float64), second) <= (1e-5 if dtype == np.float32 else 1e-12)
    lib.delete_csr_hw_matrix(hw_matrix)
    lib.free_bitmap(bitmap)
    lib.delete_csr_hw_x_vector(hx)


def test_two_matrices_with_different_unit_counts_coexist(torch, monkeypatch):
    """Each hw_matrix array knows its own unit count (null-terminated), so matrices created
    under different SPMV_NGPUS can be used and deleted in any order; create_csr_hw_y_vector
    follows the matrix it is given."""
    lib = spmv_hw.load(np.float64)
    mats = []
    for units, name in ((3, "small"), (1, "longrow")):
        monkeypatch.setenv("SPMV_NGPUS", str(units))
        path = os.path.join(GOLDEN, manifest()[name]["file"])
        r, c, row_ptr, col, val, _ = oracle.read_csr(path, np.float64)
        x, y_gold = golden_arrays(name, "f64")
        m = lib.make_csr_matrix(row_ptr, col, val, c)
        hw, bm = lib.create_csr_hw_matrix(m)
        hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), 1, hw[0].contents.nr_cols)
        mats.append((units, r, hw, bm, hx, y_gold, m))
    for units, r, hw, bm, hx, y_gold, _ in mats[::-1]:
        count = 0
        while hw[count]:  # the array ends with a null entry
            count += 1
        assert count == units
        hy = lib.create_csr_hw_y_vector(hw)
        lib.delete_csr_hw_y_vector(hy)
        yv = lib.make_csr_vector(np.zeros(r))
        lib.spmv_hw(hw, hx, yv, bm)
        y = np.ctypeslib.as_array(yv.values, shape=(r,))
        assert lib.verification(y_gold, y.copy()) == 0
    for _, _, hw, bm, hx, _, _ in mats:
        lib.delete_csr_hw_matrix(hw)
        lib.free_bitmap(bm)
        lib.delete_csr_hw_x_vector(hx)


EDGE_CASES = {
    # name: (n, m, lengths-builder)
    "tile_aligned_rows": (64, 4096, lambda rng: np.full(64, 512)),
    "one_entry": (1, 1, lambda rng: np.array([1])),
    "nnz_511": (7, 300, lambda rng: np.array([100, 100, 100, 100, 100, 11, 0])),
    "nnz_513": (3, 600, lambda rng: np.array([0, 513, 0])),
    "long_row_100k": (5, 200_000, lambda rng: np.array([3, 100_000, 0, 7, 1])),
    "mostly_empty": (5000, 5000, lambda rng: (rng.random(5000) < 0.02) * rng.integers(1, 40, 5000)),
    "leading_empty": (1000, 1000, lambda rng: np.r_[np.zeros(600, int), rng.integers(1, 9, 400)]),
    "all_empty": (100, 100, lambda rng: np.zeros(100, int)),
    "mixed_powerlaw": (20000, 20000, lambda rng: np.minimum(np.floor(8 * rng.random(20000) ** -0.5), 5000)),
    "rows_ending_at_lane_edges": (512, 2048, lambda rng: np.tile([4, 3, 1, 8, 16, 64, 128, 32], 64)),
}


def _structured(kind, dtype):
    """Structured shapes with explicit columns: an arrow matrix (dense first row, dense first
    column, diagonal), block-diagonal dense 64x64 blocks, one dense column, an upper bidiagonal
    band with a far corner entry per row (two clusters per slot)."""
    rng = np.random.default_rng(sum(map(ord, kind)))
    n = 3000
    rows = []
    if kind == "arrow":
        rows = [np.arange(n)] + [np.unique([0, i]) for i in range(1, n)]
    elif kind == "block_diagonal":
        rows = [np.arange(i // 64 * 64, min(n, i // 64 * 64 + 64)) for i in range(n)]
    elif kind == "dense_column":
        rows = [np.unique([7, i]) for i in range(n)]
    elif kind == "band_plus_corner":
        rows = [np.unique([i, min(i + 1, n - 1), (i * 7919) % n + 200_000]) for i in range(n)]
    m = int(max(r.max() for r in rows)) + 1
    lens = np.array([len(r) for r in rows])
    row_ptr = np.zeros(n + 1, np.int64)
    row_ptr[1:] = np.cumsum(lens)
    col = np.concatenate(rows).astype(np.uint32)
    val = rng.uniform(-1, 1, len(col)).astype(dtype)
    x = rng.uniform(0, 1, m).astype(dtype)
    return row_ptr.astype(np.uint32), col, val, x, m


@pytest.mark.parametrize("kind", ["arrow", "block_diagonal", "dense_column", "band_plus_corner"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_structured_shapes(torch, kernel, kind, dtype):
    row_ptr, col, val, x, m = _structured(kind, dtype)
    lib = spmv_hw.load(dtype)
    y, _ = run_device(torch, lib, row_ptr, col, val, x, m, expect_kernel=kernel)
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), y, dtype)


@pytest.mark.parametrize("case", sorted(EDGE_CASES))
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_edge_cases(torch, kernel, case, dtype):
    rng = np.random.default_rng(sum(map(ord, case)))
    n, m, lens_fn = EDGE_CASES[case]
    row_ptr, col, val, x = random_csr(rng, n, m, lens_fn(rng), dtype)
    lib = spmv_hw.load(dtype)
    y_ref = oracle.spmv_gold(row_ptr, col, val, x)
    y, st = run_device(torch, lib, row_ptr, col, val, x, m, expect_kernel=kernel)
    check(row_ptr, col, val, x, y_ref, y, dtype)
    assert st["nr_nzeros"] == row_ptr[-1]
    assert st["nr_nonempty_rows"] == int((np.diff(row_ptr.astype(np.int64)) > 0).sum())


def test_nan_in_unused_x_does_not_leak(torch, kernel):
    """Padding entries use column 0; a non-finite x[0] must not reach any row that does not
    reference column 0 (SURVEY B-edge: padded FPGA entries read x[0] too)."""
    rng = np.random.default_rng(7)
    n, m = 300, 1000
    row_ptr, col, val, x = random_csr(rng, n, m, rng.integers(1, 9, n), np.float64)
    col[col == 0] = 1
    x[0] = np.nan
    y, _ = run_device(torch, spmv_hw.load(np.float64), row_ptr, col, val, x, m)
    assert not np.any(np.isnan(y))


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_nonfinite_x_propagates_like_spmv_gold(torch, kernel, dtype):
    """NaN, +inf and -inf in used columns of x, and explicit zero values on inf columns (0 * inf
    = NaN): whether a row ends NaN, +inf, -inf or finite does not depend on the summation order,
    so every kernel's rows must match spmv_gold's class exactly (csr.cpp:184-194), and the
    finite rows stay within the tolerance."""
    rng = np.random.default_rng(23)
    n, m = 5_000, 40_000
    row_ptr, col, val, x = random_csr(rng, n, m, rng.integers(0, 30, n), dtype)
    special = rng.choice(m, 60, replace=False)
    x[special[:20]] = np.nan
    x[special[20:40]] = np.inf
    x[special[40:]] = -np.inf
    hits_inf = np.isin(col, special[20:]) & (rng.random(len(col)) < 0.3)
    val[hits_inf] = 0  # 0 * inf = NaN in that row
    ref = oracle.spmv_gold(row_ptr, col, val, x)
    y, _ = run_device(torch, spmv_hw.load(dtype), row_ptr, col, val, x, m)
    assert np.isnan(ref).sum() > 10 and np.isinf(ref).sum() > 10  # the case exercises all classes
    assert np.array_equal(np.isnan(y), np.isnan(ref))
    assert np.array_equal(np.isposinf(y), np.isposinf(ref)) and np.array_equal(np.isneginf(y), np.isneginf(ref))
    fin = np.isfinite(ref)
    keep = np.repeat(fin, np.diff(row_ptr.astype(np.int64)))  # entries of the finite rows
    sub_rp = np.zeros(int(fin.sum()) + 1, np.int64)
    sub_rp[1:] = np.cumsum(np.diff(row_ptr.astype(np.int64))[fin])
    xf = np.where(np.isfinite(x), x, 0).astype(dtype)  # finite rows use no non-finite x
    check(sub_rp.astype(np.uint32), col[keep], val[keep], xf, ref[fin], y[fin], dtype)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("shape", ["wide", "tall"])
def test_extreme_aspect_ratios(torch, kernel, shape, dtype):
    """wide: 1,000 rows over 10M columns (x of 80 MB, ~200 scattered entries a row: many column
    windows / blocks, few rows); tall: 1M rows over 64 columns (x in one cache line or two)."""
    rng = np.random.default_rng(29)
    if shape == "wide":
        n, m, k = 1_000, 10_000_000, 200
    else:
        n, m, k = 1_000_000, 64, 4
    cols = np.sort(rng.integers(0, m, (n, k)), axis=1).astype(np.uint32).ravel()
    row_ptr = (np.arange(n + 1, dtype=np.int64) * k).astype(np.uint32)
    val = rng.uniform(-1, 1, n * k).astype(dtype)
    x = rng.uniform(0, 1, m).astype(dtype)
    y, _ = run_device(torch, spmv_hw.load(dtype), row_ptr, cols, val, x, m, expect_kernel=kernel)
    check(row_ptr, cols, val, x, oracle.spmv_gold(row_ptr, cols, val, x), y, dtype)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_unaligned_x_and_y(torch, kernel, dtype):
    """x and y given as views one element into their buffers (not 16-byte aligned): kernels
    that stage x with 16-byte loads (the binned kernel's pass 1) take their element-wise path."""
    rng = np.random.default_rng(17)
    n, m = 20_000, 70_000
    row_ptr, col, val, x = random_csr(rng, n, m, rng.integers(0, 40, n), dtype)
    lib = spmv_hw.load(dtype)
    plan = spmv_hw.Plan.from_device(lib, to_dev(torch, row_ptr), to_dev(torch, col), to_dev(torch, val), m)
    xb = to_dev(torch, np.concatenate([np.zeros(1, dtype), x]))
    yb = torch.full((n + 1,), float("nan"), dtype=xb.dtype, device="cuda")
    plan.run(xb[1:], yb[1:])
    torch.cuda.synchronize()
    plan.destroy()
    y = yb.cpu().numpy()
    assert np.isnan(y[0]), "wrote before y"
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), y[1:], dtype)


def test_out_of_range_column_is_rejected(torch, kernel):
    lib = spmv_hw.load(np.float64)
    row_ptr = np.array([0, 2], np.uint32)
    col = np.array([0, 5], np.uint32)
    with pytest.raises(RuntimeError, match="out of range"):
        spmv_hw.Plan.from_device(lib, to_dev(torch, row_ptr), to_dev(torch, col),
                                 to_dev(torch, np.ones(2)), 5)


def test_malformed_row_ptr_and_variant_are_rejected(torch, kernel):
    lib = spmv_hw.load(np.float64)
    row_ptr = np.array([0, 3, 2, 4], np.uint32)  # decreasing at row 1
    col = np.array([0, 1, 2, 3], np.uint32)
    with pytest.raises(RuntimeError, match="non-decreasing"):
        spmv_hw.Plan.from_device(lib, to_dev(torch, row_ptr), to_dev(torch, col), to_dev(torch, np.ones(4)), 4)
    plan = spmv_hw.Plan.from_device(lib, to_dev(torch, np.array([0, 2, 4], np.uint32)), to_dev(torch, col),
                                    to_dev(torch, np.ones(4)), 4)
    with pytest.raises(RuntimeError, match="bad arguments"):
        plan.set_variant(64)
    with pytest.raises(RuntimeError, match="iters"):
        plan.run_graph(to_dev(torch, np.ones(4)), torch.empty(2, dtype=torch.float64, device="cuda"), 0)
    plan.destroy()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_deterministic(torch, kernel, dtype):
    """The tile kernel is bitwise reproducible (partials added in a fixed order). The sweep kernel
    adds into LDS with atomics, so only rounding-level run-to-run differences are allowed."""
    rng = np.random.default_rng(3)
    row_ptr, col, val, x = random_csr(rng, 30000, 30000, np.minimum(np.floor(8 * rng.random(30000) ** -0.5), 3000), dtype)
    lib = spmv_hw.load(dtype)
    y1, _ = run_device(torch, lib, row_ptr, col, val, x, 30000)
    y2, _ = run_device(torch, lib, row_ptr, col, val, x, 30000)
    if kernel.startswith("tiles") or kernel.startswith("slices") or kernel in ("gold", "blocked"):
        assert np.array_equal(y1.view(np.uint8), y2.view(np.uint8))
    else:
        assert oracle.scaled_error(row_ptr, col, val, x, y1, y2) <= TIGHT[np.dtype(dtype)]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_synthetic_banded_vs_oracle(torch, kernel, dtype):
    lib = spmv_hw.load(dtype)
    n = 200_000
    rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    x = spmv_hw.gen_vector(lib, n, seed=3)
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    plan.run(x, y)
    torch.cuda.synchronize()
    h = [t.cpu().numpy() for t in (rp, col, val, x, y)]
    row_ptr, c, v, xx, yy = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3], h[4]
    assert np.all(np.diff(row_ptr.astype(np.int64)) == 16)
    check(row_ptr, c, v, xx, oracle.spmv_gold(row_ptr, c, v, xx), yy, dtype)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_synthetic_powerlaw_vs_oracle(torch, kernel, dtype):
    """Config-3 shape scaled to 1M rows / 16M nnz (same generator, same tail)."""
    lib = spmv_hw.load(dtype)
    n, z = 1_000_000, 16_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    plan.run(x, y)
    torch.cuda.synchronize()
    row_ptr = rp.cpu().numpy().view(np.uint32)
    c, v, xx, yy = col.cpu().numpy().view(np.uint32), val.cpu().numpy(), x.cpu().numpy(), y.cpu().numpy()
    assert row_ptr[-1] == z and c.max() < n
    lens = np.diff(row_ptr.astype(np.int64))
    inner = ~np.isin(np.arange(1, z), row_ptr)  # pairs (k-1, k) inside one row
    assert np.all(np.diff(c.astype(np.int64))[inner] > 0), "columns must strictly increase within rows"
    assert lens.max() > 1000
    check(row_ptr, c, v, xx, oracle.spmv_gold(row_ptr, c, v, xx), yy, dtype)


def test_row_slices_match_whole_matrix(torch, kernel):
    """Plans over nnz-balanced row slices (the multi-unit path) concatenate to the full y."""
    lib = spmv_hw.load(np.float64)
    rng = np.random.default_rng(11)
    n = 50_000
    row_ptr, col, val, x = random_csr(rng, n, n, np.minimum(np.floor(8 * rng.random(n) ** -0.5), 4000), np.float64)
    y_ref = oracle.spmv_gold(row_ptr, col, val, x)
    for units in (2, 4, 8):
        b = lib.partition_rows(row_ptr, units)
        parts = []
        for u in range(units):
            r0, r1 = int(b[u]), int(b[u + 1])
            rp = row_ptr[r0:r1 + 1]
            y, _ = run_device(torch, lib, (rp - rp[0]).astype(np.uint32), col[rp[0]:rp[-1]], val[rp[0]:rp[-1]], x, n)
            parts.append(y)
        check(row_ptr, col, val, x, y_ref, np.concatenate(parts), np.float64)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_narrow_tiles_bitwise_equal_to_wide(torch, monkeypatch, dtype):
    """8- and 16-bit per-tile column offsets change the bytes streamed, not the arithmetic: all
    three tile representations give bitwise identical y."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "tiles")
    lib = spmv_hw.load(dtype, ablations=True)
    n = 300_000
    rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    x = spmv_hw.gen_vector(lib, n, seed=3)
    ys, fmts, nbytes = [], [], []
    for narrow in ("", "16", "0"):
        tools_env(monkeypatch, "SPMV_TILE_NARROW", narrow)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
        y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        torch.cuda.synchronize()
        st = plan.stats()
        fmts.append(st["format"] & 9)
        nbytes.append(st["device_bytes"])
        ys.append(y.cpu().numpy())
        plan.destroy()
    assert fmts == [9, 1, 0]  # banded tiles span < 256 columns: 8-bit by default
    z = 16 * n
    assert nbytes[2] - nbytes[1] >= 2 * z - 4 * (z // 512 + 1)  # 2 B/nnz saved
    assert nbytes[1] - nbytes[0] == z + (-z) % 512                  # 1 more B/nnz
    for y in ys[1:]:
        assert np.array_equal(ys[0].view(np.uint8), y.view(np.uint8))


@pytest.mark.parametrize("span,narrow", [(255, 9), (256, 1), (65535, 1), (65536, 0)])
def test_narrow_tiles_span_limit(torch, monkeypatch, span, narrow):
    """The widest tile decides the plan's column width: span < 256 -> 8-bit offsets,
    < 65536 -> 16-bit, else 32-bit columns."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "tiles")
    monkeypatch.delenv("SPMV_TILE_NARROW", raising=False)
    tools_env(monkeypatch, "SPMV_TILE_CLUSTER", "0")  # the plain narrow limits (clusters: below)
    lib = spmv_hw.load(np.float64)
    m = 70_000
    rng = np.random.default_rng(5)
    n = 40
    lens = np.full(n, 20)
    lens[0] = 2
    row_ptr, col, val, x = random_csr(rng, n, span - 8, lens, np.float64)
    col += 8                      # every other column in [8, span)
    col[0], col[1] = 7, 7 + span  # row 0 spans exactly `span` columns
    x = rng.uniform(0, 1, size=m)
    y, st = run_device(torch, lib, row_ptr, col, val, x, m, expect_kernel="tiles")
    assert st["format"] & 9 == narrow
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), y, np.float64)


PACKED_VARIANTS = [15, 20, 22, 26, 27, 28, 29, 30, 31, 32, 33, 34]
UNPACKED_VARIANTS = [0, 1, 3, 7, 15, 20, 22]


@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_variants_agree(torch, monkeypatch, packed, dtype):
    """Every sweep variant (barrier / loose-sync forms, group counts) computes the same y."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    tools_env(monkeypatch, "SPMV_SWEEP_PACKED", "1" if packed else "0")
    lib = spmv_hw.load(dtype)
    n, z = 200_000, 3_200_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    assert bool(plan.stats()["format"] & 2) == packed
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_gold(row_ptr, c, v, xx)
    y = torch.empty(n, dtype=x.dtype, device="cuda")
    for var in (PACKED_VARIANTS if packed else UNPACKED_VARIANTS):
        y.fill_(float("nan"))
        plan.set_variant(var)
        plan.run(x, y)
        torch.cuda.synchronize()
        check(row_ptr, c, v, xx, ref, y.cpu().numpy(), dtype)
    plan.destroy()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_wide_chunks_ride_in_the_side_table(torch, monkeypatch, dtype):
    """A run of 49K empty rows at the top makes the first panels a few entries spread over the
    columns: their 128-entry chunks span >= 65536 columns, which 16-bit offsets cannot hold. Those chunks
    (well under 1 in 10) keep their absolute columns in the delta plan's side table (format bit
    12) and the rest of the plan keeps the 11-byte entries. y is the oracle's; a variant that
    needs the 12-byte entries is refused on such a plan."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    rng = np.random.default_rng(21)
    n = 6_000_000
    lens = rng.poisson(16, n)
    lens[rng.random(n) < 0.2] = 0
    lens[1000:50_000] = 0  # the first panels hold a few entries over ~20K rows each
    row_ptr = np.zeros(n + 1, np.int64)
    row_ptr[1:] = np.cumsum(lens)
    z = int(row_ptr[-1])
    row_ptr = row_ptr.astype(np.uint32)
    col = rng.integers(0, n, z, dtype=np.uint32)  # (unsorted within a row: CSR allows it)
    val = rng.uniform(-1, 1, z).astype(dtype)
    x = rng.uniform(0, 1, n).astype(dtype)
    lib = spmv_hw.load(dtype)
    y, st = run_device(torch, lib, row_ptr, col, val, x, n, expect_kernel="sweep")
    assert st["format"] & 2 and st["format"] & 64 and st["format"] & 4096, st
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), y, dtype)
    plan = spmv_hw.Plan.from_device(lib, to_dev(torch, row_ptr), to_dev(torch, col), to_dev(torch, val), n)
    with pytest.raises(RuntimeError, match="wide chunks"):
        plan.set_variant(94)
    plan.destroy()


def test_sweep_falls_back_to_unpacked_entries_on_sparse_panels(torch, monkeypatch):
    """A panel too sparse for 16-bit column offsets inside a 128-entry chunk (here 16K entries
    per panel over 10M columns: a chunk spans ~80K columns) keeps the 14-byte entries."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    monkeypatch.delenv("SPMV_SWEEP_PACKED", raising=False)
    tools_env(monkeypatch, "SPMV_SWEEP_SPLIT", "0")  # 256 small panels, not 13 full ones in pieces
    lib = spmv_hw.load(np.float64)
    n, m = 256_000, 10_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, 16 * n, seed=4)
    x = spmv_hw.gen_vector(lib, m, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
    assert plan.stats()["format"] & 2 == 0
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    h = [t.cpu().numpy() for t in (rp, col, val, x, y)]
    row_ptr, c, v, xx, yy = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3], h[4]
    check(row_ptr, c, v, xx, oracle.spmv_gold(row_ptr, c, v, xx), yy, np.float64)
    plan.destroy()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_split_pieces_match_oracle(torch, monkeypatch, dtype):
    """A strong-scaling-like slice (few rows, wide x): full-size panels cut into column pieces
    whose fp64 partial sums k_sweep_combine adds per row; also the same plan forced unsplit."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    lib = spmv_hw.load(dtype, ablations=True)
    n_full, z_full = 10_000_000, 160_000_000
    r0, r1 = 0, 1_250_000  # rank 0 of 8 (row slice of the 10M/160M matrix, rows only)
    ys = {}
    for split in ("1", "0"):
        tools_env(monkeypatch, "SPMV_SWEEP_SPLIT", split)
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n_full, n_full, z_full, seed=4, row_begin=r0, row_end=r1)
        x = spmv_hw.gen_vector(lib, n_full, seed=6)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n_full)
        st = plan.stats()
        y = torch.full((r1 - r0,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        plan.run(x, y)  # every run overwrites y: no accumulation across calls
        torch.cuda.synchronize()
        ys[split] = (st["nr_tiles"], y.cpu().numpy())
        plan.destroy()
    assert ys["1"][0] < 256 and ys["0"][0] == 256  # pieces of ~62 full panels vs 256 small ones
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_gold(row_ptr, c, v, xx)
    for split, (_, y) in ys.items():
        check(row_ptr, c, v, xx, ref, y, dtype)


def test_sweep_fused_combine_bitwise_equals_combine_kernel(torch, monkeypatch):
    """The split sweep's combine done by the last piece of each panel (SPMV_SWEEP_COMBINE=fused)
    adds the pieces' partials in the same piece order as the separate k_sweep_combine launch
    (the default): with the deterministic sweep (fixed partials) the two give the
    same bits, on every run of a plan (the per-panel counters re-arm), also with 8 pieces per
    panel (two rounds of workgroups, SPMV_SWEEP_PIECES=8); and y matches the oracle."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    monkeypatch.setenv("SPMV_SWEEP_DETERMINISTIC", "1")
    lib = spmv_hw.load(np.float64, ablations=True)
    n_full, z_full = 10_000_000, 160_000_000
    r0, r1 = 1_250_000, 2_500_000  # rank 1 of 8
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n_full, n_full, z_full, seed=4, row_begin=r0, row_end=r1)
    x = spmv_hw.gen_vector(lib, n_full, seed=6)
    ys = {}
    for combine, pieces in (("fused", ""), ("kernel", ""), ("fused", "8"), ("kernel", "8")):
        tools_env(monkeypatch, "SPMV_SWEEP_COMBINE", combine)
        if pieces:
            tools_env(monkeypatch, "SPMV_SWEEP_PIECES", pieces)
        else:
            monkeypatch.delenv("SPMV_SWEEP_PIECES", raising=False)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n_full)
        st = plan.stats()
        assert st["nr_tiles"] > 100 and st["tile_nnz"] > 0
        runs = []
        for _ in range(3):
            y = torch.full((r1 - r0,), float("nan"), dtype=x.dtype, device="cuda")
            plan.run(x, y)
            torch.cuda.synchronize()
            runs.append(y.cpu().numpy())
        plan.destroy()
        for r in runs[1:]:
            _bitwise(runs[0], r)
        ys[(combine, pieces)] = (st["nr_tiles"], runs[0])
    assert ys[("fused", "8")][0] == 2 * ys[("fused", "")][0]  # 8 pieces instead of 4 per panel
    _bitwise(ys[("fused", "")][1], ys[("kernel", "")][1])
    _bitwise(ys[("fused", "8")][1], ys[("kernel", "8")][1])
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_gold(row_ptr, c, v, xx)
    for _, y in ys.values():
        check(row_ptr, c, v, xx, ref, y, np.float64)
    # the default (non-deterministic) sweep with the fused combine, 4 and 8 pieces
    monkeypatch.delenv("SPMV_SWEEP_DETERMINISTIC")
    tools_env(monkeypatch, "SPMV_SWEEP_COMBINE", "fused")
    for pieces in ("", "8"):
        if pieces:
            tools_env(monkeypatch, "SPMV_SWEEP_PIECES", pieces)
        else:
            monkeypatch.delenv("SPMV_SWEEP_PIECES", raising=False)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n_full)
        for _ in range(3):
            y = torch.full((r1 - r0,), float("nan"), dtype=x.dtype, device="cuda")
            plan.run(x, y)
            torch.cuda.synchronize()
            check(row_ptr, c, v, xx, ref, y.cpu().numpy(), np.float64)
        plan.destroy()


# ---- gold order: bitwise the reference's spmv_gold (csr.cpp:184-194) ----
def _bitwise(a, b):
    assert a.dtype == b.dtype and a.shape == b.shape
    bad = np.nonzero(a.view(np.uint8).reshape(len(a), -1).any(axis=1) !=
                     b.view(np.uint8).reshape(len(b), -1).any(axis=1))[0]
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), f"first differing rows {bad[:5]}"


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
def test_gold_kernel_bitwise_equals_fixture(torch, monkeypatch, name, dtype, tag):
    monkeypatch.setenv("SPMV_HW_KERNEL", "gold")
    lib = spmv_hw.load(dtype)
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    _, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
    x, y_gold = golden_arrays(name, tag)
    y, st = run_device(torch, lib, row_ptr, col, val, x, c, expect_kernel="gold")
    _bitwise(y, y_gold)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("workload", ["powerlaw", "banded"])
def test_gold_kernel_bitwise_equals_oracle_synthetic(torch, monkeypatch, dtype, workload):
    """1M rows: power-law rows up to ~20K entries exercise the wave-per-long-row path."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "gold")
    lib = spmv_hw.load(dtype)
    n = 1_000_000
    if workload == "powerlaw":
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 16 * n, seed=4)
    else:
        rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    st = plan.stats()
    assert st["kernel"] == 1 and (st["nr_tiles"] > 0) == (workload == "powerlaw")  # long rows
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    h = [t.cpu().numpy() for t in (rp, col, val, x, y)]
    row_ptr, c, v, xx, yy = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3], h[4]
    _bitwise(yy, oracle.spmv_gold(row_ptr, c, v, xx))
    plan.destroy()


@pytest.mark.parametrize("units", [1, 3])
def test_gold_kernel_through_reference_api_is_bitwise(torch, monkeypatch, units):
    """main.cpp's flow with SPMV_HW_KERNEL=gold: y_fpga (zeroed, then +=) equals spmv_gold's y
    bit for bit, so the reference's own verification sees zero difference."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "gold")
    monkeypatch.setenv("SPMV_NGPUS", str(units))
    lib = spmv_hw.load(np.float64)
    for name in FIXTURES:
        path = os.path.join(GOLDEN, manifest()[name]["file"])
        n, c, row_ptr, col, val, _ = oracle.read_csr(path, np.float64)
        x, y_gold = golden_arrays(name, "f64")
        m = lib.make_csr_matrix(row_ptr, col, val, c)
        hw, bm = lib.create_csr_hw_matrix(m)
        hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), hw[0].contents.blocks, hw[0].contents.nr_cols)
        y_vec = lib.make_csr_vector(np.zeros(n))
        lib.spmv_hw(hw, hx, y_vec, bm)
        y = np.ctypeslib.as_array(y_vec.values, (n,)).copy()
        lib.delete_csr_hw_matrix(hw)
        lib.free_bitmap(bm)
        lib.delete_csr_hw_x_vector(hx)
        _bitwise(y, y_gold)


# ---- FPGA order: bitwise the reference hardware path's sums (spmv.cpp:66-104,
#      csr_hw.cpp:209-243 + 1543-1562) for a VF / column-block width ----
#      kernel 3 ("fpga": CSR, one in-order pass per row) and kernel 4 ("blocked": the reference's
#      dataflow, x blocks in LDS, per-block partials, block-ordered merge) ----
KERNEL_ID["fpga"] = 3
FPGA_KERNELS = ["fpga", "blocked"]


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
@pytest.mark.parametrize("vf", [1, 2, 4, 8])
@pytest.mark.parametrize("block", [32768, 700])
@pytest.mark.parametrize("kern", FPGA_KERNELS)
def test_fpga_order_bitwise_equals_oracle_fixture(torch, monkeypatch, name, dtype, tag, vf, block, kern):
    monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    monkeypatch.setenv("SPMV_FPGA_VF", str(vf))
    monkeypatch.setenv("SPMV_FPGA_BLOCK", str(block))
    lib = spmv_hw.load(dtype)
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    _, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
    x, y_gold = golden_arrays(name, tag)
    y, _ = run_device(torch, lib, row_ptr, col, val, x, c, expect_kernel=kern)
    _bitwise(y, oracle.spmv_fpga_order(row_ptr, col, val, x, c, block, vf))
    check(row_ptr, col, val, x, y_gold, y, dtype)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("vf,block", [(1, 32768), (4, 65536), (8, 4096), (2, 16384)])
@pytest.mark.parametrize("kern", FPGA_KERNELS)
def test_fpga_order_bitwise_synthetic(torch, monkeypatch, dtype, vf, block, kern):
    """1M-row power-law matrix (rows up to ~20K entries, many blocks per row). For the blocked
    kernel the x block sits in LDS when it fits 128 KiB (fp32 up to 32768 columns, fp64 up to
    16384) and is read from L2 otherwise: both forms are covered."""
    monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    monkeypatch.setenv("SPMV_FPGA_VF", str(vf))
    monkeypatch.setenv("SPMV_FPGA_BLOCK", str(block))
    lib = spmv_hw.load(dtype)
    n = 1_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 16 * n, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    assert plan.stats()["kernel"] == KERNEL_ID[kern]
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    h = [t.cpu().numpy() for t in (rp, col, val, x, y)]
    row_ptr, c, v, xx, yy = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3], h[4]
    _bitwise(yy, oracle.spmv_fpga_order(row_ptr, c, v, xx, n, block, vf))
    plan.run(x, y)  # partials are scratch: a second run gives the same y
    torch.cuda.synchronize()
    _bitwise(y.cpu().numpy(), oracle.spmv_fpga_order(row_ptr, c, v, xx, n, block, vf))
    plan.destroy()


@pytest.mark.parametrize("vf", [2, 8])
@pytest.mark.parametrize("kern", FPGA_KERNELS)
def test_fpga_order_unsorted_rows(torch, monkeypatch, vf, kern):
    """Rows whose columns are not ordered: the plan stably groups each row's entries by column
    block (as create_block_matrix visits them), keeping the CSR order within a block."""
    monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    monkeypatch.setenv("SPMV_FPGA_VF", str(vf))
    monkeypatch.setenv("SPMV_FPGA_BLOCK", "97")
    rng = np.random.default_rng(21)
    n, m = 5000, 1000
    row_ptr, col, val, x = random_csr(rng, n, m, rng.integers(0, 70, n), np.float64)
    for i in range(n):  # shuffle every row
        rng.shuffle(col[row_ptr[i]:row_ptr[i + 1]])
    lib = spmv_hw.load(np.float64)
    y, _ = run_device(torch, lib, row_ptr, col, val, x, m, expect_kernel=kern)
    _bitwise(y, oracle.spmv_fpga_order(row_ptr, col, val, x, m, 97, vf))


@pytest.mark.parametrize("kern", FPGA_KERNELS)
def test_fpga_order_env_errors(torch, monkeypatch, kern):
    monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    lib = spmv_hw.load(np.float64)
    row_ptr = np.array([0, 1], np.uint32)
    for var, bad in (("SPMV_FPGA_VF", "3"), ("SPMV_FPGA_BLOCK", "0")):
        with monkeypatch.context() as mp:
            mp.setenv(var, bad)
            with pytest.raises(RuntimeError, match=var):
                run_device(torch, lib, row_ptr, np.zeros(1, np.uint32), np.ones(1), np.ones(1), 1)


def test_blocked_rejects_blocks_wider_than_16_bit_offsets(torch, monkeypatch):
    monkeypatch.setenv("SPMV_HW_KERNEL", "blocked")
    monkeypatch.setenv("SPMV_FPGA_BLOCK", "65537")
    lib = spmv_hw.load(np.float64)
    row_ptr = np.array([0, 1], np.uint32)
    with pytest.raises(RuntimeError, match="16-bit"):
        run_device(torch, lib, row_ptr, np.zeros(1, np.uint32), np.ones(1), np.ones(1), 1)


@pytest.mark.parametrize("units", [1, 3])
@pytest.mark.parametrize("kern", FPGA_KERNELS)
def test_fpga_order_through_reference_api(torch, monkeypatch, units, kern):
    """main.cpp's flow (y_fpga zeroed, then spmv_hw) with SPMV_HW_KERNEL=fpga|blocked and the
    block width of read_csr_header: y equals the restated FPGA arithmetic bit for bit."""
    monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    monkeypatch.setenv("SPMV_FPGA_VF", "4")
    monkeypatch.setenv("SPMV_NGPUS", str(units))
    lib = spmv_hw.load(np.float64)
    for name in FIXTURES:
        path = os.path.join(GOLDEN, manifest()[name]["file"])
        n, c, row_ptr, col, val, _ = oracle.read_csr(path, np.float64)
        x, _ = golden_arrays(name, "f64")
        m = lib.make_csr_matrix(row_ptr, col, val, c)
        hw, bm = lib.create_csr_hw_matrix(m)
        hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), hw[0].contents.blocks, hw[0].contents.nr_cols)
        y_vec = lib.make_csr_vector(np.zeros(n))
        lib.spmv_hw(hw, hx, y_vec, bm)
        y = np.ctypeslib.as_array(y_vec.values, (n,)).copy()
        lib.delete_csr_hw_matrix(hw)
        lib.free_bitmap(bm)
        lib.delete_csr_hw_x_vector(hx)
        _bitwise(y, oracle.spmv_fpga_order(row_ptr, col, val, x, c, 32768, 4))


@pytest.mark.parametrize("kern", ["sweep", "tiles", "gold"])
def test_dense_rows_among_short_ones(torch, monkeypatch, kern):
    """Ragged extreme: two rows of 600K entries among 400K rows of ~16. The sweep cuts the
    panels holding them into pieces (more units than panels); the tiles carry them across
    ~1200 tiles each through the fix-up; gold gives them a wave each."""
    monkeypatch.setenv("SPMV_HW_KERNEL", kern)
    rng = np.random.default_rng(12)
    n, m = 400_000, 1_000_000
    lens = rng.poisson(16, n)
    dense = [77, 250_001]
    lens[dense] = 600_000
    row_ptr, col, val, x = random_csr(rng, n, m, lens, np.float64)
    lib = spmv_hw.load(np.float64)
    y, st = run_device(torch, lib, row_ptr, col, val, x, m, expect_kernel=kern)
    ref = oracle.spmv_gold(row_ptr, col, val, x)
    if kern == "gold":
        assert np.array_equal(y.view(np.uint8), ref.view(np.uint8))
    else:
        check(row_ptr, col, val, x, ref, y, np.float64)


@pytest.mark.parametrize("workload,want", [("powerlaw", (2,)), ("banded", (0, 5))])
def test_tune_mode_keeps_the_faster_layout(torch, monkeypatch, workload, want):
    """SPMV_HW_KERNEL=tune builds the tile, sweep and slice layouts, times them on the matrix and
    keeps the fastest: the sweep for scattered columns; for a band the tiles and the slices are
    within ~10 % of each other (profiles/), so either may win."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "tune")
    lib = spmv_hw.load(np.float64)
    n = 2_000_000
    if workload == "powerlaw":
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 16 * n, seed=4)
    else:
        rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    assert plan.stats()["kernel"] in want
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    h = [t.cpu().numpy() for t in (rp, col, val, x, y)]
    row_ptr, c, v, xx, yy = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3], h[4]
    check(row_ptr, c, v, xx, oracle.spmv_gold(row_ptr, c, v, xx), yy, np.float64)
    plan.destroy()


@pytest.mark.parametrize("workload", ["powerlaw", "banded"])
def test_tune_mode_is_reproducible(torch, monkeypatch, workload):
    """SPMV_HW_KERNEL=tune times every candidate with the median of 7
    graph-replayed samples and replaces the preferred layout (the automatic choice first) only
    when a later one is > 3 % faster, so two tuned builds of one matrix -- for the band, tiles
    and slices within ~10 % of each other -- give the same layout: identical spmv_plan_stats."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "tune")
    lib = spmv_hw.load(np.float64)
    n = 2_000_000
    if workload == "powerlaw":
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 16 * n, seed=4)
    else:
        rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
    stats = []
    for _ in range(2):
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
        stats.append(plan.stats())
        plan.destroy()
    assert stats[0] == stats[1], stats


def _clustered_rows(n, gaps):
    """Row i has columns i + g for g in gaps (sorted): len(gaps) far-apart column clusters per
    tile, like a 3-D stencil's grid planes."""
    row_ptr = (np.arange(n + 1) * len(gaps)).astype(np.uint32)
    col = (np.arange(n)[:, None] + np.array(gaps)[None, :]).reshape(-1).astype(np.uint32)
    return row_ptr, col


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("gaps,clustered", [((0, 100_000, 200_000), True),
                                            ((0, 70_000, 140_000, 210_000), True),
                                            ((0, 50_000, 100_000, 150_000, 200_000), False)])
def test_clustered_tile_columns(torch, monkeypatch, dtype, gaps, clustered):
    """Tiles whose columns fall into <= 4 narrow clusters store 16-bit (cluster, offset)
    columns; bitwise the same y as 32-bit columns; 5 clusters keep 32-bit columns."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "tiles")
    monkeypatch.delenv("SPMV_TILE_NARROW", raising=False)
    rng = np.random.default_rng(21)
    n = 60_000
    row_ptr, col = _clustered_rows(n, gaps)
    m = int(col.max()) + 1
    val = rng.uniform(-1, 1, len(col)).astype(dtype)
    x = rng.uniform(0, 1, m).astype(dtype)
    lib = spmv_hw.load(dtype, ablations=True)
    outs = {}
    for mode in ("1", "0"):
        tools_env(monkeypatch, "SPMV_TILE_CLUSTER", mode)
        y, st = run_device(torch, lib, row_ptr, col, val, x, m, expect_kernel="tiles")
        outs[mode] = (y, st["format"])
    assert bool(outs["1"][1] & 16) == clustered and not outs["0"][1] & 16
    assert np.array_equal(outs["1"][0].view(np.uint8), outs["0"][0].view(np.uint8))
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), outs["1"][0], dtype)


def test_auto_kernel_choice(torch, monkeypatch):
    """Automatic choice: banded (local columns, 8-bit spans) -> tiles; 3-D stencils (rows of equal
    length, 16-bit slot spans) -> slices; power-law with columns spread over an x much larger
    than the L2s -> sweep (fp32 from 80M non-zeros: binned)."""
    monkeypatch.delenv("SPMV_HW_KERNEL", raising=False)
    lib = spmv_hw.load(np.float64)
    n = 6_000_000
    rp, col, val = spmv_hw.gen_banded(lib, n, 16)
    assert spmv_hw.Plan.from_device(lib, rp, col, val, n).stats()["kernel"] == 0
    del rp, col, val
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 16 * n)
    assert spmv_hw.Plan.from_device(lib, rp, col, val, n).stats()["kernel"] == 2
    del rp, col, val
    # around the measured crossover: x of 2.4 MB -> sweep, x of 0.8 MB -> tiles
    for n, want in ((300_000, 2), (100_000, 0)):
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 16 * n)
        assert spmv_hw.Plan.from_device(lib, rp, col, val, n).stats()["kernel"] == want, n
    # fp32: the two-pass binned kernel once the matrix is large (>= 80M non-zeros, >= 5M columns)
    lib32 = spmv_hw.load(np.float32)
    for n, want in ((6_000_000, 6), (4_000_000, 2)):
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib32, n, n, 16 * n)
        assert spmv_hw.Plan.from_device(lib32, rp, col, val, n).stats()["kernel"] == want, n
        if want == 6:  # fixed bits requested: the turn-ordered sweep, not the binned kernel
            monkeypatch.setenv("SPMV_SWEEP_DETERMINISTIC", "1")
            assert spmv_hw.Plan.from_device(lib32, rp, col, val, n).stats()["kernel"] == 2
            monkeypatch.delenv("SPMV_SWEEP_DETERMINISTIC")
        del rp, col, val
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from ab_variants import stencil
    for points in (7, 27):
        rp, col, val, n = stencil(60 ** 3, points, np.float64)
        assert spmv_hw.Plan.from_device(lib, rp, col, val, n).stats()["kernel"] == 5, points


def test_auto_binned_skips_skewed_fp32(torch, monkeypatch):
    """fp32 with x of 6M columns would take the binned kernel, but one row of 2M entries makes
    its panel 2x+ the mean: pass 2 would serialise that row's LDS adds on one address (2.6 vs
    0.42 ms, tools/skew_probe.py), so the automatic choice keeps the sweep, which cuts such
    panels into pieces. Forced, the binned kernel still gives the right y."""
    monkeypatch.delenv("SPMV_HW_KERNEL", raising=False)
    lib = spmv_hw.load(np.float32)
    n, m, z, dense = 1_200_000, 6_000_000, 19_200_000, 2_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, z, seed=9)
    dcol = torch.arange(0, 3 * dense, 3, dtype=torch.int32, device="cuda")
    rp = torch.cat([rp, (rp[-1:].long() + dense).int()])
    col = torch.cat([col[:z], dcol])
    val = torch.cat([val[:z], torch.full((dense,), 0.5, dtype=val.dtype, device="cuda")])
    x = spmv_hw.gen_vector(lib, m, seed=6)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_gold(row_ptr, c, v, xx)
    ref64 = oracle.spmv_fp64acc(row_ptr, c, v, xx)
    for forced, want in ((None, 2), ("binned", 6)):
        if forced:
            monkeypatch.setenv("SPMV_HW_KERNEL", forced)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
        assert plan.stats()["kernel"] == want
        y = torch.full((n + 1,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        torch.cuda.synchronize()
        plan.destroy()
        # against spmv_gold's own fp32 running sum over the 2M-entry row: the north_star
        # tolerance (the fp64-accumulating kernels are the more accurate side here) ...
        yy = y.cpu().numpy()
        assert not np.isnan(yy).any()
        assert oracle.scaled_error(row_ptr, c, v, xx, ref, yy) <= TOL[np.dtype(np.float32)]
        # ... and tight against the same products summed in fp64, which is
        # what both kernels compute up to reassociation
        assert oracle.scaled_error(row_ptr, c, v, xx, ref64, yy) <= 2e-6


@pytest.mark.parametrize("ratio,limit,want", [(0.4, None, 2), (0.4, "1", 6), (0.15, None, 6)])
def test_auto_binned_row_limit(torch, monkeypatch, ratio, limit, want):
    """balanced panels let a row of up to ~2x the mean panel entries through the panel
    test, and pass 2 adds all of it into one LDS address. The automatic choice also checks the
    longest row against 0.3x the mean panel entries (profiles/r03e_skew_rowlimit.jsonl): a row of
    0.4x keeps the sweep, 0.15x keeps the binned kernel; SPMV_BIN_ROW_LIMIT=1 lifts the row test
    (the panel test still holds). y matches the oracle either way."""
    monkeypatch.delenv("SPMV_HW_KERNEL", raising=False)
    if limit:
        monkeypatch.setenv("SPMV_BIN_ROW_LIMIT", limit)
    else:
        monkeypatch.delenv("SPMV_BIN_ROW_LIMIT", raising=False)
    lib = spmv_hw.load(np.float32)
    n, m, z = 2_000_000, 6_000_000, 32_000_000
    panels = 256  # 2M rows: one round of the CUs, ~125K entries per panel
    long_len = int(ratio * (z / panels))
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, z, seed=11)
    dcol = torch.arange(0, 5 * long_len, 5, dtype=torch.int32, device="cuda")
    rp = torch.cat([rp, (rp[-1:].long() + long_len).int()])
    col = torch.cat([col[:z], dcol])
    val = torch.cat([val[:z], torch.full((long_len,), 0.25, dtype=val.dtype, device="cuda")])
    x = spmv_hw.gen_vector(lib, m, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
    assert plan.stats()["kernel"] == want
    y = torch.full((n + 1,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    plan.destroy()
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref64 = oracle.spmv_fp64acc(row_ptr, c, v, xx)
    assert oracle.scaled_error(row_ptr, c, v, xx, ref64, y.cpu().numpy()) <= 2e-6


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("points", [7, 27])
def test_slices_stencil_narrow_equals_wide(torch, monkeypatch, dtype, points):
    """3-D stencil matrix through the slice kernel: narrow slot offsets give bitwise the same y
    as 32-bit columns, and both match the oracle."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from ab_variants import stencil
    rp, col, val, n = stencil(40 ** 3, points, dtype)
    lib = spmv_hw.load(dtype, ablations=True)
    x = spmv_hw.gen_vector(lib, n, seed=3)
    ys = []
    for narrow in ("1", "0"):
        monkeypatch.setenv("SPMV_HW_KERNEL", "slices")
        tools_env(monkeypatch, "SPMV_SLICE_NARROW", narrow)
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
        st = plan.stats()
        assert st["kernel"] == 5 and bool(st["format"] & 1) == (narrow == "1")
        y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        torch.cuda.synchronize()
        ys.append(y.cpu().numpy())
        plan.destroy()
    assert np.array_equal(ys[0].view(np.uint8), ys[1].view(np.uint8))
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    y_gold = oracle.spmv_gold(row_ptr, c, v, xx)
    check(row_ptr, c, v, xx, y_gold, ys[0], dtype)
    if dtype == np.float64:  # CSR order from +0.0, separate mul/add: spmv_gold bit for bit
        _bitwise(ys[0], y_gold)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_slices_clustered_offsets(torch, monkeypatch, dtype):
    """Slots whose columns span >= 65536 but fall into <= 4 clusters of < 16384 (here: the second
    entry of even rows lies 100000 columns right, of odd rows 200000) use clustered 16-bit
    offsets; a slot with 5 clusters forces 32-bit columns. Both bitwise equal 32-bit columns."""
    n, m = 100_000, 400_000
    r = np.arange(n, dtype=np.int64)
    for far, clustered in ((lambda r: 100_000 + (r % 2) * 100_000, True),
                           (lambda r: 20_000 * (r % 5) + 100_000, False)):
        cols = np.stack([r, r + far(r)], axis=1).astype(np.uint32).ravel()
        row_ptr = (2 * np.arange(n + 1)).astype(np.uint32)
        rng = np.random.default_rng(5)
        val = rng.uniform(-1, 1, 2 * n).astype(dtype)
        x = rng.uniform(0, 1, m).astype(dtype)
        lib = spmv_hw.load(dtype, ablations=True)
        ys = []
        for narrow in ("1", "0"):
            monkeypatch.setenv("SPMV_HW_KERNEL", "slices")
            tools_env(monkeypatch, "SPMV_SLICE_NARROW", narrow)
            y, st = run_device(torch, lib, row_ptr, cols, val, x, m, expect_kernel="slices")
            assert bool(st["format"] & 16) == (narrow == "1" and clustered)
            ys.append(y)
        assert np.array_equal(ys[0].view(np.uint8), ys[1].view(np.uint8))
        check(row_ptr, cols, val, x, oracle.spmv_gold(row_ptr, cols, val, x), ys[0], dtype)


@pytest.mark.parametrize("units", [1, 3])
@pytest.mark.parametrize("prefault", ["1", "0"])
def test_spmv_hw_adds_into_nonzero_y_fpga(torch, monkeypatch, units, prefault):
    """spmv_hw is `y_fpga += A x` (csr_hw.cpp:1555): on a 600K-row matrix (the threaded
    accumulation, with and without mapping y's pages first, SPMV_HW_PREFAULT) a y_fpga holding
    nonzero values gets exactly y0 + (A x) — the same device sums added on the host — and
    the rows past the matrix (y_fpga longer than the matrix) are not touched."""
    monkeypatch.setenv("SPMV_NGPUS", str(units))
    monkeypatch.setenv("SPMV_HW_PREFAULT", prefault)
    lib = spmv_hw.load(np.float64)
    rng = np.random.default_rng(5)
    n, w = 600_000, 16
    rp = (np.arange(n + 1, dtype=np.int64) * w).astype(np.uint32)
    start = np.clip(np.arange(n) - w // 2, 0, n - w)
    col = (start[:, None] + np.arange(w)[None, :]).ravel().astype(np.uint32)
    val = rng.uniform(-1, 1, n * w)
    x = rng.uniform(0, 1, n)
    m = lib.make_csr_matrix(rp, col, val, n)
    hw, bm = lib.create_csr_hw_matrix(m)
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), hw[0].contents.blocks, hw[0].contents.nr_cols)
    ya = lib.make_csr_vector(np.zeros(n))
    lib.spmv_hw(hw, hx, ya, bm)
    y_ax = np.ctypeslib.as_array(ya.values, (n,)).copy()
    y0 = rng.uniform(-10, 10, n + 1000)
    yv = lib.make_csr_vector(y0.copy())
    lib.spmv_hw(hw, hx, yv, bm)
    got = np.ctypeslib.as_array(yv.values, (n + 1000,))
    assert np.array_equal(got[:n], y0[:n] + y_ax)
    assert np.array_equal(got[n:], y0[n:])
    check(rp, col, val, x, oracle.spmv_gold(rp, col, val, x), y_ax, np.float64)
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("shape", ["powerlaw", "sparse_cols"])
def test_sweep_delta_columns(torch, monkeypatch, dtype, shape):
    """Delta-coded sweep columns (format bit 6: a u16 row word + a u8 per entry holding the row and
    a 9-bit column delta, a DPP prefix sum per wave instruction; chunks with a gap above 511 read
    absolute columns from the side table). The same plan run on its 12-byte words (variant 35)
    gives the same sums up to the LDS adds' order, and both match the oracle. "sparse_cols": 330K
    rows (256 panels of ~1,290 rows) over 2M columns, ~97 columns between a panel's consecutive
    entries, so about half the chunks hold a gap above 511 (side table) and half do not, and
    gaps of 256-511 (bit 8 of the delta) are common. The power-law matrix of 10M columns sorts on
    bucketed keys (shift 1), which the delta build re-sorts per chunk."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    monkeypatch.delenv("SPMV_SWEEP_DELTA", raising=False)
    lib = spmv_hw.load(dtype, ablations=True)  # variant 35 below: tools library
    if shape == "powerlaw":
        n, m, z = 2_000_000, 10_000_000, 32_000_000
    else:
        n, m, z = 330_000, 2_000_000, 5_280_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, z, seed=8)
    x = spmv_hw.gen_vector(lib, m, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
    st = plan.stats()
    assert st["kernel"] == 2 and st["format"] & 64 and st["format"] & 2
    ys = []
    for variant in (28, 35):  # 28: the default on the 11-byte entries, 35: on the 12-byte words
        plan.set_variant(variant)
        y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        torch.cuda.synchronize()
        ys.append(y.cpu().numpy())
    plan.destroy()
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_fp64acc(row_ptr, c, v, xx) if dtype == np.float32 else oracle.spmv_gold(row_ptr, c, v, xx)
    for y in ys:
        assert not np.isnan(y).any()
        assert oracle.scaled_error(row_ptr, c, v, xx, ref, y) <= TIGHT[np.dtype(dtype)]
    assert oracle.scaled_error(row_ptr, c, v, xx, ys[1].astype(np.float64), ys[0]) <= TIGHT[np.dtype(dtype)]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_delta_gap_edges(torch, monkeypatch, dtype):
    """Column gaps at the edges of the delta encoding, in one panel whose column-sorted entries
    form three chunks: chunk 0 cycles the gaps 0 (a repeated column), 1, 255, 256 and 511 (all
    encodable: bit 8 of the delta rides in the row word); chunk 1 is the same plus one gap of 512
    (the chunk reads the side table); chunk 2 has gaps of 256 and 511 only, ending in a partial
    chunk (pad entries). y matches the oracle on the 11-byte and the 12-byte entries alike."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    monkeypatch.delenv("SPMV_SWEEP_DELTA", raising=False)
    lib = spmv_hw.load(dtype, ablations=True)  # variant 35 below: tools library
    cyc = [0, 1, 255, 256, 511]
    gaps = [cyc[k % 5] for k in range(128)] + [cyc[k % 5] for k in range(127)] + [512] \
        + [(256, 511)[k % 2] for k in range(100)]
    cols = np.cumsum(np.array(gaps, np.int64)) + 7
    z = len(cols)
    n = 997
    rows = (np.arange(z) * 7919) % n
    order = np.lexsort((cols, rows))  # CSR: by row, then column
    rows, cols = rows[order], cols[order]
    row_ptr = np.zeros(n + 1, np.int64)
    np.add.at(row_ptr, rows + 1, 1)
    row_ptr = np.cumsum(row_ptr).astype(np.uint32)
    m = int(cols.max()) + 1
    rng = np.random.default_rng(3)
    val = rng.uniform(-1, 1, z).astype(dtype)
    x = rng.uniform(0, 1, m).astype(dtype)
    col = cols.astype(np.uint32)
    plan = spmv_hw.Plan.from_device(lib, to_dev(torch, row_ptr), to_dev(torch, col), to_dev(torch, val), m)
    st = plan.stats()
    assert st["kernel"] == 2 and st["format"] & 64, st
    ref = oracle.spmv_gold(row_ptr, col, val, x)
    xd = to_dev(torch, x)
    for variant in (28, 35):
        plan.set_variant(variant)
        y = torch.full((n,), float("nan"), dtype=xd.dtype, device="cuda")
        plan.run(xd, y)
        torch.cuda.synchronize()
        check(row_ptr, col, val, x, ref, y.cpu().numpy(), dtype)
    plan.destroy()


@pytest.mark.parametrize("setting", ["threads512", "threads256", "acc32"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_workgroup_and_accumulator_settings(torch, monkeypatch, dtype, setting):
    """The sweep's other product settings: SPMV_SWEEP_THREADS=512/256 (half / quarter-size panels
    per workgroup; packed chunks delta-coded, or the unpacked form when the smaller panels make
    chunk spans too wide) and, for fp32, SPMV_SWEEP_ACC=32 (an fp32 LDS accumulator through
    compare-and-swap, up to 40,895-row panels; delta-coded only while the panels stay below
    32,768 rows). y matches the oracle: fp64-accumulating settings within the tight bound of the
    fp64-accumulated reference, the fp32 accumulator within the north-star 1e-4 of spmv_gold."""
    if setting == "acc32" and dtype == np.float64:
        pytest.skip("SPMV_SWEEP_ACC=32 applies to fp32 matrices only")
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    if setting.startswith("threads"):
        tools_env(monkeypatch, "SPMV_SWEEP_THREADS", setting[7:])
    else:
        tools_env(monkeypatch, "SPMV_SWEEP_ACC", "32")
    lib = spmv_hw.load(dtype)
    n, m, z = 600_000, 3_000_000, 9_600_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, z, seed=12)
    x = spmv_hw.gen_vector(lib, m, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
    st = plan.stats()
    assert st["kernel"] == 2, st
    if st["format"] & 2 and st["nr_nonempty_rows"] and setting != "acc32":
        # packed chunks carry delta-coded columns (quarter-size panels of 256-thread workgroups
        # are sparse enough for chunk spans >= 65536, i.e. the unpacked 14-byte form)
        assert st["format"] & 64, st
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    plan.destroy()
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    yy = y.cpu().numpy()
    assert not np.isnan(yy).any()
    if setting == "acc32":
        ref = oracle.spmv_gold(row_ptr, c, v, xx)
        assert oracle.scaled_error(row_ptr, c, v, xx, ref, yy) <= TOL[np.dtype(dtype)]
    else:
        ref = oracle.spmv_fp64acc(row_ptr, c, v, xx) if dtype == np.float32 else oracle.spmv_gold(row_ptr, c, v, xx)
        assert oracle.scaled_error(row_ptr, c, v, xx, ref, yy) <= TIGHT[np.dtype(dtype)]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("knob", ["tile_xcd", "sweep_no_lane_order"])
def test_measurement_layout_switches(torch, monkeypatch, dtype, knob):
    """Two layout switches kept for measurements: SPMV_TILE_XCD=1 (the tiles
    dealt XCD-contiguously) on a banded matrix, and SPMV_SWEEP_LANE_ORDER=0 (packed sweep chunks in
    plain column order, hence no delta-coded columns) on a power-law one. y matches the oracle."""
    lib = spmv_hw.load(dtype, ablations=True)
    if knob == "tile_xcd":
        monkeypatch.setenv("SPMV_HW_KERNEL", "tiles")
        tools_env(monkeypatch, "SPMV_TILE_XCD", "1")
        n = 1_000_000
        rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
        m = n
    else:
        monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
        tools_env(monkeypatch, "SPMV_SWEEP_LANE_ORDER", "0")
        n, m = 2_000_000, 10_000_000
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, 16 * n, seed=13)
    x = spmv_hw.gen_vector(lib, m, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
    st = plan.stats()
    if knob == "sweep_no_lane_order":
        assert st["kernel"] == 2 and st["format"] & 2 and not st["format"] & (4 | 64), st
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    plan.destroy()
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_fp64acc(row_ptr, c, v, xx) if dtype == np.float32 else oracle.spmv_gold(row_ptr, c, v, xx)
    yy = y.cpu().numpy()
    assert not np.isnan(yy).any()
    assert oracle.scaled_error(row_ptr, c, v, xx, ref, yy) <= TIGHT[np.dtype(dtype)]


@pytest.mark.parametrize("bias", ["0", "0.1", "0.02", "-0.02", "default"])
@pytest.mark.parametrize("shape", ["panels", "pieces", "full"])
def test_sweep_xcc_bias(torch, monkeypatch, shape, bias):
    """The sweep's XCC bias: units that run on even XCCs cut lighter than odd ones.
    'panels': 2M x 2M / 32M, whole panels (the biased panel cut); 'pieces': an N = 8-like slice,
    1.25M x 10M / 20M, split pieces (the biased piece cut; the default cuts them evenly, and
    stats format bit 10 / 11 names a pinned even- / odd-lighter cut); 'full': the 10M/160M
    matrix, whose panels sit within 5 % of the LDS row cap, so a 10 % bias clamps panels at the
    cap and then falls back to the even cut. The unit count never changes, and y matches the
    oracle."""
    if shape == "full" and bias != "0.1":
        pytest.skip("the full matrix with the default cut runs in test_gpu_fullsize.py")
    if shape == "panels" and bias in ("0.02", "-0.02"):
        pytest.skip("whole panels: 0 and 0.1 cover the panel cut")
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    if bias == "default":
        monkeypatch.delenv("SPMV_SWEEP_XCC_BIAS", raising=False)
    else:
        monkeypatch.setenv("SPMV_SWEEP_XCC_BIAS", bias)
    lib = spmv_hw.load(np.float64)
    n, m, z = {"panels": (2_000_000, 2_000_000, 32_000_000), "pieces": (1_250_000, 10_000_000, 20_000_000),
               "full": (10_000_000, 10_000_000, 160_000_000)}[shape]
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, z, seed=4)
    x = spmv_hw.gen_vector(lib, m, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
    st = plan.stats()
    assert st["kernel"] == 2, st
    assert st["nr_tiles"] == {"panels": 256, "pieces": 252, "full": 512}[shape], st
    if shape == "pieces":
        d = 0.0 if bias == "default" else float(bias)
        assert bool(st["format"] & 1024) == (d > 0) and bool(st["format"] & 2048) == (d < 0), st
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    plan.destroy()
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    del rp, col, val
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    yy = y.cpu().numpy()
    assert not np.isnan(yy).any()
    ref = oracle.spmv_gold(row_ptr, c, v, xx)
    assert oracle.scaled_error(row_ptr, c, v, xx, ref, yy) <= TIGHT[np.dtype(np.float64)]


@pytest.mark.parametrize("rank", [1, 3])
def test_split_plan_build_is_reproducible(torch, monkeypatch, rank):
    """a split sweep plan's layout is a function of the matrix and the chip
    (the reference's cut is, csr_hw.cpp:459-468): the N = 4 slices of the 10M/160M matrix built
    twice on one device give identical plan stats (format bits 10 / 11 included: the even default
    cut), and both plans' y match the oracle."""
    monkeypatch.delenv("SPMV_SWEEP_XCC_BIAS", raising=False)
    monkeypatch.delenv("SPMV_HW_KERNEL", raising=False)
    lib = spmv_hw.load(np.float64)
    n = 10_000_000
    rp_full, _ = lib.powerlaw_row_ptr(n, 160_000_000, 65536, 4)
    b = lib.partition_rows(rp_full, 4)
    r0, r1 = int(b[rank]), int(b[rank + 1])
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 160_000_000, seed=4, row_begin=r0, row_end=r1)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    stats, ys = [], []
    for _ in range(2):
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
        stats.append(plan.stats())
        y = torch.full((r1 - r0,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        torch.cuda.synchronize()
        ys.append(y.cpu().numpy())
        plan.destroy()
    assert stats[0] == stats[1], stats
    st = stats[0]
    assert st["kernel"] == 2 and not st["format"] & (1024 | 2048), st
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_gold(row_ptr, c, v, xx)
    for yy in ys:
        assert oracle.scaled_error(row_ptr, c, v, xx, ref, yy) <= TIGHT[np.dtype(np.float64)]


@pytest.mark.parametrize("bias", ["0.025", "0.2", "-0.1", "0"])
@pytest.mark.parametrize("dtype,m", [(np.float32, 300_001), (np.float64, 6_000_001)])
@pytest.mark.parametrize("aligned", [True, False])
def test_binned_xcc_bias_windows(torch, monkeypatch, bias, dtype, m, aligned):
    """Pass-1 XCC bias (SPMV_BIN_XCC_BIAS=d, binned.hip build_binned): even windows W (1 + d)
    columns wide, odd ones W (1 - d), so a column's window and offset come from the closed form
    bin_win_of / bin_win_base in the key build, the scatter and k_bin_mul. Columns cover every
    window (one round of 256 windows in fp32, two rounds in fp64 where W is LDS-capped), a
    partial last pair, a negative and a large bias; x aligned and one element in."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "binned")
    tools_env(monkeypatch, "SPMV_BIN_XCC_BIAS", bias)
    rng = np.random.default_rng(31)
    n = 3000
    row_ptr, col, val, x = random_csr(rng, n, m, rng.integers(0, 30, n), dtype)
    col[-1] = m - 1  # the last column of the last (partial) window
    col[0] = 0
    lib = spmv_hw.load(dtype)
    plan = spmv_hw.Plan.from_device(lib, to_dev(torch, row_ptr), to_dev(torch, col), to_dev(torch, val), m)
    assert plan.stats()["kernel"] == KERNEL_ID["binned"]
    off = 0 if aligned else 1
    xb = to_dev(torch, np.concatenate([np.zeros(off, dtype), x]))
    y = torch.full((n,), float("nan"), dtype=xb.dtype, device="cuda")
    plan.run(xb[off:], y)
    torch.cuda.synchronize()
    plan.destroy()
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), y.cpu().numpy(), dtype)


# ---- work stealing among a panel's pieces (split sweep plans) ----
# Built, measured 3.5-5.5 % slower than the static split (profiles/r04c_steal_ab.jsonl) and kept
# as measurement variants 37-39 of the tools library only; these tests keep those measurements
# honest (same y) and check that the product refuses the variants.

@pytest.mark.parametrize("rank", [0, 7])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_work_stealing_on_the_n8_slices(torch, monkeypatch, dtype, rank):
    """Ranks 0 and 7 of the N = 8 strong-scaling cut of the 10M/160M matrix (csr_hw.cpp:459-468,
    as bench.py --gpus 8 cuts it) on a split sweep plan of the tools library: the stealing
    variants (39 / 37 / 38: the last quarter / half / all of each piece's iterations claimable;
    steals land in timing order, so every run hands out the work differently), repeated, and the
    static split (28) all match the oracle."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    lib = spmv_hw.load(dtype, ablations=True)
    n = 10_000_000
    rp_full, _ = lib.powerlaw_row_ptr(n, 160_000_000, 65536, 4)
    b = lib.partition_rows(rp_full, 8)
    r0, r1 = int(b[rank]), int(b[rank + 1])
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, 160_000_000, seed=4, row_begin=r0, row_end=r1)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    st = plan.stats()
    assert st["kernel"] == 2 and not st["format"] & 128, st
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    row_ptr, c, v, xx = h[0].view(np.uint32), h[1].view(np.uint32), h[2], h[3]
    ref = oracle.spmv_fp64acc(row_ptr, c, v, xx) if dtype == np.float32 else oracle.spmv_gold(row_ptr, c, v, xx)
    for variant in (39, 39, 37, 38, 38, 28):
        plan.set_variant(variant)
        assert bool(plan.stats()["format"] & 128) == (variant != 28)
        y = torch.full((r1 - r0,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        torch.cuda.synchronize()
        check(row_ptr, c, v, xx, ref, y.cpu().numpy(), dtype)
    plan.destroy()
    # the product library refuses the measurement variants
    lp = spmv_hw.load(dtype)
    pp = spmv_hw.Plan.from_device(lp, rp, col, val, n)
    with pytest.raises(RuntimeError, match="tools library only"):
        pp.set_variant(38)
    pp.destroy()


@pytest.mark.parametrize("pieces", ["2", "5", "8"])
@pytest.mark.parametrize("name", FIXTURES)
def test_sweep_work_stealing_forced_splits(torch, monkeypatch, name, pieces):
    """Every fixture through a forced split sweep (tools build: SPMV_SWEEP_SPLIT=2,
    SPMV_SWEEP_PIECES=k) and the stealing variants: units of fewer iterations than the claim
    lookahead, empty pieces and pieces dealt over more than one round of workgroups all take the
    claim paths; y matches the oracle on repeated runs (the counters re-arm) and with the static
    split."""
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    tools_env(monkeypatch, "SPMV_SWEEP_SPLIT", "2")
    tools_env(monkeypatch, "SPMV_SWEEP_PIECES", pieces)
    lib = spmv_hw.load(np.float64, ablations=True)
    _, m, row_ptr, col, val, _ = oracle.read_csr(os.path.join(GOLDEN, manifest()[name]["file"]), np.float64)
    x, y_gold = golden_arrays(name, "f64")
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int32) if a.dtype == np.uint32 else a).cuda()  # noqa: E731
    plan = spmv_hw.Plan.from_device(lib, to(row_ptr), to(col if len(col) else np.zeros(1, np.uint32)),
                                    to(val if len(val) else np.zeros(1)), m)
    st = plan.stats()
    n = len(row_ptr) - 1
    for variant in (38, 38, 37, 39, 28):
        plan.set_variant(variant)
        y = torch.full((max(n, 1),), float("nan"), dtype=torch.float64, device="cuda")
        plan.run(to(x if len(x) else np.zeros(1)), y)
        torch.cuda.synchronize()
        check(row_ptr, col, val, x, y_gold, y.cpu().numpy()[:n], np.float64)
    plan.destroy()
    assert st["kernel"] == 2


def _empty_run_csr(rng, n, run, dtype):
    """Poisson(16) rows with a run of empty rows at `run` (slice), random columns."""
    lens = rng.poisson(16, n)
    lens[run] = 0
    row_ptr = np.zeros(n + 1, np.int64)
    row_ptr[1:] = np.cumsum(lens)
    z = int(row_ptr[-1])
    col = rng.integers(0, n, z, dtype=np.uint32)
    val = rng.uniform(-1, 1, z).astype(dtype)
    x = rng.uniform(0, 1, n).astype(dtype)
    return row_ptr.astype(np.uint32), col, val, x


@pytest.mark.timeout(240)
@pytest.mark.parametrize("case", ["trailing_fp64_sweep", "trailing_fp64_nobias", "middle_fp64_nobias",
                                  "trailing_fp32_binned"])
def test_panels_past_a_long_run_of_empty_rows(torch, monkeypatch, case):
    """A run of empty rows longer than a panel (here the last 30K rows of 1M, or 60K in the
    middle) that no nnz-balanced cut can reach: the panel search is bounded and the panel over
    the run is split into panels of at most the LDS rows -- the plan builds in seconds (it used
    to search on to P = n and fail) and y is the oracle's. For the sweep (fp64) and the binned
    kernel (fp32, >= 5M columns), with and without the XCC bias (whose clipped cuts covered a
    middle run but not a trailing one)."""
    import time
    dtype = np.float32 if "fp32" in case else np.float64
    n = 6_000_000 if "fp32" in case else 1_000_000
    run = slice(100_000, 160_000) if case.startswith("middle") else slice(n - 30_000 if n < 5_000_000 else n - 100_000, n)
    if "nobias" in case:
        monkeypatch.setenv("SPMV_SWEEP_XCC_BIAS", "0")
    rng = np.random.default_rng(5)
    row_ptr, col, val, x = _empty_run_csr(rng, n, run, dtype)
    lib = spmv_hw.load(dtype)
    t0 = time.perf_counter()
    y, st = run_device(torch, lib, row_ptr, col, val, x, n)
    assert time.perf_counter() - t0 < 60
    assert st["kernel"] == (6 if "binned" in case else 2), st
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), y, dtype)
    assert not np.any(y[run])
