"""spmv_hw's streamed copy-back (csr_hw_wrapper.cpp spmv_hw_streamed): on plans whose sweep runs
one workgroup per panel, each workgroup flags its panel in host memory once the panel's rows of y
are in memory (a system-scope release), and a feeder thread copies each piece of y (whole panels)
while the rest still sweeps; the adding threads add every piece as it lands (accum_results'
`+=`, csr_hw.cpp:1531-1565). The reference's three lines keep their meaning. y must be the
oracle's (spmv_gold, csr.cpp:184-194) call after call -- the flags carry a per-call epoch, so a
piece is never copied on the previous call's flag -- with one unit and with two units sharing the
GPU, and identical to the unstreamed merge (SPMV_HW_STREAM=0)."""
import re

import numpy as np
import pytest

import oracle
import spmv_hw
from conftest import tools_env

pytestmark = pytest.mark.gpu


def _matrix(lib, n, z, seed=4):
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=seed)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    h = (rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32), val.cpu().numpy(), x.cpu().numpy())
    del rp, col, val, x
    return h


def _flow(lib, h_rp, h_col, h_val, h_x, calls):
    n = len(h_rp) - 1
    m = lib.make_csr_matrix(h_rp, h_col, h_val, n)
    hw, bm = lib.create_csr_hw_matrix(m)
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(h_x), 1, hw[0].contents.nr_cols)
    yv = lib.make_csr_vector(np.zeros(n, h_val.dtype))
    ys = []
    for _ in range(calls):
        lib.spmv_hw(hw, hx, yv, bm)
        ys.append(np.ctypeslib.as_array(yv.values, shape=(n,)).copy())
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)
    return ys


def _check_tapered_pieces(err, units, calls):
    """The trace's pieces (csr_hw_wrapper.cpp piece_bounds): per call and unit, whole panels
    that tile [0, P) in order, 8 / units of them (at least 2), tapering -- no piece larger than
    the one before it -- so the last copy to land leaves a small add (the last is 1/16 of the
    first at 8 pieces, 1/4 at 4; 2 or 3 pieces are equal)."""
    found = [(int(u), int(a), int(b)) for u, a, b in re.findall(r"piece unit (\d+) panels \[(\d+), (\d+)\)", err)]
    assert len(found) % calls == 0 and found, err[-2000:]
    per_call = found[:len(found) // calls]
    k = max(2, 8 // units)
    for u in range(units):
        ps = [(a, b) for v, a, b in per_call if v == u]
        assert len(ps) == k and ps[0][0] == 0, ps
        assert all(ps[j][1] == ps[j + 1][0] for j in range(k - 1)), ps
        sizes = [b - a for a, b in ps]
        assert all(sizes[j] + 1 >= sizes[j + 1] >= 1 for j in range(k - 1)), sizes  # (+1: rounding)
        if k >= 4:  # (fewer pieces: equal parts)
            assert sizes[-1] * (16 if k >= 8 else 4) <= sizes[0] + 16, sizes  # (weights 16..1, 1 / 4, 2, 1, 1)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("units", [1, 2])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_streamed_copy_back_matches_the_oracle(monkeypatch, capfd, units, dtype):
    """A 6M-row power-law matrix (one whole-panel sweep plan per unit) through spmv_hw three
    times: every call's y is A x added once more, within the oracle's tolerance; the trace
    names the streamed branch; with SPMV_HW_STREAM=0 the same calls give the same bits."""
    monkeypatch.setenv("SPMV_NGPUS", str(units))
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    monkeypatch.delenv("SPMV_HW_STREAM", raising=False)
    if dtype == np.float32:  # (fp32 matrices this size take the binned kernel by default)
        monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    lib = spmv_hw.load(dtype)
    n, z = 6_000_000, 96_000_000
    h = _matrix(lib, n, z)
    ys = _flow(lib, *h, calls=3)
    _, err = capfd.readouterr()
    assert err.count("D2H landed (streamed)") == 3, err[-2000:]
    _check_tapered_pieces(err, units, calls=3)
    ref = oracle.spmv_gold(*h) if dtype == np.float64 else oracle.spmv_fp64acc(*h)
    tight = 1e-12 if dtype == np.float64 else 2e-6
    assert oracle.scaled_error(*h, ref, ys[0]) <= tight
    for k in (1, 2):  # each call adds A x once more (in the library's precision)
        d = ys[k].astype(np.float64) - ys[k - 1].astype(np.float64)
        assert oracle.scaled_error(*h, ref.astype(np.float64), d) <= (1e-12 if dtype == np.float64 else 1e-5)
    monkeypatch.setenv("SPMV_HW_STREAM", "0")
    ys0 = _flow(lib, *h, calls=1)
    _, err = capfd.readouterr()
    assert "streamed" not in err
    # the sweep's LDS adds run in timing order: two runs agree to rounding, not bit for bit
    scale = float(np.abs(ys[0].astype(np.float64)).max())
    assert float(np.abs(ys0[0].astype(np.float64) - ys[0]).max()) <= (1e-13 if dtype == np.float64 else 1e-5) * scale


@pytest.mark.timeout(600)
def test_streamed_copy_back_at_headline_size(monkeypatch, capfd):
    """Config 3's 10M/160M fp64 matrix through the drop-in with one unit (the bench's `dropin`
    field): two rounds of whole panels, so half of y is copied while the second round sweeps.
    y is spmv_gold's (verification 0, scaled error <= 1e-12) on every call, and the printed
    Total is Hardware + Accumulation."""
    monkeypatch.setenv("SPMV_NGPUS", "1")
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    lib = spmv_hw.load(np.float64)
    h = _matrix(lib, 10_000_000, 160_000_000)
    ys = _flow(lib, *h, calls=3)
    out, err = capfd.readouterr()
    assert err.count("D2H landed (streamed)") == 3
    _check_tapered_pieces(err, 1, calls=3)
    ref = oracle.spmv_gold(*h)
    assert oracle.scaled_error(*h, ref, ys[0]) <= 1e-12
    assert lib.verification(ref, ys[0]) == 0
    assert oracle.scaled_error(*h, ref, ys[2] - ys[1]) <= 1e-12
    hw = [float(v) for v in re.findall(r"Hardware execution time : ([0-9.]+)", out)]
    ra = [float(v) for v in re.findall(r"Result accumulation time : ([0-9.]+)", out)]
    tot = [float(v) for v in re.findall(r"Total time  : ([0-9.]+)", out)]
    assert len(hw) == len(ra) == len(tot) == 3
    assert all(abs(t - a - b) < 1e-3 for t, a, b in zip(tot, hw, ra))


@pytest.mark.timeout(300)
def test_direct_form_of_the_tools_build(monkeypatch, capfd):
    """The tools build's direct form (SPMV_HW_DIRECT=1, a measurement variant): the sweep stores
    each panel's y straight into pinned host memory over PCIe and flags it; the host adds from
    there with no copy. y is the oracle's on every call."""
    monkeypatch.setenv("SPMV_NGPUS", "1")
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    tools_env(monkeypatch, "SPMV_HW_DIRECT", "1")
    lib = spmv_hw.load(np.float64)
    h = _matrix(lib, 6_000_000, 96_000_000)
    ys = _flow(lib, *h, calls=3)
    _, err = capfd.readouterr()
    assert err.count("D2H landed (streamed)") == 3
    ref = oracle.spmv_gold(*h)
    assert oracle.scaled_error(*h, ref, ys[0]) <= 1e-12
    assert oracle.scaled_error(*h, ref, ys[2] - ys[1]) <= 1e-12


@pytest.mark.timeout(300)
@pytest.mark.parametrize("run", [False, True], ids=["scattered", "with_a_long_run"])
def test_streamed_copy_back_with_empty_rows(monkeypatch, capfd, run):
    """Empty rows (20 % scattered) and a last row that is empty: every row of y comes back
    through the flagged panels -- the empty ones as 0 -- and matches spmv_gold (here with a
    y_fpga that starts non-zero, since spmv_hw adds). With a run of 49K empty rows as well, the
    panels around it hold chunks of a few entries spread over > 65536 columns; those chunks keep
    their absolute columns in the side table (format bit 12), and the plan stays on the packed,
    flagged sweep."""
    monkeypatch.setenv("SPMV_NGPUS", "1")
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    rng = np.random.default_rng(21)
    n = 6_000_000
    lens = rng.poisson(16, n)
    lens[rng.random(n) < 0.2] = 0
    if run:
        lens[1000:50_000] = 0  # a run of empty rows longer than a panel
    lens[-1] = 0
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    z = int(rp[-1])
    col = rng.integers(0, n, z, dtype=np.uint32)
    val = rng.uniform(-1, 1, z)
    x = rng.uniform(0, 1, n)
    rp = rp.astype(np.uint32)
    lib = spmv_hw.load(np.float64)
    m = lib.make_csr_matrix(rp, col, val, n)
    hw, bm = lib.create_csr_hw_matrix(m)
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), 1, hw[0].contents.nr_cols)
    y0 = rng.uniform(-1, 1, n)
    yv = lib.make_csr_vector(y0.copy())
    lib.spmv_hw(hw, hx, yv, bm)
    y = np.ctypeslib.as_array(yv.values, shape=(n,)).copy()
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)
    _, err = capfd.readouterr()
    assert "D2H landed (streamed)" in err, err[-2000:]
    ref = oracle.spmv_gold(rp, col, val, x)
    # y = y0 + A x: componentwise against the oracle, scaled by |y0| + |A||x| (the add's rounding)
    absax = oracle.spmv_gold(rp, col, np.abs(val), x)
    assert float(np.max(np.abs(y - (y0 + ref)) / (np.abs(y0) + absax + 1e-300))) <= 1e-12
    assert np.array_equal(y[lens == 0], y0[lens == 0])  # empty rows: y_fpga += 0


@pytest.mark.timeout(300)
@pytest.mark.parametrize("units", [1, 2])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_streamed_copy_back_of_the_binned_kernel(monkeypatch, capfd, units, dtype):
    """The two-pass binned kernel (config 5's automatic choice in fp32) streams too: its second
    pass writes whole panels (binned.hip k_bin_acc) and flags each one. Three calls through
    spmv_hw, y against the oracle each time, tapered pieces, and the same y as the unstreamed
    merge to rounding (the LDS adds run in timing order)."""
    monkeypatch.setenv("SPMV_NGPUS", str(units))
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    monkeypatch.setenv("SPMV_HW_KERNEL", "binned")
    monkeypatch.delenv("SPMV_HW_STREAM", raising=False)
    lib = spmv_hw.load(dtype)
    h = _matrix(lib, 6_000_000, 96_000_000)
    ys = _flow(lib, *h, calls=3)
    _, err = capfd.readouterr()
    assert err.count("D2H landed (streamed)") == 3, err[-2000:]
    _check_tapered_pieces(err, units, calls=3)
    ref = oracle.spmv_gold(*h) if dtype == np.float64 else oracle.spmv_fp64acc(*h)
    assert oracle.scaled_error(*h, ref, ys[0]) <= (1e-12 if dtype == np.float64 else 2e-6)
    for k in (1, 2):
        d = ys[k].astype(np.float64) - ys[k - 1].astype(np.float64)
        assert oracle.scaled_error(*h, ref.astype(np.float64), d) <= (1e-12 if dtype == np.float64 else 1e-5)
    monkeypatch.setenv("SPMV_HW_STREAM", "0")
    ys0 = _flow(lib, *h, calls=1)
    _, err = capfd.readouterr()
    assert "streamed" not in err
    scale = float(np.abs(ys[0].astype(np.float64)).max())
    assert float(np.abs(ys0[0].astype(np.float64) - ys[0]).max()) <= (1e-13 if dtype == np.float64 else 1e-5) * scale


@pytest.mark.timeout(300)
@pytest.mark.parametrize("units", [3, 4])
def test_streamed_copy_back_with_more_units(monkeypatch, capfd, units):
    """3 and 4 units on one GPU (2 pieces each, landing in unit-interleaved order) through the
    streamed copy-back: y is the oracle's on every call."""
    monkeypatch.setenv("SPMV_NGPUS", str(units))
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    monkeypatch.delenv("SPMV_HW_STREAM", raising=False)
    lib = spmv_hw.load(np.float64)
    h = _matrix(lib, 8_000_000, 128_000_000)
    ys = _flow(lib, *h, calls=2)
    _, err = capfd.readouterr()
    assert err.count("D2H landed (streamed)") == 2, err[-2000:]
    _check_tapered_pieces(err, units, calls=2)
    ref = oracle.spmv_gold(*h)
    assert oracle.scaled_error(*h, ref, ys[0]) <= 1e-12
    assert oracle.scaled_error(*h, ref, ys[1] - ys[0]) <= 1e-12


@pytest.mark.timeout(300)
def test_copy_back_when_a_unit_holds_only_empty_rows(monkeypatch, capfd):
    """The last third of the rows empty, 3 units: the nnz-balanced cut leaves the last unit a run
    of empty rows (whatever plan that gets, it cannot flag panels of a sweep), so spmv_hw takes
    the unstreamed merge or streams the others -- either way y_fpga += A x row for row, and the
    empty rows keep the caller's values."""
    monkeypatch.setenv("SPMV_NGPUS", "3")
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    monkeypatch.delenv("SPMV_HW_STREAM", raising=False)
    rng = np.random.default_rng(8)
    n = 6_000_000
    lens = rng.poisson(16, n)
    lens[4_000_000:] = 0
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    z = int(rp[-1])
    col = rng.integers(0, n, z, dtype=np.uint32)
    val = rng.uniform(-1, 1, z)
    x = rng.uniform(0, 1, n)
    rp = rp.astype(np.uint32)
    lib = spmv_hw.load(np.float64)
    m = lib.make_csr_matrix(rp, col, val, n)
    hw, bm = lib.create_csr_hw_matrix(m)
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), 1, hw[0].contents.nr_cols)
    y0 = rng.uniform(-1, 1, n)
    yv = lib.make_csr_vector(y0.copy())
    lib.spmv_hw(hw, hx, yv, bm)
    y = np.ctypeslib.as_array(yv.values, shape=(n,)).copy()
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)
    capfd.readouterr()
    ref = oracle.spmv_gold(rp, col, val, x)
    absax = oracle.spmv_gold(rp, col, np.abs(val), x)
    assert float(np.max(np.abs(y - (y0 + ref)) / (np.abs(y0) + absax + 1e-300))) <= 1e-12
    assert np.array_equal(y[4_000_000:], y0[4_000_000:])
