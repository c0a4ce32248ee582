"""Fast parallel reader (Part 3 of the C-ABI) against the oracle's
restatement of the reference reader (csr.cpp:10-46, :87-136). CPU only.

Bar: bitwise-equal row_ptr / col_ind / values on every file the reference format accepts, for
both precisions and any thread count; the superset (MatrixMarket banner, comments, unsorted
rows, symmetric expansion, pattern) checked against numpy restatements of the same rules."""
import os

import numpy as np
import pytest

import oracle
import spmv_hw
from conftest import DTYPES, FIXTURES, GOLDEN, manifest


def _same(a, b):
    assert a.dtype == b.dtype and a.shape == b.shape
    assert np.array_equal(a.view(np.uint8), b.view(np.uint8))


def _check_against_oracle(path, dtype):
    n, m, rp, col, val, _ = oracle.read_csr(path, dtype)
    lib = spmv_hw.load(dtype)
    rp2, col2, val2, m2 = lib.read_csr(path)
    assert m2 == m and len(rp2) == n + 1
    _same(rp2, rp)
    _same(col2, col)
    _same(val2, val)
    return rp2, col2, val2


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
@pytest.mark.parametrize("threads", ["1", "3", "16"])
def test_fixtures_bitwise_equal_oracle_reader(monkeypatch, name, dtype, tag, threads):
    monkeypatch.setenv("SPMV_READ_THREADS", threads)
    _check_against_oracle(os.path.join(GOLDEN, manifest()[name]["file"]), dtype)


def _write(path, header, lines, newline="\n"):
    with open(path, "w", newline="") as f:
        f.write(header + newline)
        for ln in lines:
            f.write(ln + newline)


def _random_entries(rng, n, m, z):
    rows = np.sort(rng.integers(1, n + 1, z))
    cols = rng.integers(1, m + 1, z)
    vals = rng.uniform(-1e3, 1e3, z) * 10.0 ** rng.integers(-30, 30, z)
    return rows, cols, vals


FORMATS = [
    lambda v: "%.17g" % v,
    lambda v: "%.6e" % v,
    lambda v: "%+.3f" % v,
    lambda v: "%d" % int(v) if abs(v) < 1e9 else "%.17g" % v,
    lambda v: ("%.17g" % v).upper(),
]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("crlf", [False, True])
def test_number_formats_whitespace_and_line_ends(tmp_path, monkeypatch, dtype, crlf):
    """Values in several printf forms (exponents, '+', integers), spaces/tabs between fields,
    CRLF line ends: parsed exactly as sscanf("%u %u %lf") / ("%f") parses them."""
    rng = np.random.default_rng(7)
    n, m, z = 3000, 5000, 40_000
    rows, cols, vals = _random_entries(rng, n, m, z)
    lines = []
    for i in range(z):
        sep = ["  ", "\t", " "][i % 3]
        lines.append(f"{rows[i]}{sep}{cols[i]} {FORMATS[i % len(FORMATS)](vals[i])}")
    p = str(tmp_path / "f.mtx")
    _write(p, f"{n} {m} {z}", lines, "\r\n" if crlf else "\n")
    monkeypatch.setenv("SPMV_READ_THREADS", "7")
    _check_against_oracle(p, dtype)


def test_values_round_once_in_fp32(tmp_path):
    """fp32 values come straight from the text (util.h:20 '%f'), not through a double."""
    # 1 + 2^-24 + 2^-60: rounding to double first gives a tie (-> 1.0), direct rounding gives
    # the next float up
    txt = "1.0000000596046447753906250867361737988403547205962240695953369140625"
    p = str(tmp_path / "r.mtx")
    _write(p, "1 1 1", [f"1 1 {txt}"])
    lib = spmv_hw.load(np.float32)
    _, _, val, _ = lib.read_csr(p)
    assert val[0] == np.nextafter(np.float32(1), np.float32(2))
    _check_against_oracle(p, np.float32)


def _csr_from_entries(n, rows0, cols0, vals, dtype):
    """numpy restatement: stable sort by row, entries of a row in file order."""
    order = np.argsort(rows0, kind="stable")
    rp = np.zeros(n + 1, np.int64)
    np.add.at(rp, rows0 + 1, 1)
    return (np.cumsum(rp).astype(np.uint32), cols0[order].astype(np.uint32),
            np.asarray(vals, dtype)[order])


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_matrix_market_banner_comments_unsorted(tmp_path, monkeypatch, dtype):
    rng = np.random.default_rng(3)
    n, m, z = 4000, 3000, 30_000
    rows = rng.integers(1, n + 1, z)          # NOT sorted
    cols = rng.integers(1, m + 1, z)
    vals = rng.uniform(-1, 1, z)
    lines = []
    for i in range(z):
        if i % 997 == 0:
            lines.append("% a comment line")
        lines.append(f"{rows[i]} {cols[i]} {vals[i]:.17g}")
    p = str(tmp_path / "mm.mtx")
    _write(p, "%%MatrixMarket matrix coordinate real general\n% generated\n%\n" + f"{n} {m} {z}", lines)
    lib = spmv_hw.load(dtype)
    rc, h = lib.read_csr_header(p)
    assert rc == 0 and (h.nr_rows, h.nr_cols, h.nr_nzeros, h.blocks) == (n, m, z, 1)
    for threads in ("1", "5"):
        monkeypatch.setenv("SPMV_READ_THREADS", threads)
        rp, col, val, m2 = lib.read_csr(p)
        erp, ecol, evals = _csr_from_entries(n, rows - 1, cols - 1, vals.astype(dtype), dtype)
        assert m2 == m
        _same(rp, erp)
        _same(col, ecol)
        _same(val, evals)


@pytest.mark.parametrize("symmetry,sign", [("symmetric", 1.0), ("skew-symmetric", -1.0)])
def test_symmetric_files_are_expanded(tmp_path, symmetry, sign):
    rng = np.random.default_rng(9)
    n, z = 500, 3000
    r = rng.integers(1, n + 1, z)
    c = rng.integers(1, n + 1, z)
    lo = np.minimum(r, c) if symmetry == "symmetric" else np.minimum(r, c)
    hi = np.maximum(r, c)
    if symmetry == "skew-symmetric":
        keep = hi != lo  # a skew-symmetric matrix has a zero diagonal
        lo, hi = lo[keep], hi[keep]
    v = rng.uniform(-1, 1, len(lo))
    p = str(tmp_path / "s.mtx")
    _write(p, f"%%MatrixMarket matrix coordinate real {symmetry}\n{n} {n} {len(lo)}",
           [f"{a} {b} {x:.17g}" for a, b, x in zip(hi, lo, v)])
    lib = spmv_hw.load(np.float64)
    rc, h = lib.read_csr_header(p)
    exp_r, exp_c, exp_v = [], [], []
    for a, b, x in zip(hi, lo, v):
        exp_r.append(a - 1), exp_c.append(b - 1), exp_v.append(x)
        if a != b:
            exp_r.append(b - 1), exp_c.append(a - 1), exp_v.append(sign * x)
    assert rc == 0 and h.nr_nzeros == len(exp_r)
    rp, col, val, _ = lib.read_csr(p)
    erp, ecol, evals = _csr_from_entries(n, np.array(exp_r), np.array(exp_c), np.array(exp_v), np.float64)
    _same(rp, erp)
    _same(col, ecol)
    _same(val, evals)


def test_pattern_entries_are_ones(tmp_path):
    p = str(tmp_path / "p.mtx")
    _write(p, "%%MatrixMarket matrix coordinate pattern general\n3 4 4", ["1 2", "1 4", "3 1", "3 3"])
    rp, col, val, m = spmv_hw.load(np.float64).read_csr(p)
    assert list(rp) == [0, 2, 2, 4] and list(col) == [1, 3, 0, 2] and m == 4
    assert np.all(val == 1.0)


@pytest.mark.parametrize("body,what", [
    (["1 1 0.5", "2 x 1.0"], "parse error"),
    (["1 1 0.5", "3 1 1.0"], "parse error"),     # row beyond the header
    (["1 1 0.5", "2 9 1.0"], "parse error"),     # column beyond the header
    (["1 1 0.5"], "entries in the file"),         # fewer entries than the header says
    (["1 1 0.5", "2 2 1", "2 1 1"], "entries in the file"),
])
def test_malformed_files_are_rejected(tmp_path, body, what):
    p = str(tmp_path / "bad.mtx")
    _write(p, "2 2 2", body)
    lib = spmv_hw.load(np.float64)
    with pytest.raises(RuntimeError, match=what):
        lib.read_csr(p)


def test_header_return_codes(tmp_path):
    """read_csr_header's codes (csr.cpp:10-46): 1 = cannot open / EOF, 3 = parse error."""
    lib = spmv_hw.load(np.float64)
    assert lib.read_csr_header(str(tmp_path / "missing.mtx"))[0] == 1
    p = tmp_path / "empty.mtx"
    p.write_text("")
    assert lib.read_csr_header(str(p))[0] == 1
    p.write_text("10 ten 3\n")
    assert lib.read_csr_header(str(p))[0] == 3
    p.write_text("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    assert lib.read_csr_header(str(p))[0] == 3


def test_large_file_many_threads_equals_one_thread(tmp_path, monkeypatch):
    rng = np.random.default_rng(1)
    n, m, z = 50_000, 50_000, 600_000
    rows, cols, vals = _random_entries(rng, n, m, z)
    p = str(tmp_path / "big.mtx")
    with open(p, "w") as f:
        f.write(f"{n} {m} {z}\n")
        np.savetxt(f, np.column_stack([rows, cols, vals]), fmt=["%d", "%d", "%.17g"])
    monkeypatch.setenv("SPMV_READ_THREADS", "1")
    a = spmv_hw.load(np.float64).read_csr(p)
    monkeypatch.setenv("SPMV_READ_THREADS", "8")
    b = spmv_hw.load(np.float64).read_csr(p)
    for u, v in zip(a[:3], b[:3]):
        _same(u, v)
    _check_against_oracle(p, np.float64)
