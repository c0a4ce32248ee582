"""The CPU oracle (oracle/csr_ref.c) against the golden fixtures and known answers.

Parity status of the oracle: "parity unpinned" (the reference cannot be built here, it ships no
fixtures). What pins it: glibc rand() known answers recorded in SURVEY.md §8(a3), an independent
numpy restatement (bit-exact), and the reference's own self-check (main.cpp:77-82) applied to
the restated FPGA arithmetic order.
"""
import os

import numpy as np
import pytest

import oracle
from conftest import DTYPES, FIXTURES, GOLDEN, golden_arrays, manifest


def numpy_spmv_gold(row_ptr, col, val, x):
    """Independent restatement of csr.cpp:184-194: rows accumulate from 0 in CSR order;
    vectorised over rows by position-in-row, which keeps every row's addition order."""
    n = len(row_ptr) - 1
    y = np.zeros(n, val.dtype)
    lens = np.diff(row_ptr.astype(np.int64))
    starts = row_ptr[:-1].astype(np.int64)
    for k in range(int(lens.max()) if n else 0):
        rows = np.nonzero(lens > k)[0]
        idx = starts[rows] + k
        y[rows] = y[rows] + val[idx] * x[col[idx]]
    return y


def parse_mtx(path, dtype):
    with open(path) as f:
        n, m, z = (int(t) for t in f.readline().split())
        data = [ln.split() for ln in f]
    r = np.array([int(d[0]) for d in data], np.int64) - 1
    c = np.array([int(d[1]) for d in data], np.int64) - 1
    v = np.array([float(d[2]) for d in data], np.float64).astype(dtype)
    row_ptr = np.zeros(n + 1, np.int64)
    np.add.at(row_ptr, r + 1, 1)
    return n, m, z, np.cumsum(row_ptr).astype(np.uint32), c.astype(np.uint32), v


def test_init_vector_rand_glibc_known_answers():
    # x[0]=0.84018771715470952, x[1]=0.39438292681909304 (libc rand, seed 1)
    x = oracle.init_vector_rand(2, np.float64, seed=1)
    assert x[0] == 0.84018771715470952
    assert x[1] == 0.39438292681909304
    x32 = oracle.init_vector_rand(2, np.float32, seed=1)
    assert x32[0] == np.float32(1804289383) / np.float32(2147483647)


@pytest.mark.parametrize("name", FIXTURES)
def test_reader_matches_independent_parse(name):
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    n, m, z, row_ptr, col, val = parse_mtx(path, np.float64)
    r, c, rp, ci, v, _ = oracle.read_csr(path, np.float64)
    assert (r, c) == (n, m)
    assert np.array_equal(rp, row_ptr)
    assert np.array_equal(ci, col)
    assert np.array_equal(v, val)
    _, _, _, _, v32, _ = oracle.read_csr(path, np.float32)
    assert np.array_equal(v32, val.astype(np.float32))


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
def test_spmv_gold_matches_fixture(name, dtype, tag):
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    r, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
    x_ref, y_ref = golden_arrays(name, tag)
    x = oracle.init_vector_rand(c, dtype, seed=1)
    assert np.array_equal(x, x_ref)
    y = oracle.spmv_gold(row_ptr, col, val, x)
    assert y.dtype == y_ref.dtype
    assert np.array_equal(y.view(np.uint8), y_ref.view(np.uint8)), "oracle drifted from the fixture"


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
def test_spmv_gold_matches_numpy_restatement(name, dtype, tag):
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    _, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
    x, _ = golden_arrays(name, tag)
    assert np.array_equal(oracle.spmv_gold(row_ptr, col, val, x), numpy_spmv_gold(row_ptr, col, val, x))


# valid reference configurations: VF >= RATIO_v; COLS_DIV_BLOCKS by CU (util.h:41-59)
FPGA_CONFIGS = [(32768, 2), (32768, 4), (32768, 8), (16384, 2), (16384, 8)]


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
@pytest.mark.parametrize("cdb,vf", FPGA_CONFIGS)
def test_fpga_order_passes_reference_self_check(name, dtype, tag, cdb, vf):
    """The reference's own check (main.cpp:77-82, verification csr_hw.cpp:1571-1590) holds for
    the restated FPGA arithmetic order against spmv_gold."""
    if dtype == np.float32 and vf < 4:
        pytest.skip("VF < RATIO_v is an invalid reference configuration for fp32 (SURVEY B1)")
    path = os.path.join(GOLDEN, manifest()[name]["file"])
    _, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
    x, y_gold = golden_arrays(name, tag)
    y_fpga = oracle.spmv_fpga_order(row_ptr, col, val, x, c, cdb, vf)
    if dtype == np.float64:
        assert oracle.verification_errors(y_gold, y_fpga) == 0
        assert oracle.scaled_error(row_ptr, col, val, x, y_gold, y_fpga) <= 1e-12
    else:
        # fp32: the reference's absolute 1e-5 threshold is below fp32 resolution once |y| ~ 20
        # (longrow: 21.905691 vs 21.905714), so only the scaled error gates it.
        assert oracle.scaled_error(row_ptr, col, val, x, y_gold, y_fpga) <= 1e-5


def test_trailing_empty_rows_are_filled():
    """rows after the last entry get row_ptr = nnz (the reference leaves them unset)."""
    path = os.path.join(GOLDEN, "trail.mtx")
    r, _, row_ptr, _, _, _ = oracle.read_csr(path, np.float64)
    nnz = row_ptr[-1]
    assert np.all(row_ptr[-11:] == nnz)
    assert np.all(np.diff(row_ptr.astype(np.int64)) >= 0)


def test_blocks_from_header():
    """csr.cpp:39-43: blocks = ceil(cols / COLS_DIV_BLOCKS)."""
    *_, blocks = oracle.read_csr(os.path.join(GOLDEN, "wide.mtx"), np.float64, cols_div_blocks=32768)
    assert blocks == 4
    *_, blocks = oracle.read_csr(os.path.join(GOLDEN, "wide.mtx"), np.float64, cols_div_blocks=16384)
    assert blocks == 7


def test_scaled_error_metric():
    row_ptr = np.array([0, 2, 2, 3], np.uint32)
    col = np.array([0, 1, 1], np.uint32)
    val = np.array([1.0, -1.0, 2.0])
    x = np.array([1.0, 1.0])
    y = np.array([0.0, 0.0, 2.0])
    assert oracle.scaled_error(row_ptr, col, val, x, y, y) == 0.0
    assert oracle.scaled_error(row_ptr, col, val, x, y, y + np.array([1e-9, 0, 0])) == pytest.approx(5e-10)
    assert oracle.scaled_error(row_ptr, col, val, x, y, y + np.array([0, 1e-30, 0])) == float("inf")
