"""Seeded random CSR matrices through every kernel and layout (the edge cases of
test_gpu_parity.py, mixed): row-length families from all-empty to heavy-tailed, columns
uniform, windowed (spans around the 8/16-bit offset limits of the narrow tiles, packed sweep
entries and slice offsets), clustered, unsorted with duplicates; x with both signs so rows
cancel. Gate as in test_gpu_parity: scaled error <= 1e-12 fp64 / 2e-6 fp32 against spmv_gold
(csr.cpp:184-194); the gold kernel bitwise against spmv_gold and the FPGA-order kernels (3, 4)
bitwise against the restated hardware order (spmv.cpp:66-104, csr_hw.cpp:1531-1565) for a
random VF and column-block width. "auto" and "tune" run the automatic and the timed
layout choice (SPMV_HW_KERNEL unset / =tune)."""
import os

import numpy as np
import pytest

import oracle
import spmv_hw
from conftest import TOOLS_ONLY_ENV, tools_env
from test_gpu_parity import KERNEL_ID, _bitwise, check, run_device

pytestmark = pytest.mark.gpu

# 48 seeds in the suite; SPMV_FUZZ_SEEDS=a-b runs seeds [a, b) instead (one-off extended runs)
_SR = os.environ.get("SPMV_FUZZ_SEEDS", "0-48").split("-")
SEEDS = list(range(int(_SR[0]), int(_SR[1])))
FUZZ_KERNELS = ["tiles", "tiles_wide", "sweep", "sweep_rc", "sweep_unpacked", "sweep_det", "gold", "slices", "slices_wide",
                "slices_acc32", "fpga", "blocked", "binned", "binned_delta", "auto", "tune"]
ENV = {"tiles_wide": {"SPMV_TILE_NARROW": "0"}, "sweep_unpacked": {"SPMV_SWEEP_PACKED": "0"},
       "sweep_rc": {"SPMV_SWEEP_DELTA": "0"},
       "sweep_det": {"SPMV_SWEEP_DETERMINISTIC": "1"},
       "slices_wide": {"SPMV_SLICE_NARROW": "0"}, "slices_acc32": {"SPMV_SLICE_ACC": "32"},
       "binned_delta": {"SPMV_BIN_DELTA": "1"}}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def fuzz_case(seed, dtype):
    """(row_ptr, col, val, x, m, unsorted) for one seed; the family cycles with the seed."""
    rng = np.random.default_rng(1000 + seed)
    fam = seed % 8
    n = int(rng.integers(1, 5000))
    m = int(rng.choice([1, 17, 1000, 70_000, 300_000], p=[0.05, 0.1, 0.3, 0.25, 0.3]))
    if fam == 0:  # geometric lengths
        lens = rng.geometric(1.0 / rng.uniform(1, 40), n) - 1
    elif fam == 1:  # heavy tail (Pareto), a few very long rows
        lens = np.minimum((rng.pareto(1.2, n) * 4).astype(np.int64), 40_000)
    elif fam == 2:  # mostly empty with a few dense rows
        lens = np.where(rng.random(n) < 0.02, rng.integers(100, 3000, n), 0)
    elif fam == 3:  # multiples of the wave/tile widths, and one-off
        lens = rng.choice([0, 1, 63, 64, 65, 511, 512, 513], n)
    elif fam == 4:  # all rows empty but one
        lens = np.zeros(n, np.int64)
        lens[rng.integers(0, n)] = rng.integers(1, 2000)
    else:  # uniform short rows
        lens = rng.integers(0, 48, n)
    lens = np.asarray(lens, np.int64)
    unsorted = fam == 7
    if not unsorted:
        lens = np.minimum(lens, m)  # sorted rows hold distinct columns
    row_ptr = np.zeros(n + 1, np.int64)
    row_ptr[1:] = np.cumsum(lens)
    z = int(row_ptr[-1])
    col = np.empty(z, np.uint32)
    span = int(rng.choice([200, 256, 257, 16_384, 65_535, 65_537, m]))
    for i in range(n):
        k = int(lens[i])
        if not k:
            continue
        if fam == 5:  # windowed: a band whose per-row window is `span` columns wide
            lo = min(max(0, i * m // n - span // 2), max(0, m - span))
            w = min(span, m)
            c = lo + np.sort(rng.choice(w, size=min(k, w), replace=False))
        elif fam == 6:  # clustered: a few runs of adjacent columns spread over [0, m)
            runs = max(1, k // 16)
            starts = np.sort(rng.choice(max(1, m - 16), size=min(runs, max(1, m - 16)), replace=False))
            c = np.unique((starts[:, None] + np.arange(16)[None, :]).ravel() % m)[:k]
            if len(c) < k:
                c = np.sort(rng.choice(m, size=k, replace=False))
        elif unsorted:  # unordered, duplicates allowed
            c = rng.integers(0, m, k)
        else:
            c = np.sort(rng.choice(m, size=k, replace=False))
        col[row_ptr[i]:row_ptr[i + 1]] = c
    val = rng.uniform(-1, 1, z).astype(dtype)
    val[rng.random(z) < 0.05] = 0
    x = rng.uniform(-1, 1, m).astype(dtype)
    return row_ptr.astype(np.uint32), col, val, x, m, unsorted


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kern", FUZZ_KERNELS)
@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz(torch, monkeypatch, seed, kern, dtype):
    row_ptr, col, val, x, m, unsorted = fuzz_case(seed, dtype)
    monkeypatch.setenv("SPMV_HW_KERNEL", kern.split("_")[0])
    for k, v in ENV.get(kern, {}).items():
        if k in TOOLS_ONLY_ENV:
            tools_env(monkeypatch, k, v)
        else:
            monkeypatch.setenv(k, v)
    rng = np.random.default_rng(seed)
    vf, block = int(rng.choice([1, 2, 4, 8])), int(rng.choice([1, 7, 97, 700, 4096, 32768, 65536]))
    block = max(block, -(-m // 4096))  # kernel 4: at most one fp64 row chunk (4096) of blocks
    monkeypatch.setenv("SPMV_FPGA_VF", str(vf))
    monkeypatch.setenv("SPMV_FPGA_BLOCK", str(block))
    lib = spmv_hw.load(dtype)
    y, st = run_device(torch, lib, row_ptr, col, val, x, m)
    if kern in ("auto", "tune"):  # the automatic choice / the timed choice among tiles, sweep, slices, binned
        assert st["kernel"] in (0, 2, 5, 6)
    else:
        assert st["kernel"] == KERNEL_ID[kern.split("_")[0]]
    if kern == "gold" or (kern.startswith("slices") and (dtype == np.float64 or kern == "slices_acc32")):
        # kernel 5 adds each row's products in CSR order from +0 with separate multiplies and
        # adds (no fused multiply-add in its ISA): bit for bit spmv_gold's arithmetic in fp64,
        # and in fp32 with the fp32 accumulator (SPMV_SLICE_ACC=32)
        _bitwise(y, oracle.spmv_gold(row_ptr, col, val, x))
    elif kern in ("fpga", "blocked"):
        _bitwise(y, oracle.spmv_fpga_order(row_ptr, col, val, x, m, block, vf))
    elif kern == "sweep_det":  # the deterministic sweep gives the same bits again
        y2, _ = run_device(torch, lib, row_ptr, col, val, x, m)
        _bitwise(y2, y)
    check(row_ptr, col, val, x, oracle.spmv_gold(row_ptr, col, val, x), y, dtype)
