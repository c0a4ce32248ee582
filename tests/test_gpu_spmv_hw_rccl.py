"""spmv_hw (the reference's entry, csr_hw_wrapper.cpp:193-288) with the RCCL merge: with
SPMV_HW_MERGE=gather (or reduce) and the units on distinct GPUs, the slices meet on GPU 0 over
xGMI -- an RCCL gather of the disjoint slices, or the literal ncclReduce(sum) of full-length
partials (accum_results' `+=`, csr_hw.cpp:1531-1565) -- and one D2H copy brings y home. The
default (auto) is the per-GPU PCIe merge. The box has one GPU, so these tests run the RCCL branch
with one unit: there a gather issues NO RCCL call (its schedule has no exchange op; the trace
says "0 RCCL calls") and only the reduce goes through RCCL (one ncclReduce that copies the
partial). The multi-rank send / receive arithmetic of the same schedule is executed on the CPU by
tests/test_exchange_schedule.py (gloo replay). y is checked against the oracle's spmv_gold
(csr.cpp:184-194) and the golden fixtures."""
import re
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
import spmv_hw
from conftest import DTYPES, FIXTURES, GOLDEN, golden_arrays, manifest, tools_env

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIGHT = {np.dtype(np.float64): 1e-12, np.dtype(np.float32): 2e-6}


def _ndev():
    import torch
    return torch.cuda.device_count()


def _flow(lib, row_ptr, col, val, x, ncols, dtype, calls=1):
    m = lib.make_csr_matrix(row_ptr, col, val, ncols)
    hw, bm = lib.create_csr_hw_matrix(m)
    hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(x), 1, hw[0].contents.nr_cols)
    r = len(row_ptr) - 1
    yv = lib.make_csr_vector(np.zeros(r, dtype))
    ys = []
    for _ in range(calls):
        lib.spmv_hw(hw, hx, yv, bm)
        ys.append(np.ctypeslib.as_array(yv.values, shape=(r,)).copy())
    lib.delete_csr_hw_matrix(hw)
    lib.free_bitmap(bm)
    lib.delete_csr_hw_x_vector(hx)
    return ys


@pytest.mark.parametrize("merge", ["gather", "reduce"])
@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("dtype,tag", DTYPES)
def test_rccl_merge_on_golden_fixtures(monkeypatch, capfd, merge, name, dtype, tag):
    monkeypatch.setenv("SPMV_NGPUS", str(_ndev()))
    monkeypatch.setenv("SPMV_HW_MERGE", merge)
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    lib = spmv_hw.load(dtype)
    _, c, row_ptr, col, val, _ = oracle.read_csr(os.path.join(GOLDEN, manifest()[name]["file"]), dtype)
    x, y_gold = golden_arrays(name, tag)
    y1, y2 = _flow(lib, row_ptr, col, val, x, c, dtype, calls=2)
    tol = TIGHT[np.dtype(dtype)]
    assert oracle.scaled_error(row_ptr, col, val, x, y_gold, y1) <= tol
    # spmv_hw accumulates (+=): the second call adds another A*x
    second = y2.astype(np.float64) - y1.astype(np.float64)
    assert oracle.scaled_error(row_ptr, col, val, x, y1.astype(np.float64), second) <= (1e-5 if dtype == np.float32 else 1e-12)
    out, err = capfd.readouterr()
    # the reference's three lines (csr_hw_wrapper.cpp:274,284-285), once per call
    assert out.count("Hardware execution time : ") == 2
    assert out.count("Result accumulation time : ") == 2
    assert out.count("Total time  : ") == 2
    assert "RCCL merge" in err  # the trace names the branch that ran
    calls = [int(c) for c in re.findall(r"(\d+) RCCL calls", err)]
    assert len(calls) == 2
    ndev = _ndev()
    if merge == "reduce":  # one ncclReduce per rank, also at one rank
        assert calls == [ndev, ndev]
    else:  # rank 0 receives every other non-empty slice, every other rank sends its own
        assert all(c <= 2 * (ndev - 1) for c in calls)
        if ndev == 1:
            assert calls == [0, 0]


@pytest.mark.parametrize("pipeline", ["1", "0"])
@pytest.mark.parametrize("merge", ["gather", "reduce", "host"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_rccl_merge_powerlaw(monkeypatch, capfd, merge, dtype, pipeline):
    """A 1M-row power-law matrix (sweep / binned plans) through each merge; host is the PCIe
    merge the RCCL branch replaces. pipeline 1 (default): y comes back in 64 pieces, each added
    in as soon as it landed; 0: one copy, every add after it (SPMV_HW_PIPELINE)."""
    monkeypatch.setenv("SPMV_NGPUS", str(_ndev()))
    monkeypatch.setenv("SPMV_HW_MERGE", merge)
    monkeypatch.setenv("SPMV_HW_PIPELINE", pipeline)
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    lib = spmv_hw.load(dtype)
    n, z = 1_000_000, 16_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    h_rp, h_col = rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32)
    h_val, h_x = val.cpu().numpy(), x.cpu().numpy()
    (y,) = _flow(lib, h_rp, h_col, h_val, h_x, n, dtype)
    ref = oracle.spmv_fp64acc(h_rp, h_col, h_val, h_x) if dtype == np.float32 else oracle.spmv_gold(h_rp, h_col, h_val, h_x)
    assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, y) <= TIGHT[np.dtype(dtype)]
    _, err = capfd.readouterr()
    assert ("RCCL merge" in err) == (merge != "host")


def test_rccl_merge_refuses_shared_gpus():
    """SPMV_HW_MERGE=gather asks for one RCCL rank per unit: more units than GPUs fails fast
    (the Part-1 error behaviour: a message and exit(1)), in a child process."""
    code = (
        "import sys, numpy as np; sys.path[:0] = [%r, %r]\n"
        "import spmv_hw\n"
        "lib = spmv_hw.load(np.float64)\n"
        "rp = np.array([0, 1, 2], np.uint32)\n"
        "m = lib.make_csr_matrix(rp, np.array([0, 1], np.uint32), np.ones(2), 2)\n"
        "lib.create_csr_hw_matrix(m)\n"
    ) % (os.path.join(ROOT, "spmv-fpga_amd"), os.path.join(ROOT, "oracle"))
    env = dict(os.environ, SPMV_NGPUS=str(_ndev() + 1), SPMV_HW_MERGE="gather")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 1
    assert "needs one unit per GPU" in p.stderr


@pytest.mark.parametrize("extra", [0, 2])
def test_auto_merge_is_host(monkeypatch, capfd, extra):
    """Automatic choice: the per-unit PCIe merge (y_fpga is host memory), with one
    unit per GPU and with virtual units sharing a GPU; y is the oracle's."""
    monkeypatch.setenv("SPMV_NGPUS", str(_ndev() + extra))
    monkeypatch.delenv("SPMV_HW_MERGE", raising=False)
    monkeypatch.setenv("SPMV_HW_TRACE", "1")
    lib = spmv_hw.load(np.float64)
    _, c, row_ptr, col, val, _ = oracle.read_csr(os.path.join(GOLDEN, manifest()["small"]["file"]), np.float64)
    x, y_gold = golden_arrays("small", "f64")
    (y,) = _flow(lib, row_ptr, col, val, x, c, np.float64)
    assert oracle.scaled_error(row_ptr, col, val, x, y_gold, y) <= 1e-12
    _, err = capfd.readouterr()
    assert "RCCL merge" not in err


@pytest.mark.parametrize("split", ["1", "0"])
def test_host_merge_pieces_of_several_units(monkeypatch, split):
    """The host merge with 3 units (virtual CUs on the box's GPU) of a 1M-row power-law matrix:
    every unit's slice comes back in pieces, the pieces are added in landing order (piece j of
    every unit, then j + 1) by 16 threads, each taking a sixteenth of every piece (split 1) or
    whole pieces (split 0); y matches the oracle and a second call adds A*x once more."""
    monkeypatch.setenv("SPMV_NGPUS", str(_ndev() + 2))
    monkeypatch.setenv("SPMV_HW_MERGE", "host")
    tools_env(monkeypatch, "SPMV_HW_ADD_SPLIT", split)
    lib = spmv_hw.load(np.float64)
    n, z = 1_000_000, 16_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=9)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    h_rp, h_col = rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32)
    h_val, h_x = val.cpu().numpy(), x.cpu().numpy()
    y1, y2 = _flow(lib, h_rp, h_col, h_val, h_x, n, np.float64, calls=2)
    ref = oracle.spmv_gold(h_rp, h_col, h_val, h_x)
    assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, y1) <= 1e-12
    assert oracle.scaled_error(h_rp, h_col, h_val, h_x, ref, y2 - y1) <= 1e-12
