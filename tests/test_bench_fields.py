"""bench.py's derived fields on the CPU: `value_e2e` (2 nnz / (SpMV step +
the exchange that completes y), the reference's "Total time" = hardware + accumulation,
csr_hw_wrapper.cpp:276-285) and the parser of the reference's timing lines that the `dropin`
field reads from the drop-in child (csr_hw_wrapper.cpp:274,284-285, main.cpp:72)."""
import os
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
bench = pytest.importorskip("bench")


def _out(**kw):
    d = {"value": 400.0, "n_ranks": 8, "dist_rehearsal": False, "exchange": None}
    d.update(kw)
    return d


def test_value_e2e_one_gpu_is_the_value():
    v, form = bench.value_e2e(_out(n_ranks=1), 0.8, 160e6)
    assert v == 400.0 and "no exchange" in form["form"]


def test_value_e2e_prefers_the_library_reduce():
    ex = {"reduce_ms": 0.5, "native": {"reduce_exchange_ms": 0.2}}
    v, form = bench.value_e2e(_out(exchange=ex), 0.12, 160e6)
    assert v == pytest.approx(2 * 160e6 / (0.32e-3) / 1e9, rel=1e-3)
    assert form["exchange_ms"] == 0.2 and "library RCCL reduce" in form["exchange_src"]
    assert "with_gather" not in form
    ex["native"]["gather_exchange_ms"] = 0.05
    v2, form = bench.value_e2e(_out(exchange=ex), 0.12, 160e6)
    assert v2 == v and form["with_gather"]["value"] == pytest.approx(2 * 160e6 / (0.17e-3) / 1e9, rel=1e-3)


def test_value_e2e_falls_back_to_torch_reduce_then_to_none():
    v, form = bench.value_e2e(_out(exchange={"reduce_ms": 0.5, "native": {"error": "no RCCL"}}), 0.5, 160e6)
    assert v == pytest.approx(320.0) and "torch.distributed" in form["exchange_src"]
    v, form = bench.value_e2e(_out(exchange={"error": "boom"}), 0.5, 160e6)
    assert v is None and form["form"] == "no exchange was measured"
    v, _ = bench.value_e2e(_out(n_ranks=1, dist_rehearsal=True, exchange={"native": {"reduce_exchange_ms": 0.1}}),
                           0.4, 160e6)
    assert v == pytest.approx(640.0)


def test_reference_line_parser():
    text = ("Total non-zeros : 16. Total 1 MB transferred ( in : 0.5, out : 0.5)\n"
            "Matrix read time        : 122.253000 ms elapsed\n"
            "Hardware execution time : 0.873000 ms elapsed\n"
            "Result accumulation time : 1.854000 ms elapsed\n"
            "Total time  : 2.727000 ms elapsed\n"
            "Verification PASSED!\n"
            "Hardware execution time : 0.851000 ms elapsed\n"
            "Hardware execution time : garbled\n")
    assert bench._ref_lines(text, "Hardware execution time") == [0.873, 0.851]
    assert bench._ref_lines(text, "Matrix read time") == [122.253]
    assert bench._ref_lines(text, "Total time") == [2.727]
    assert bench._ref_lines(text, "Software execution time") == []


def test_dropin_child_is_in_the_package():
    """The drop-in run is the package's own script (no oracle import: it takes the software y
    from the bench)."""
    path = os.path.join(ROOT, "spmv-fpga_amd", "dropin_main.py")
    src = open(path).read()
    assert "import oracle" not in src and "allow_pickle=False" in src
