"""Kernel variants through the product library's C-ABI (spmv_plan_set_variant).

VERDICT r1 item 6: the measurement-only ablations (sweep variants 54-63, blocked variant 1;
several give a wrong y by design) exist only in the tools library built with -DSPMV_ABLATIONS
(`make -C spmv-fpga_amd ablations`); the shipped library refuses them with an error code."""
import numpy as np
import pytest

import spmv_hw

pytestmark = pytest.mark.gpu


def _plan(monkeypatch, kernel, dtype=np.float64, n=50_000, z=800_000):
    monkeypatch.setenv("SPMV_HW_KERNEL", kernel)
    lib = spmv_hw.load(dtype)
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    return lib, spmv_hw.Plan.from_device(lib, rp, col, val, n), x


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_ablation_variants_are_refused(monkeypatch, dtype):
    import torch
    lib, plan, x = _plan(monkeypatch, "sweep", dtype)
    assert plan.stats()["kernel"] == 2
    y_ref = torch.empty(x.numel(), dtype=x.dtype, device="cuda")
    plan.run(x, y_ref)
    for v in range(54, 64):
        with pytest.raises(RuntimeError, match="measurement-only"):
            plan.set_variant(v)
    # the refusal leaves the plan on its previous (default) variant: same y, bit for bit up to
    # the LDS-atomic order (the sweep default is not bitwise reproducible)
    y = torch.empty_like(y_ref)
    plan.run(x, y)
    torch.cuda.synchronize()
    rel = float(((y.double() - y_ref.double()).abs().max() / y_ref.double().abs().max()).item())
    assert rel < (1e-13 if dtype == np.float64 else 1e-6)
    for v in (15, 28, 34):  # real variants are still accepted
        plan.set_variant(v)
    plan.destroy()


def test_blocked_ablation_variant_is_refused(monkeypatch):
    lib, plan, x = _plan(monkeypatch, "blocked")
    assert plan.stats()["kernel"] == 4
    with pytest.raises(RuntimeError, match="measurement-only"):
        plan.set_variant(1)
    plan.set_variant(0)
    plan.destroy()
