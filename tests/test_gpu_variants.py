"""Kernel variants through the C-ABI (spmv_plan_set_variant).

VERDICT r1 item 6 / r4 item 5: the product library accepts only the plan's default (0, and the
sweep's 28), the deterministic sweep (94) and the binned test rebases (1 / 2); every performance
experiment and measurement-only ablation (several give a wrong y by design) exists only in the
tools library built with -DSPMV_ABLATIONS (`make -C spmv-fpga_amd ablations`), which these tests
load for them. tests/test_abi.py checks the product's refusals kernel by kernel."""
import numpy as np
import pytest

import spmv_hw
from conftest import tools_env

pytestmark = pytest.mark.gpu


def _plan(monkeypatch, kernel, dtype=np.float64, n=50_000, z=800_000, ablations=None):
    monkeypatch.setenv("SPMV_HW_KERNEL", kernel)
    lib = spmv_hw.load(dtype, ablations=ablations)
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    return lib, spmv_hw.Plan.from_device(lib, rp, col, val, n), x


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sweep_ablation_variants_are_refused(monkeypatch, dtype):
    import torch
    lib, plan, x = _plan(monkeypatch, "sweep", dtype, ablations=False)
    assert plan.stats()["kernel"] == 2
    y_ref = torch.empty(x.numel(), dtype=x.dtype, device="cuda")
    plan.run(x, y_ref)
    for v in list(range(51, 64)) + [15, 34, 35, 91]:
        with pytest.raises(RuntimeError, match="tools library only"):
            plan.set_variant(v)
    # the refusal leaves the plan on its previous (default) variant: same y, bit for bit up to
    # the LDS-atomic order (the sweep default is not bitwise reproducible)
    y = torch.empty_like(y_ref)
    plan.run(x, y)
    torch.cuda.synchronize()
    rel = float(((y.double() - y_ref.double()).abs().max() / y_ref.double().abs().max()).item())
    assert rel < (1e-13 if dtype == np.float64 else 1e-6)
    for v in (0, 28, 94, 28):  # the default and the deterministic kernel are accepted
        plan.set_variant(v)
    plan.destroy()
    _, tplan, _ = _plan(monkeypatch, "sweep", dtype, ablations=True)
    for v in (15, 28, 34, 91):  # the measurement variants: tools library
        tplan.set_variant(v)
    tplan.destroy()


def test_blocked_ablation_variant_is_refused(monkeypatch):
    lib, plan, x = _plan(monkeypatch, "blocked", ablations=False)
    assert plan.stats()["kernel"] == 4
    with pytest.raises(RuntimeError, match="tools library only"):
        plan.set_variant(1)
    plan.set_variant(0)
    plan.destroy()


# ---- deterministic sweep: env SPMV_SWEEP_DETERMINISTIC=1 ----

def _det_plan(monkeypatch, lib, rp, col, val, n):
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    monkeypatch.setenv("SPMV_SWEEP_DETERMINISTIC", "1")
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    monkeypatch.delenv("SPMV_SWEEP_DETERMINISTIC")
    return plan


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_deterministic_sweep_is_bitwise_reproducible(monkeypatch, dtype):
    """1M-row power-law matrix (16M nnz): five runs of one plan and a run of a second plan built
    from the same CSR give the same bits, and y meets the oracle (spmv_gold, csr.cpp:184-194)."""
    import torch
    import oracle
    lib = spmv_hw.load(dtype)
    n, z = 1_000_000, 16_000_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = _det_plan(monkeypatch, lib, rp, col, val, n)
    assert plan.stats()["kernel"] == 2 and plan.stats()["format"] & 2
    ys = []
    for _ in range(5):
        y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        ys.append(y)
    plan2 = _det_plan(monkeypatch, lib, rp, col, val, n)
    y2 = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan2.run(x, y2)
    torch.cuda.synchronize()
    ref_bits = ys[0].cpu().numpy().view(np.uint8)
    for y in ys[1:] + [y2]:
        assert np.array_equal(y.cpu().numpy().view(np.uint8), ref_bits)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    err = oracle.scaled_error(r, c, h[2], h[3], ref, ys[0].cpu().numpy())
    assert err <= (1e-12 if dtype == np.float64 else 2e-6), err
    plan.destroy()
    plan2.destroy()


@pytest.mark.parametrize("shape", ["skewed", "empty_rows", "few_rows"])
def test_deterministic_sweep_edge_shapes(monkeypatch, shape):
    """Segments with empty rows, panels with fewer rows than waves, one very long row."""
    import torch
    import oracle
    lib = spmv_hw.load(np.float64)
    rng = np.random.default_rng(7)
    n = {"skewed": 60_000, "empty_rows": 80_000, "few_rows": 10}[shape]
    m = 2_000_000
    if shape == "skewed":
        lens = rng.integers(1, 20, n)
        lens[123] = 300_000
    elif shape == "empty_rows":
        lens = rng.integers(0, 30, n) * (rng.random(n) < 0.4)
    else:
        lens = rng.integers(1, 5000, n)
    rp = np.zeros(n + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    col = np.concatenate([np.sort(rng.choice(m, int(k), replace=False)) for k in lens]).astype(np.uint32)
    val = rng.uniform(-1, 1, len(col))
    x = rng.uniform(0, 1, m)
    t = lambda a: torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).cuda()
    plan = _det_plan(monkeypatch, lib, t(rp.astype(np.uint32)), t(col), t(val), m)
    assert plan.stats()["kernel"] == 2
    y = torch.full((n,), float("nan"), dtype=torch.float64, device="cuda")
    plan.run(t(x), y)
    torch.cuda.synchronize()
    ref = oracle.spmv_gold(rp.astype(np.uint32), col, val, x)
    assert oracle.scaled_error(rp.astype(np.uint32), col, val, x, ref, y.cpu().numpy()) <= 1e-12
    plan.destroy()


# ---- the deterministic kernel (k_spmv_sweep_turn) as a variant of any sweep plan: 91 = the
# SPMV_SWEEP_DETERMINISTIC=1 form, 94 = its hand-over after the adds complete ----

@pytest.mark.parametrize("variant", [91, 94])
@pytest.mark.parametrize("n,z,dtype", [(1_000_000, 16_000_000, np.float64),
                                       (1_000_000, 16_000_000, np.float32),
                                       (3_000_000, 48_000_000, np.float64)])
def test_turn_sweep_is_bitwise_reproducible(monkeypatch, variant, n, z, dtype):
    """Both turn variants: five runs give the same bits and y meets the oracle. The 1M-row
    matrix cuts its panels into column pieces (partials + k_sweep_combine), the 3M-row one runs
    whole panels."""
    import torch
    import oracle
    monkeypatch.setenv("SPMV_HW_KERNEL", "sweep")
    lib = spmv_hw.load(dtype, ablations=variant == 91)  # 91: a measurement variant (tools library)
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    assert plan.stats()["kernel"] == 2 and plan.stats()["format"] & 2
    plan.set_variant(variant)
    ys = []
    for _ in range(5):
        y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
        plan.run(x, y)
        ys.append(y)
    torch.cuda.synchronize()
    ref_bits = ys[0].cpu().numpy().view(np.uint8)
    for y in ys[1:]:
        assert np.array_equal(y.cpu().numpy().view(np.uint8), ref_bits)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    err = oracle.scaled_error(r, c, h[2], h[3], ref, ys[0].cpu().numpy())
    assert err <= (1e-12 if dtype == np.float64 else 2e-6), err
    plan.destroy()


# ---- binned pass 2 past 2^31 / 2^32 entries without a 2^31-entry matrix ----

@pytest.mark.parametrize("delta", ["1", "0"], ids=["row_deltas", "u16_rows"])
@pytest.mark.parametrize("variant", [1, 2], ids=["straddle_2^31", "straddle_2^32"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_binned_segment_offsets_past_2_31(monkeypatch, dtype, variant, delta):
    """Session bn5 (round 2) faulted (hipErrorIllegalAddress) on a 2.2e9-entry fp32 slice:
    k_bin_acc reads its segment bounds with readlane, which returns a signed int, so a low word
    >= 2^31 sign-extended into the high word of the 64-bit offset. Variants 1 / 2 rebase the
    segment offsets by ~2^31 / ~2^32 (and the product / row arrays the other way: same
    addresses), so half the segments lie past the boundary; y must match the oracle."""
    import torch
    import oracle
    if delta == "0":  # u16 rows: a layout only the tools library forces (the product takes row deltas)
        tools_env(monkeypatch, "SPMV_BIN_DELTA", delta)
    lib, plan, x = _plan(monkeypatch, "binned", dtype, n=200_000, z=3_200_000)
    st = plan.stats()
    assert st["kernel"] == 6 and bool(st["format"] & 32) == (delta == "1")
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, 200_000, 200_000, 3_200_000, seed=4)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    plan.set_variant(variant)
    y = torch.full((200_000,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    plan.run(x, y)
    torch.cuda.synchronize()
    err = oracle.scaled_error(r, c, h[2], h[3], ref, y.cpu().numpy())
    assert err <= (1e-12 if dtype == np.float64 else 2e-6), err
    with pytest.raises(RuntimeError, match="tools library only" if delta == "1" else "binned variants are 0-7"):
        plan.set_variant(8)
    plan.set_variant(0)
    plan.destroy()


@pytest.mark.parametrize("variant", [3, 4, 5, 6, 7], ids=["plain_stores", "plain_loads", "plain_both", "nt_stores",
                                                          "mirrored"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_binned_pass1_cache_policy_variants(monkeypatch, dtype, variant):
    """Binned variants 3-6 (tools library) change only pass 1's cache policy (temporal product
    stores / entry loads / both; 6: non-temporal stores), 7 where the products go (mirrored:
    stored down the array, read back there by pass 2): y matches the oracle as with the default."""
    import torch
    import oracle
    lib, plan, x = _plan(monkeypatch, "binned", dtype, n=200_000, z=3_200_000, ablations=True)
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, 200_000, 200_000, 3_200_000, seed=4)
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    plan.set_variant(variant)
    y = torch.full((200_000,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    err = oracle.scaled_error(r, c, h[2], h[3], ref, y.cpu().numpy())
    assert err <= (1e-12 if dtype == np.float64 else 2e-6), err
    plan.destroy()
