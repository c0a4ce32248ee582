"""CPU-side checks of the C-ABI library: it loads, exports every function include/*.h declares,
and its host-only logic (partitioning, generators' row structure, verification,
storage_overhead) behaves like the reference. No compute call touches a GPU here."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import spmv_hw
from conftest import ROOT, gpu_available

HEADERS = [os.path.join(ROOT, "include", h) for h in ("csr_hw_wrapper.h",)]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", text, flags=re.M):
            if m.group(1) not in ("if", "defined"):
                names.add(m.group(1))
    return names


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_library_exports_every_declared_symbol(dtype):
    path = spmv_hw.lib_path(dtype)
    assert os.path.exists(path), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    declared = declared_functions()
    assert len(declared) >= 20
    missing = declared - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"
    assert set(spmv_hw.EXPORTS) == declared
    lib = spmv_hw.load(dtype)
    assert lib.L.spmv_hw_value_bytes() == np.dtype(dtype).itemsize


def test_reference_names_have_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", spmv_hw.lib_path(np.float64)], check=True,
                         capture_output=True, text=True).stdout
    for name in ("create_csr_hw_matrix", "spmv_hw", "create_csr_hw_x_vector", "delete_csr_hw_matrix",
                 "storage_overhead", "verification"):
        assert re.search(rf"\bT {name}$", out, flags=re.M), name


def test_units_from_env(monkeypatch):
    lib = spmv_hw.load(np.float64)
    monkeypatch.delenv("SPMV_NGPUS", raising=False)
    assert lib.units() == 1
    monkeypatch.setenv("SPMV_NGPUS", "8")
    assert lib.units() == 8


@pytest.mark.parametrize("units", [1, 2, 3, 4, 8])
def test_partition_is_contiguous_and_nnz_balanced(units):
    lib = spmv_hw.load(np.float64)
    rp, _ = lib.powerlaw_row_ptr(200_000, 3_200_000, 65536, 4)
    b = lib.partition_rows(rp, units)
    assert b[0] == 0 and b[-1] == 200_000 and np.all(np.diff(b.astype(np.int64)) >= 0)
    per = np.diff(rp[b].astype(np.int64))
    assert per.sum() == 3_200_000
    longest = int(np.diff(rp.astype(np.int64)).max())
    assert per.max() - 3_200_000 / units <= longest + 1


def test_partition_degenerate_inputs():
    lib = spmv_hw.load(np.float64)
    rp = np.array([0, 0, 0, 5, 5], np.uint32)  # all nnz in one row
    b = lib.partition_rows(rp, 3)
    assert b[0] == 0 and b[-1] == 4 and np.all(np.diff(b.astype(np.int64)) >= 0)
    rp = np.zeros(1, np.uint32)  # zero rows
    assert list(lib.partition_rows(rp, 2)) == [0, 0, 0]


def test_powerlaw_row_ptr_exact_and_heavy_tailed():
    lib = spmv_hw.load(np.float64)
    n, z = 1_000_000, 16_000_000
    rp, s = lib.powerlaw_row_ptr(n, z, 65536, 4)
    lens = np.diff(rp.astype(np.int64))
    assert rp[-1] == z and lens.min() >= 1 and lens.max() <= 65536
    assert 7.5 < s < 9.0
    # Pareto(alpha=2) tail: P(l >= k) ~ (s/k)^2
    k = 128
    assert abs((lens >= k).mean() / (s / k) ** 2 - 1) < 0.15
    rp2, s2 = lib.powerlaw_row_ptr(n, z, 65536, 4)
    assert np.array_equal(rp, rp2) and s == s2  # deterministic


def test_powerlaw_rejects_impossible_request():
    lib = spmv_hw.load(np.float64)
    with pytest.raises(RuntimeError):
        lib.powerlaw_row_ptr(10, 5, 16, 1)  # fewer nnz than rows


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_verification_semantics(dtype, capfd):
    """csr_hw.cpp:1571-1590: abs threshold 1e-5, NaN is an error."""
    lib = spmv_hw.load(dtype)
    a = np.array([1.0, 2.0, 3.0, 4.0], dtype)
    assert lib.verification(a, a.copy()) == 0
    b = a.copy()
    b[1] += dtype(2e-5)
    b[2] = np.nan
    assert lib.verification(a, b) == 1
    assert "Total errors : 2" in capfd.readouterr().out


def test_storage_overhead_uses_64bit_sums():
    """csr_hw.cpp:1401-1409 with the 32-bit overflow fixed."""
    lib = spmv_hw.load(np.float64)
    m = lib.csr_hw_matrix()
    nr_ci = (spmv_hw.IndexType * 1)(40_000_000)
    nr_val = (spmv_hw.IndexType * 1)(80_000_000)
    m.nr_ci = ctypes.cast(nr_ci, ctypes.POINTER(spmv_hw.IndexType))
    m.nr_val = ctypes.cast(nr_val, ctypes.POINTER(spmv_hw.IndexType))
    m.blocks = 1
    mb = lib.storage_overhead(ctypes.pointer(m))
    expect = (5 * 32 + 120_000_000 * 128) / (8.0 * 1024 * 1024)
    assert mb == pytest.approx(expect, rel=1e-12)


DROPIN_TU = r"""
// Stand-in for the reference's util.h/csr.h as a caller would have them: a class-typed
// IndexType of ap_uint<32>'s size and the csr_* structs in the reference's field order.
#include <cstdint>
#include <cstdio>
struct IndexType { uint32_t v; IndexType() = default; IndexType(uint32_t x) : v(x) {} operator uint32_t() const { return v; } };
typedef double ValueType;
struct BusDataType { uint64_t w[2]; };
#define INDEX_TYPE_BIT_WIDTH 32
#define VALUE_TYPE_BIT_WIDTH 64
#define BUS_BIT_WIDTH 128
typedef struct csr_header { IndexType nr_rows, nr_cols, nr_nzeros; int blocks; } csr_header;
typedef struct csr_matrix { IndexType *row_ptr; IndexType *col_ind; ValueType *values;
                            IndexType nr_nzeros, nr_rows, nr_cols; char *Filename; } csr_matrix;
typedef struct csr_vector { ValueType *values; IndexType nr_values; } csr_vector;
// --- the replacement src/csr_hw_wrapper.h of INTEGRATION.md ---
#define SPMV_USE_CALLER_CSR_TYPES
#include "spmv_mi355x.h"
static_assert(sizeof(IndexType) == 4, "ap_uint<32> layout");
int main() {
    csr_matrix m{}; csr_hw_matrix **hw = nullptr; bool **bm = nullptr; csr_hw_vector *hx = nullptr;
    csr_vector x{}, y{};
    if (std::getenv("RUN")) {   // never executed in the CPU test: linking is what is checked
        create_csr_hw_matrix(&m, &hw, &bm);
        create_csr_hw_x_vector(&hx, &x, hw[0]->blocks, hw[0]->nr_cols);
        spmv_hw(hw, hx, &y, bm);
        std::printf("%d %f\n", verification(y.nr_values, y.values, y.values, 0), (double)storage_overhead(hw[0]));
        IndexType bounds[2];  // a by-value count in the caller's IndexType: converted to the ABI's uint32_t
        std::printf("%d\n", spmv_partition_rows(m.row_ptr, m.nr_rows, 1, bounds));
        delete_csr_hw_matrix(hw); std::free(bm); delete_csr_hw_x_vector(hx);
    }
    return 0;
}
"""


def test_dropin_header_compiles_and_links_against_caller_types(tmp_path):
    """the reference's sources keep their own csr_* types (class-typed
    IndexType) and link the C-ABI library by name."""
    src = tmp_path / "dropin.cpp"
    src.write_text("#include <cstdlib>\n" + DROPIN_TU)
    exe = tmp_path / "dropin"
    lib_dir = os.path.dirname(spmv_hw.lib_path(np.float64))
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(exe), "-L", lib_dir, "-lspmv_hw_f64", f"-Wl,-rpath,{lib_dir}"], check=True)
    assert exe.exists()


def test_dropin_header_with_a_plain_uint32_index_type(tmp_path):
    """a caller whose IndexType is a plain uint32_t typedef (not a class) defines
    SPMV_USE_CALLER_CSR_TYPES too; the caller-typed verification forward must not clash with the
    C-ABI declaration, and the by-value counts must take its values unchanged."""
    tu = DROPIN_TU.replace(
        "struct IndexType { uint32_t v; IndexType() = default; IndexType(uint32_t x) : v(x) {} "
        "operator uint32_t() const { return v; } };", "typedef uint32_t IndexType;")
    assert "typedef uint32_t IndexType;" in tu
    src = tmp_path / "dropin_u32.cpp"
    src.write_text("#include <cstdlib>\n" + tu)
    exe = tmp_path / "dropin_u32"
    lib_dir = os.path.dirname(spmv_hw.lib_path(np.float64))
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src),
                    "-o", str(exe), "-L", lib_dir, "-lspmv_hw_f64", f"-Wl,-rpath,{lib_dir}"], check=True)
    assert exe.exists()


def test_part2_argument_errors_return_codes_without_a_gpu():
    """Part 2 reports bad arguments through its return code and spmv_hw_last_error() (the
    reference has no error channel; Part 1 exits instead). None of these reach a HIP call."""
    lib = spmv_hw.load(np.float64)
    L = lib.L
    cases = [
        (lambda: L.spmv_plan_create_device(None, 0, 4, 4, 0, None, None, None, None), "null argument"),
        (lambda: L.spmv_plan_run(None, None, None, None), "null plan"),
        (lambda: L.spmv_plan_run_graph(None, None, None, 1, None), "iters"),
        (lambda: L.spmv_plan_get_stats(None, None), "null argument"),
        (lambda: L.spmv_plan_set_variant(None, 0), "bad arguments"),
        (lambda: L.spmv_plan_set_timing(None, 1), "null plan"),
        (lambda: L.spmv_partition_rows(None, 0, 1, None), "bad arguments"),
    ]
    for call, msg in cases:
        assert call() == 1
        assert msg in L.spmv_hw_last_error().decode()
    rp = np.array([0, 1], np.uint32)
    bounds = np.zeros(1, np.uint32)
    assert L.spmv_partition_rows(rp.ctypes.data_as(ctypes.POINTER(spmv_hw.IndexType)), 1, 0,
                                 bounds.ctypes.data_as(ctypes.POINTER(spmv_hw.IndexType))) == 1


DROPIN = os.path.join(ROOT, "tests", "dropin")


def _dropin_build():
    subprocess.run(["make", "-s", "-C", DROPIN], check=True)


def test_dropin_forwards_build_main_cpp_include_list_on_cpu():
    """VERDICT r1 item 4 / ADVICE r1: include/dropin/ forwards spmv.h, csr_hw.h, csr_hw_wrapper.h
    and sds_lib.h, so a main.cpp with the reference's include list (main.cpp:8-14) and caller-side
    util.h / csr.h (class-typed IndexType, -DCU) compiles with -Werror and links. The compile-time
    ComputeUnits reaches the library before main() (spmv_hw_set_units); without the hint the
    count is SPMV_NGPUS. With no GPU the library stops loudly at create_csr_hw_matrix."""
    _dropin_build()
    fixture = os.path.join(ROOT, "tests", "golden", "small.mtx")
    env = {k: v for k, v in os.environ.items() if k != "SPMV_NGPUS"}
    for exe, ngpus, units in (("dropin_cu4.elf", None, 4), ("dropin_cu4.elf", "2", 4),
                              ("dropin_cu12_nohint.elf", "2", 2), ("dropin_cu12_nohint.elf", None, 1)):
        e = dict(env, SPMV_NGPUS=ngpus) if ngpus else env
        out = subprocess.run([os.path.join(DROPIN, exe), fixture], capture_output=True, text=True, env=e,
                             timeout=60)
        assert f"library units {units}" in out.stdout, (exe, ngpus, out.stdout)
        if not gpu_available():
            assert out.returncode == 1
            assert "no HIP device available" in out.stderr
    syms = subprocess.run(["nm", "-C", os.path.join(DROPIN, "dropin_cu4.elf")], capture_output=True,
                          text=True, check=True).stdout
    assert "spmv_hw_set_units" in syms


def test_set_units_overrides_env(monkeypatch):
    lib = spmv_hw.load(np.float64)
    monkeypatch.setenv("SPMV_NGPUS", "3")
    try:
        assert lib.set_units(5) == 0
        assert lib.units() == 5
        assert lib.set_units(0) == 5
        assert lib.units() == 3
    finally:
        lib.set_units(0)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_measurement_ablations_are_not_in_the_product_library_symbols(dtype):
    """the ablation kernels (ABL != 0 instantiations) are compiled only into the
    tools library (-DSPMV_ABLATIONS); the product .so has no such instantiation."""
    out = subprocess.run(["nm", "-C", spmv_hw.lib_path(dtype)], capture_output=True, text=True, check=True).stdout
    sweeps = [ln for ln in out.splitlines() if "k_spmv_sweep_packed<" in ln]
    assert sweeps
    for ln in sweeps:  # template args <V, T, Q, NT, LAG, ABL, A>: ABL must be 0
        args = ln.split("k_spmv_sweep_packed<", 1)[1].split(">", 1)[0].split(", ")
        assert args[5] == "0", ln
    blocked = [ln for ln in out.splitlines() if "k_blocked_partials<" in ln]
    for ln in blocked:  # <V, VF, XLDS, ABL>
        args = ln.split("k_blocked_partials<", 1)[1].split(">", 1)[0].split(", ")
        assert args[3] == "0", ln


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_deterministic_kernel_ships_only_its_ordered_forms(dtype):
    """k_spmv_sweep_turn<V, T, Q, PK, ORD, A>: the product library holds ORD 0 and 1 (ordered
    adds); ORD 2 / 3 (the same pipeline without ordering, ablations 51 / 52) exist only in the
    tools library."""
    out = subprocess.run(["nm", "-C", spmv_hw.lib_path(dtype)], capture_output=True, text=True, check=True).stdout
    turns = [ln for ln in out.splitlines() if "k_spmv_sweep_turn<" in ln]
    assert turns
    ords = {ln.split("k_spmv_sweep_turn<", 1)[1].split(">", 1)[0].split(", ")[4] for ln in turns}
    assert ords == {"0"}, ords  # ORD 1 (variant 91) is a measurement variant: tools library


# what spmv_plan_set_variant accepts in the product library, per kernel (plan.cpp product_variant)
PRODUCT_VARIANTS = {"tiles": {0}, "gold": {0}, "sweep": {0, 28, 94}, "fpga": {0}, "blocked": {0},
                    "slices": {0}, "binned": {0, 1, 2}}
KERNEL_IDS = {"tiles": 0, "gold": 1, "sweep": 2, "fpga": 3, "blocked": 4, "slices": 5, "binned": 6}


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", sorted(PRODUCT_VARIANTS))
def test_product_refuses_every_measurement_variant(monkeypatch, kernel):
    """the product library's variant surface is the default, the deterministic
    sweep (94) and the binned kernel's test rebases (1 / 2); every other variant in 0..127 is
    refused with "tools library only" (or "bad arguments" past 63), on a plan of every kernel.
    The plan still runs afterwards and matches the oracle."""
    import torch
    import oracle
    monkeypatch.setenv("SPMV_HW_KERNEL", kernel)
    lib = spmv_hw.load(np.float64, ablations=False)
    n, z = 20_000, 320_000
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
    x = spmv_hw.gen_vector(lib, n, seed=6)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n)
    assert plan.stats()["kernel"] == KERNEL_IDS[kernel]
    accepted = set()
    for v in range(128):
        try:
            plan.set_variant(v)
            accepted.add(v)
        except RuntimeError as e:
            assert "tools library only" in str(e) or (v > 63 and "bad arguments" in str(e)), (v, str(e))
    assert accepted == PRODUCT_VARIANTS[kernel], sorted(accepted)
    plan.set_variant(0)
    y = torch.full((n,), float("nan"), dtype=x.dtype, device="cuda")
    plan.run(x, y)
    torch.cuda.synchronize()
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    assert oracle.scaled_error(r, c, h[2], h[3], ref, y.cpu().numpy()) <= 1e-12
    plan.destroy()


def test_product_variant_table_matches_the_source():
    """The CPU side of the same check: plan.cpp's product_variant lists exactly the variants above
    (the measurement variants' kernel forms are compiled only under -DSPMV_ABLATIONS)."""
    src = open(os.path.join(ROOT, "spmv-fpga_amd", "csrc", "plan.cpp")).read()
    body = src[src.index("bool product_variant(int kernel, int variant)"):]
    body = body[:body.index("\n}\n")]
    assert "variant == 0" in body
    assert "kKernelSweep)\n        return variant == 28 || variant == kSweepTurnOrdered;" in body
    assert "kKernelBinned)\n        return variant == 1 || variant == 2;" in body
    assert body.rstrip().endswith("return false;")
    sweep = open(os.path.join(ROOT, "spmv-fpga_amd", "csrc", "sweep.hip")).read()
    head = sweep[:sweep.index("case 15: PK(2, 0); break;")]
    assert head.rfind("#ifdef SPMV_ABLATIONS") > head.rfind("#endif")


DOCUMENTED_ENV = {"SPMV_NGPUS", "SPMV_HW_MERGE", "SPMV_HW_KERNEL", "SPMV_FPGA_VF", "SPMV_FPGA_BLOCK",
                  "SPMV_SLICE_ACC", "SPMV_SWEEP_DETERMINISTIC", "SPMV_SWEEP_DELTA", "SPMV_SWEEP_XCC_BIAS",
                  "SPMV_BIN_ROW_LIMIT", "SPMV_READ_THREADS", "SPMV_HW_TRACE", "SPMV_HW_PREFAULT",
                  "SPMV_HW_PIPELINE", "SPMV_HW_STREAM"}


def test_product_reads_only_the_documented_switches():
    """outside the tools build (ablation_env, -DSPMV_ABLATIONS) the library reads
    exactly the environment switches INTEGRATION.md documents; the tools-only ones are read
    through ablation_env only, and INTEGRATION.md names every product switch."""
    from conftest import TOOLS_ONLY_ENV
    csrc = os.path.join(ROOT, "spmv-fpga_amd", "csrc")
    direct, tools = set(), set()
    for f in os.listdir(csrc):
        text = open(os.path.join(csrc, f)).read()
        direct |= set(re.findall(r'std::getenv\("([A-Z0-9_]+)"\)', text))
        tools |= set(re.findall(r'ablation_env\("([A-Z0-9_]+)"\)', text))
        # the one getenv of ablation_env itself sits under #ifdef SPMV_ABLATIONS
        for m in re.finditer(r"\bgetenv\((?!\")", text):
            head = text[:m.start()]
            assert head.rfind("#ifdef SPMV_ABLATIONS") > head.rfind("#endif"), f
    assert direct == DOCUMENTED_ENV
    assert tools == set(TOOLS_ONLY_ENV)
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert all(f"`{k}" in doc for k in DOCUMENTED_ENV)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_product_library_carries_no_tools_only_switch_names(dtype):
    """The product build drops the tools-only switch names altogether (ablation_env returns null
    there, so the names are never referenced); the tools build keeps them."""
    from conftest import TOOLS_ONLY_ENV
    blob = open(spmv_hw.lib_path(dtype), "rb").read()
    assert not [k for k in TOOLS_ONLY_ENV if k.encode() + b"\0" in blob]
    tools = spmv_hw.lib_path(dtype, ablations=True)
    if os.path.exists(tools):
        tblob = open(tools, "rb").read()
        assert all(k.encode() + b"\0" in tblob for k in TOOLS_ONLY_ENV)
