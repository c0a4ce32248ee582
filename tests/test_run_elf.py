"""run.elf (restated src/main.cpp flow) on the golden .mtx inputs through the drop-in library:
the reference's own end-to-end check, "Verification PASSED!" (main.cpp:77-82)."""
import os
import subprocess

import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu
ELF = os.path.join(ROOT, "tests", "run_elf")


@pytest.mark.parametrize("name", ["small", "small_empty", "trail", "wide", "longrow", "onerow", "diagram"])
@pytest.mark.parametrize("units", ["1", "2"])
@pytest.mark.parametrize("reader", ["oracle", "fast"])
def test_run_elf_f64_passes(name, units, reader):
    extra = ["--fast-reader"] if reader == "fast" else []
    out = subprocess.run([os.path.join(ELF, "run.elf"), os.path.join(GOLDEN, f"{name}.mtx")] + extra,
                         capture_output=True, text=True, timeout=120, env=dict(os.environ, SPMV_NGPUS=units))
    assert out.returncode == 0, out.stdout + out.stderr
    for line in ("Welcome to SpMV", "Software execution time", "Matrix read time", "Total non-zeros",
                 "Hardware execution time", "Result accumulation time", "Total time",
                 "Verification PASSED!", "CSR representation"):
        assert line in out.stdout, (line, out.stdout)


@pytest.mark.parametrize("name", ["small", "small_empty", "trail"])
def test_run_elf_f32_passes(name):
    out = subprocess.run([os.path.join(ELF, "run_f32.elf"), os.path.join(GOLDEN, f"{name}.mtx")],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "Verification PASSED!" in out.stdout


DROPIN = os.path.join(ROOT, "tests", "dropin")


@pytest.mark.parametrize("name", ["small", "wide", "trail"])
@pytest.mark.parametrize("exe,ngpus,units", [("dropin_cu4.elf", None, 4), ("dropin_cu4.elf", "1", 4),
                                             ("dropin_cu12_nohint.elf", "2", 2),
                                             ("dropin_cu12_nohint.elf", None, 1)])
def test_dropin_main_runs_with_compile_time_units(name, exe, ngpus, units):
    """the main.cpp-shaped caller built against include/dropin/ runs end to end.
    CU=4 registers 4 units whatever SPMV_NGPUS says; CU=12 without the registration loops 12
    hw_matrix slots over 1 or 2 real units and reads NULL handles (storage_overhead = 0) for the
    rest, never past the array."""
    env = {k: v for k, v in os.environ.items() if k != "SPMV_NGPUS"}
    if ngpus:
        env["SPMV_NGPUS"] = ngpus
    out = subprocess.run([os.path.join(DROPIN, exe), os.path.join(GOLDEN, f"{name}.mtx")], capture_output=True,
                         text=True, timeout=120, env=env)
    assert out.returncode == 0, out.stdout + out.stderr
    assert f"library units {units}" in out.stdout
    assert "Verification PASSED!" in out.stdout
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("storage_overhead over")][0]
    assert f"{units} non-null handles" in line, line
    assert float(line.split(": ")[1].split(" MB")[0]) > 0


@pytest.mark.parametrize("name", ["small", "small_empty", "wide", "longrow"])
@pytest.mark.parametrize("merge", ["gather", "reduce"])
def test_run_elf_rccl_merge_passes(name, merge):
    """The restated main.cpp flow with spmv_hw's RCCL merge forced (one unit on the box's GPU; the
    same branch takes one unit per GPU on a multi-GPU node): "Verification PASSED!"."""
    out = subprocess.run([os.path.join(ELF, "run.elf"), os.path.join(GOLDEN, f"{name}.mtx")], capture_output=True,
                         text=True, timeout=120, env=dict(os.environ, SPMV_NGPUS="1", SPMV_HW_MERGE=merge,
                                                          SPMV_HW_TRACE="1"))
    assert out.returncode == 0, out.stdout + out.stderr
    assert "Verification PASSED!" in out.stdout
    assert "RCCL merge" in out.stderr
