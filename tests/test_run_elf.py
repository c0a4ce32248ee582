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
