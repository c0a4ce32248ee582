"""examples/cg.py: CG with the plan as operator converges on an SPD matrix, eagerly and with
the iteration captured in a graph (same iterates up to rounding)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graph", [False, True])
def test_cg_example_converges(graph):
    cmd = [sys.executable, os.path.join(ROOT, "examples", "cg.py"), "--grid", "300", "--iters", "150"]
    if graph:
        cmd.append("--graph")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    res = float(out.stdout.split("relative residual")[1].split()[0])
    assert res < 1e-8, out.stdout
