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


@pytest.mark.parametrize("gpus,backend", [(2, "gloo"), (1, "nccl")])
def test_distributed_cg_example_converges(gpus, backend):
    """examples/cg_dist.py: CG over row slices, one process per rank, the dot products as
    all-reduces and p all-gathered every iteration (the dependent form); two gloo ranks share
    the box's GPU, and one RCCL rank runs the nccl path. Converges like the one-GPU example."""
    cmd = [sys.executable, os.path.join(ROOT, "examples", "cg_dist.py"), "--gpus", str(gpus), "--backend", backend,
           "--grid", "300", "--iters", "150", "--timeout", "90"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stdout + out.stderr
    res = float(out.stdout.split("relative residual")[1].split()[0])
    assert res < 1e-8, out.stdout
    assert f"ranks={gpus} backend={backend}" in out.stdout
