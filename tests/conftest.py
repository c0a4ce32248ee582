"""Shared test setup: paths, the `gpu` marker, fixture loaders."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spmv-fpga_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box only)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_arrays(name, tag):
    x = np.load(os.path.join(GOLDEN, f"{name}.x.{tag}.npy"), allow_pickle=False)
    y = np.load(os.path.join(GOLDEN, f"{name}.y_gold.{tag}.npy"), allow_pickle=False)
    return x, y


FIXTURES = sorted(manifest().keys())
DTYPES = [(np.float64, "f64"), (np.float32, "f32")]
