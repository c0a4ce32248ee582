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


# environment switches read only by the tools build (make -C spmv-fpga_amd ablations,
# -DSPMV_ABLATIONS; csrc/spmv_host.hpp ablation_env): they force layouts and schedules the
# automatic choice takes on other matrices, or that were measured and not kept. The product
# library ignores them (tests/test_abi.py checks which switches it reads).
TOOLS_ONLY_ENV = ("SPMV_TILE_XCD", "SPMV_TILE_NARROW", "SPMV_TILE_CLUSTER", "SPMV_SWEEP_THREADS",
                  "SPMV_BIN_XCC_BIAS", "SPMV_BIN_DELTA", "SPMV_BIN_PROD_SKEW", "SPMV_SLICE_NARROW",
                  "SPMV_SWEEP_ACC", "SPMV_SWEEP_SPLIT", "SPMV_SWEEP_PIECES", "SPMV_SWEEP_COMBINE",
                  "SPMV_SWEEP_PACKED", "SPMV_SWEEP_LANE_ORDER", "SPMV_HW_BLOCKING_SYNC",
                  "SPMV_HW_PIECES", "SPMV_HW_ADD_SPLIT", "SPMV_HW_ADD_THREADS", "SPMV_GRAPH_FORM",
                  "SPMV_BEHIND_BLOCKS", "SPMV_BEHIND_ROWS", "SPMV_HW_DIRECT", "SPMV_HW_PIECE_SHAPE",
                  "SPMV_SWEEP_ROUNDS")


def tools_env(monkeypatch, name, value):
    """Sets a tools-only switch and selects the tools build for the libraries this test loads
    (spmv_hw.load with env SPMV_HW_ABLATIONS=1): the same kernels, plus the switch."""
    assert name in TOOLS_ONLY_ENV, name
    monkeypatch.setenv(name, value)
    monkeypatch.setenv("SPMV_HW_ABLATIONS", "1")
