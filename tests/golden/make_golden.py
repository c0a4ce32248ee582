#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/.

Inputs are written in the reference's row-sorted text format (header "rows cols nnz", then
1-based "r c v" lines, README.md:29, csr.cpp:87-136), values printed %.17g so fp64 round-trips
exactly and fp32 rounds from the same text like the reference's sscanf("%f").

Expected outputs come from the CPU oracle (oracle/csr_ref.c), cross-checked bit-exactly by the
independent numpy restatement in tests/test_oracle.py. The reference itself cannot be built in
this image (Xilinx headers absent, SURVEY.md §8c / DESIGN.md §5), so these vectors are
regression fixtures of the restatement: "parity unpinned" in the oracle's header.

Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def random_rows(rng, n, m, lengths):
    rows = []
    for i in range(n):
        k = int(min(lengths[i], m))
        cols = np.sort(rng.choice(m, size=k, replace=False)) if k else np.zeros(0, np.int64)
        vals = rng.uniform(-1.0, 1.0, size=k)
        rows.append((cols, vals))
    return rows


def write_mtx(path, n, m, rows):
    nnz = sum(len(c) for c, _ in rows)
    with open(path, "w") as f:
        f.write(f"{n} {m} {nnz}\n")
        for i, (cols, vals) in enumerate(rows):
            for c, v in zip(cols, vals):
                f.write(f"{i + 1} {int(c) + 1} {float(v):.17g}\n")
    return nnz


def fixtures():
    rng = np.random.default_rng(1)
    out = {}
    # config 1: ~1k x 1k, ~5k nnz, row length 1 + Exp(mean 4), last row non-empty
    n = m = 1000
    lens = 1 + np.floor(rng.exponential(4.0, size=n)).astype(int)
    out["small"] = (n, m, random_rows(rng, n, m, lens))
    # ~20% empty rows (never the last one)
    lens = 1 + np.floor(rng.exponential(4.0, size=n)).astype(int)
    lens[rng.random(n) < 0.2] = 0
    lens[-1] = max(lens[-1], 1)
    out["small_empty"] = (n, m, random_rows(rng, n, m, lens))
    # trailing empty rows (the reference reads uninitialised row_ptr here)
    lens = 1 + np.floor(rng.exponential(4.0, size=300)).astype(int)
    lens[-10:] = 0
    out["trail"] = (300, 400, random_rows(rng, 300, 400, lens))
    # wide: 4 column blocks of 32768 (fp32/fp64 CU<=8), 7 blocks of 16384 (CU 10/12)
    n, m = 2000, 100000
    lens = 1 + np.floor(rng.exponential(3.0, size=n)).astype(int)
    out["wide"] = (n, m, random_rows(rng, n, m, lens))
    # long rows crossing many 512-entry tiles, next to short and empty rows
    n, m = 40, 5000
    lens = rng.integers(0, 6, size=n)
    lens[3] = 3000
    lens[17] = 1100
    lens[18] = 513
    lens[-1] = 2
    out["longrow"] = (n, m, random_rows(rng, n, m, lens))
    # a single row
    out["onerow"] = (1, 700, random_rows(rng, 1, 700, [600]))
    # the 4x4 example of the reference's diagrams (images/1_matrix.svg), a..h = 1..8
    # (tests/golden/reference_diagram_kat.json); no random draws, so the fixtures above keep
    # their bytes
    with open(os.path.join(OUT, "reference_diagram_kat.json")) as f:
        ent = json.load(f)["matrix_4x4"]["entries"]
    rows = [(np.array([c for r, c, _ in ent if r == i]),
             np.array([float("abcdefgh".index(v) + 1) for r, _, v in ent if r == i])) for i in range(4)]
    out["diagram"] = (4, 4, rows)
    return out


def main():
    oracle.build()
    manifest = {}
    for name, (n, m, rows) in fixtures().items():
        path = os.path.join(OUT, f"{name}.mtx")
        nnz = write_mtx(path, n, m, rows)
        entry = {"file": f"{name}.mtx", "rows": n, "cols": m, "nnz": nnz,
                 "sha256": hashlib.sha256(open(path, "rb").read()).hexdigest()}
        for dtype, tag in ((np.float64, "f64"), (np.float32, "f32")):
            r, c, row_ptr, col, val, _ = oracle.read_csr(path, dtype)
            assert (r, c) == (n, m)
            x = oracle.init_vector_rand(c, dtype, seed=1)  # main.cpp:57-58 (libc rand, seed 1)
            y = oracle.spmv_gold(row_ptr, col, val, x)
            np.save(os.path.join(OUT, f"{name}.x.{tag}.npy"), x)
            np.save(os.path.join(OUT, f"{name}.y_gold.{tag}.npy"), y)
            entry[f"y_gold_{tag}_sha256"] = hashlib.sha256(y.tobytes()).hexdigest()
        manifest[name] = entry
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print(json.dumps({k: (v["rows"], v["cols"], v["nnz"]) for k, v in manifest.items()}))


if __name__ == "__main__":
    main()
