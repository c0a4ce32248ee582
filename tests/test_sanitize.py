"""Sanitizer builds of the library's host code (SURVEY §5 "ASan/UBSan host build"; VERDICT r3
item 3). tests/sanitize/Makefile compiles host.cpp (row partition, exchange schedule, threaded
accum_results '+=', verification, storage_overhead) and reader.cpp (the 16-thread mmap reader)
with g++ -fsanitize=address,undefined (fp64 and fp32) and -fsanitize=thread into host_check, a
small driver (tests/sanitize/host_check.cpp). This suite builds them and runs:

  * every host_check self-check under each sanitizer;
  * the reader on the golden fixtures and on generated files (CRLF, MatrixMarket banner and
    comments, unsorted rows, symmetric / skew-symmetric / pattern, trailing empty rows, malformed
    files, a 200k-entry file) with 1 and 16 threads: no sanitizer report, and the arrays equal the
    product library's spmv_read_csr (the same code without instrumentation) -- the class of
    defects SURVEY B2/B3 found in the reference's reader and accumulation (csr.cpp:115-126,
    csr_hw.cpp:1549-1553).
CPU only; no GPU, no HIP."""
import fcntl
import os
import shutil
import subprocess

import numpy as np
import pytest

import spmv_hw
from conftest import GOLDEN, ROOT, manifest

SAN = os.path.join(ROOT, "tests", "sanitize")
BUILD = os.path.join(SAN, "build")
BINS = {"asan": np.float64, "asan_f32": np.float32, "tsan": np.float64}
# verify_asan_link_order=0: a preloaded library of the environment may come before the ASan runtime
ENV = {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:halt_on_error=1:verify_asan_link_order=0",
       "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
       "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}


@pytest.fixture(scope="module")
def built():
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    # one build at a time: pytest-xdist workers that each run this module's fixture must not
    # relink a binary another worker is running
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-j3", "-C", SAN], check=True, timeout=600)
    return {k: os.path.join(BUILD, f"host_check_{k}") for k in BINS}


def _run(binary, *args, threads=None, timeout=300):
    env = dict(os.environ, **ENV)
    if threads is not None:
        env["SPMV_READ_THREADS"] = str(threads)
    p = subprocess.run([binary, *args], capture_output=True, text=True, timeout=timeout, env=env)
    report = [k for k in ("AddressSanitizer", "LeakSanitizer", "runtime error", "ThreadSanitizer") if k in p.stderr]
    assert not report, p.stderr[-4000:]
    return p


@pytest.mark.parametrize("kind", list(BINS))
@pytest.mark.parametrize("cmd", ["partition", "schedule", "accumulate", "verify"])
def test_host_checks_clean_under_sanitizer(built, kind, cmd):
    p = _run(built[kind], cmd)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.strip().endswith(f"OK {cmd}")


def _write(path, text, crlf=False):
    with open(path, "w", newline="") as f:
        f.write(text.replace("\n", "\r\n") if crlf else text)
    return path


def _generated(tmp):
    rng = np.random.default_rng(3)
    files = {}
    n, m, z = 300, 200, 2000
    r = np.sort(rng.integers(1, n - 20, z))  # last 20 rows empty
    c = rng.integers(1, m + 1, z)
    v = rng.uniform(-10, 10, z)
    body = "".join(f"{a} {b} {x:.17g}\n" for a, b, x in zip(r, c, v))
    files["plain"] = _write(os.path.join(tmp, "plain.mtx"), f"{n} {m} {z}\n" + body)
    files["crlf"] = _write(os.path.join(tmp, "crlf.mtx"), f"{n} {m} {z}\n" + body, crlf=True)
    perm = rng.permutation(z)
    ub = "".join(f"{r[k]}  {c[k]}\t{v[k]:.6e}\n" for k in perm)
    files["unsorted"] = _write(os.path.join(tmp, "unsorted.mtx"),
                               "%%MatrixMarket matrix coordinate real general\n% comment\n%\n" + f"{n} {m} {z}\n" + ub)
    lo = [(i, j) for i in range(1, 60) for j in range(1, i + 1) if rng.random() < 0.2]
    sb = "".join(f"{i} {j} {rng.uniform(-1, 1):.9g}\n" for i, j in lo)
    for sym in ("symmetric", "skew-symmetric"):
        files[sym] = _write(os.path.join(tmp, f"{sym}.mtx"),
                            f"%%MatrixMarket matrix coordinate real {sym}\n59 59 {len(lo)}\n" + sb)
    files["pattern"] = _write(os.path.join(tmp, "pattern.mtx"),
                              "%%MatrixMarket matrix coordinate pattern general\n3 4 4\n1 2\n1 4\n3 1\n3 3\n")
    files["bad_index"] = _write(os.path.join(tmp, "bad_index.mtx"), "2 2 2\n1 1 1.0\n3 1 2.0\n")
    files["bad_count"] = _write(os.path.join(tmp, "bad_count.mtx"), "2 2 3\n1 1 1.0\n2 1 2.0\n")
    files["bad_token"] = _write(os.path.join(tmp, "bad_token.mtx"), "2 2 2\n1 1 x\n2 1 2.0\n")
    files["empty"] = _write(os.path.join(tmp, "empty.mtx"), "")
    files["missing"] = os.path.join(tmp, "missing.mtx")
    nb, zb = 50_000, 200_000
    rb = np.sort(rng.integers(1, nb + 1, zb))
    cb = rng.integers(1, nb + 1, zb)
    with open(os.path.join(tmp, "big.mtx"), "w") as f:
        f.write(f"{nb} {nb} {zb}\n")
        f.write("".join(f"{a} {b} {x:.17g}\n" for a, b, x in zip(rb, cb, rng.uniform(-1, 1, zb))))
    files["big"] = os.path.join(tmp, "big.mtx")
    return files


def _load_dump(path):
    raw = open(path, "rb").read()
    n, m, z, vb = np.frombuffer(raw[:32], np.uint64)
    off = 32
    rp = np.frombuffer(raw, np.uint32, int(n) + 1, off)
    off += 4 * (int(n) + 1)
    col = np.frombuffer(raw, np.uint32, int(z), off)
    off += 4 * int(z)
    val = np.frombuffer(raw, np.float64 if vb == 8 else np.float32, int(z), off)
    return rp, col, val, int(m)


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    tmp = str(tmp_path_factory.mktemp("san_mtx"))
    out = _generated(tmp)
    for name, meta in manifest().items():
        out["golden_" + name] = os.path.join(GOLDEN, meta["file"])
    return out


@pytest.mark.parametrize("threads", [1, 16])
@pytest.mark.parametrize("kind", list(BINS))
def test_reader_clean_under_sanitizer_and_equal_to_product(built, files, tmp_path, kind, threads):
    dtype = BINS[kind]
    lib = spmv_hw.load(dtype)
    for name, path in sorted(files.items()):
        if kind == "tsan" and name != "big" and threads == 1:
            continue  # one thread has nothing to race on
        dump = str(tmp_path / f"{name}.bin")
        p = _run(built[kind], "read", path, dump, threads=threads)
        assert p.returncode == 0, (name, p.stdout + p.stderr)
        try:
            want = lib.read_csr(path)
        except RuntimeError:
            want = None
        if want is None:
            assert "READ_ERROR" in p.stdout, (name, p.stdout)
            continue
        assert "OK read" in p.stdout, (name, p.stdout)
        rp, col, val, m = _load_dump(dump)
        assert m == want[3], name
        assert np.array_equal(rp, want[0]) and np.array_equal(col, want[1]), name
        assert np.array_equal(val.view(np.uint8), np.ascontiguousarray(want[2]).view(np.uint8)), name
