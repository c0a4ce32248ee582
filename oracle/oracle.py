"""ctypes front-end of the CPU oracle (oracle/csr_ref.c). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as
the checker. Parity status: "parity unpinned" (see csr_ref.c header and DESIGN.md §5).

Each function names the reference code it restates (euroexa/spmv-fpga, src/...).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS: dict = {}

_u32p = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")


def build() -> None:
    """Compile liboracle_f64.so / liboracle_f32.so with gcc (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(dtype=np.float64) -> ctypes.CDLL:
    dtype = np.dtype(dtype)
    key = dtype.str
    if key in _LIBS:
        return _LIBS[key]
    name = {np.dtype(np.float64): "liboracle_f64.so", np.dtype(np.float32): "liboracle_f32.so"}[dtype]
    path = os.path.join(HERE, name)
    if not os.path.exists(path):
        build()
    L = ctypes.CDLL(path)
    vp = np.ctypeslib.ndpointer(dtype=dtype, flags="C_CONTIGUOUS")
    cval = ctypes.c_double if dtype == np.float64 else ctypes.c_float
    u32 = ctypes.c_uint32
    L.oracle_read_csr_header.argtypes = [ctypes.c_char_p, ctypes.POINTER(u32), ctypes.POINTER(u32),
                                         ctypes.POINTER(u32), u32, ctypes.POINTER(ctypes.c_int)]
    L.oracle_read_csr_matrix.argtypes = [ctypes.c_char_p, u32, u32, _u32p, _u32p, vp]
    L.oracle_srand.argtypes = [ctypes.c_uint]
    L.oracle_init_vector_rand.argtypes = [vp, u32, cval]
    L.oracle_spmv_gold.argtypes = [u32, _u32p, _u32p, vp, vp, vp]
    L.oracle_spmv_gold_rows.argtypes = [u32, u32, _u32p, _u32p, vp, vp, vp]
    L.oracle_spmv_fp64acc.argtypes = [u32, _u32p, _u32p, vp, vp, vp]
    L.oracle_spmv_fpga_order.argtypes = [u32, u32, _u32p, _u32p, vp, vp, vp, u32, ctypes.c_int]
    L.oracle_verification_errors.argtypes = [u32, vp, vp]
    L.oracle_verification_errors.restype = ctypes.c_long
    L.oracle_abs_spmv.argtypes = [u32, _u32p, _u32p, vp, vp,
                                  np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")]
    assert L.oracle_value_bytes() == dtype.itemsize
    _LIBS[key] = L
    return L


def read_csr(path: str, dtype=np.float64, cols_div_blocks: int = 32768):
    """csr.cpp:10-46 + :87-136 -> (nr_rows, nr_cols, row_ptr, col_ind, values, blocks)."""
    L = lib(dtype)
    r, c, z, b = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int()
    rc = L.oracle_read_csr_header(path.encode(), ctypes.byref(r), ctypes.byref(c), ctypes.byref(z),
                                  cols_div_blocks, ctypes.byref(b))
    if rc:
        raise IOError(f"read_csr_header({path}) failed: {rc}")
    row_ptr = np.zeros(r.value + 1, np.uint32)
    col = np.zeros(z.value, np.uint32)
    val = np.zeros(z.value, dtype)
    rc = L.oracle_read_csr_matrix(path.encode(), r.value, z.value, row_ptr, col, val)
    if rc:
        raise IOError(f"read_csr_matrix({path}) failed: {rc}")
    return r.value, c.value, row_ptr, col, val, b.value


def init_vector_rand(n: int, dtype=np.float64, seed: int | None = 1, vmax: float = 1.0):
    """csr.cpp:170-179 (libc rand(); the reference never seeds -> seed 1)."""
    L = lib(dtype)
    if seed is not None:
        L.oracle_srand(seed)
    x = np.zeros(n, dtype)
    L.oracle_init_vector_rand(x, n, vmax)
    return x


def spmv_gold(row_ptr, col, val, x):
    """csr.cpp:184-194: y[i] = sum_j val[j]*x[col[j]] accumulated from 0 in CSR order."""
    dtype = val.dtype
    n = len(row_ptr) - 1
    y = np.zeros(n, dtype)
    lib(dtype).oracle_spmv_gold(n, _c(row_ptr, np.uint32), _c(col, np.uint32), _c(val, dtype),
                                _c(x, dtype), y)
    return y


def spmv_fp64acc(row_ptr, col, val, x):
    """spmv_gold's products (csr.cpp:190, rounded to the value type) summed in fp64 in CSR order,
    rounded once per row: the arithmetic of the kernels that accumulate fp32 in fp64 up to
    reassociation. The tight fp32 checker where spmv_gold's fp32 running sum is the loose side;
    equal to spmv_gold for fp64."""
    dtype = val.dtype
    n = len(row_ptr) - 1
    y = np.zeros(n, dtype)
    lib(dtype).oracle_spmv_fp64acc(n, _c(row_ptr, np.uint32), _c(col, np.uint32), _c(val, dtype),
                                   _c(x, dtype), y)
    return y


def spmv_gold_rows(row_ptr, col, val, x, row_begin: int, row_end: int, out=None):
    dtype = val.dtype
    y = out if out is not None else np.zeros(row_end - row_begin, dtype)
    lib(dtype).oracle_spmv_gold_rows(row_begin, row_end, row_ptr, col, val, x, y)
    return y


def spmv_fpga_order(row_ptr, col, val, x, nr_cols: int, cols_div_blocks: int, vf: int, y=None):
    """Arithmetic order of spmv.cpp:66-104 + csr_hw.cpp:1531-1565 (accumulates into y)."""
    dtype = val.dtype
    n = len(row_ptr) - 1
    if y is None:
        y = np.zeros(n, dtype)
    lib(dtype).oracle_spmv_fpga_order(n, nr_cols, _c(row_ptr, np.uint32), _c(col, np.uint32),
                                      _c(val, dtype), _c(x, dtype), y, cols_div_blocks, vf)
    return y


def verification_errors(sw, hw) -> int:
    """csr_hw.cpp:1571-1590: number of entries with |sw-hw| >= 1e-5 or NaN."""
    dtype = sw.dtype
    return int(lib(dtype).oracle_verification_errors(len(sw), _c(sw, dtype), _c(hw, dtype)))


def scaled_error(row_ptr, col, val, x, y_ref, y_test) -> float:
    """max_i |y_ref_i - y_test_i| / (|A||x|)_i  (SURVEY §8d parity metric; rows with
    (|A||x|)_i == 0 must match exactly)."""
    n = len(row_ptr) - 1
    absax = np.zeros(n, np.float64)
    if n and len(col) and int(np.max(col)) >= len(x):
        raise IndexError("scaled_error: column index past the end of x")
    if n:
        dtype = np.dtype(val.dtype)
        lib(dtype).oracle_abs_spmv(n, _c(row_ptr, np.uint32), _c(col, np.uint32), _c(val, dtype),
                                   _c(x, dtype), absax)
    diff = np.abs(y_ref.astype(np.float64) - y_test.astype(np.float64))
    zero = absax == 0
    if np.any(diff[zero] != 0) or np.any(np.isnan(diff)):
        return float("inf")
    if np.all(zero):
        return 0.0
    return float(np.max(diff[~zero] / absax[~zero]))


def block_matrix(row_ptr, col, val, thres_l: int, thres_h: int, vf: int):
    """csr_hw.cpp:190-265 (create_block_matrix) for one column block [thres_l, thres_h]:
    the non-empty rows of the block only, columns rebased to thres_l, every row zero-padded
    (col 0, value 0) to a multiple of `vf`. Returns (row_ptr, col, val) of the block
    (without the trailing pad rows that only the last CU carries, csr_hw.cpp:246-255)."""
    rp_out, c_out, v_out = [0], [], []
    for i in range(len(row_ptr) - 1):
        k = [j for j in range(int(row_ptr[i]), int(row_ptr[i + 1])) if thres_l <= int(col[j]) <= thres_h]
        if not k:
            continue
        c_out += [int(col[j]) - thres_l for j in k]
        v_out += [val[j] for j in k]
        pad = (-len(k)) % vf
        c_out += [0] * pad
        v_out += [val.dtype.type(0)] * pad
        rp_out.append(rp_out[-1] + len(k) + pad)
    return (np.array(rp_out, np.uint32), np.array(c_out, np.uint32), np.array(v_out, val.dtype))


def pack_hw_submatrix(row_ptr, col, val):
    """csr_hw.cpp:270-318 (generate_balanced_hw_submatrix) for one CU's rows of one block:
    128-bit bus words in groups [C, V, V, V, V] (fp64) or [C, V, V] (fp32), util.h:61-67.
    Field k of a C word holds the column in bits [16k, 16k+14] and the last-element-of-row
    flag in bit 16k+15 (8 fields per word); lane k of a V word holds value k in bits
    [W*k, W*k+W-1]. Returns uint64 array (words, 2) = (bits 0-63, bits 64-127)."""
    w = val.dtype.itemsize * 8
    ratio_v = 128 // w              # values per V word
    ratio_col_val = 8 // ratio_v + 1  # one C word per 8 entries, then 8/ratio_v V words
    z = len(col)
    words = [0] * max(1, -(-z // 8) * ratio_col_val)
    c_i, v_i, c_cp, v_cp = 0, 1, 0, 0
    e = 0
    for i in range(len(row_ptr) - 1):
        n_row = int(row_ptr[i + 1]) - int(row_ptr[i])
        for k in range(n_row):
            field = (int(col[e]) & 0x7FFF) | ((1 << 15) if k == n_row - 1 else 0)
            words[c_i] |= field << (16 * c_cp)
            c_cp += 1
            if c_cp == 8:
                c_i += ratio_col_val
                c_cp = 0
            bits = int(np.array([val[e]], val.dtype).view(np.uint64 if w == 64 else np.uint32)[0])
            words[v_i] |= bits << (w * v_cp)
            v_cp += 1
            if v_cp == ratio_v:
                v_i += 1
                if v_i % ratio_col_val == 0:
                    v_i += 1
                v_cp = 0
            e += 1
    out = np.zeros((len(words), 2), np.uint64)
    for j, wd in enumerate(words):
        out[j, 0] = wd & 0xFFFFFFFFFFFFFFFF
        out[j, 1] = wd >> 64
    return out


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)
