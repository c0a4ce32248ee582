"""Python host mirror of the csr_hw_wrapper drop-in boundary (ctypes over libspmv_hw_*.so).

The C-ABI (include/csr_hw_wrapper.h) is the product boundary; this module binds it with the
reference's names and argument meaning (euroexa/spmv-fpga src/csr_hw_wrapper.h:9-17,
src/csr_hw.h:140,148) so tests and the bench read like the reference's main.cpp:46-97 flow.
It has no compute of its own and no fallback: if the HIP library is not built, every entry
point raises.

Two precisions, as the reference's DOUBLE build knob (util.h:18-26): dtype=np.float64 binds
libspmv_hw_f64.so, dtype=np.float32 binds libspmv_hw_f32.so.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

try:  # share torch's HIP runtime when torch is present (it must be loaded first)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the pure C-ABI path
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "lib")
_LIBS: dict = {}

IndexType = ctypes.c_uint32


def ablations_requested() -> bool:
    return os.environ.get("SPMV_HW_ABLATIONS") == "1"


def lib_path(dtype=np.float64, ablations: bool | None = None) -> str:
    """The product library; ablations=True (default: env SPMV_HW_ABLATIONS=1) selects the tools
    build (`make -C spmv-fpga_amd ablations`, -DSPMV_ABLATIONS): the same kernels plus the
    measurement-only variants and the environment switches that force layouts and schedules
    (tools/ab_variants.py, and the tests that cover those layouts)."""
    name = {8: "libspmv_hw_f64.so", 4: "libspmv_hw_f32.so"}[np.dtype(dtype).itemsize]
    if ablations_requested() if ablations is None else ablations:
        return os.path.join(LIBDIR, "ablations", name)
    return os.path.join(LIBDIR, name)


def build() -> None:
    """Compile both precisions for gfx950 (hipcc, see Makefile)."""
    subprocess.run(["make", "-s", "-C", HERE, "-j2"], check=True)


def _value_ctype(dtype):
    return ctypes.c_double if np.dtype(dtype) == np.float64 else ctypes.c_float


class BusDataType(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


def _structs(dtype):
    V = _value_ctype(dtype)

    class csr_matrix(ctypes.Structure):  # csr.h:15-24
        _fields_ = [("row_ptr", ctypes.POINTER(IndexType)), ("col_ind", ctypes.POINTER(IndexType)),
                    ("values", ctypes.POINTER(V)), ("nr_nzeros", IndexType), ("nr_rows", IndexType),
                    ("nr_cols", IndexType), ("Filename", ctypes.c_char_p)]

    class csr_vector(ctypes.Structure):  # csr.h:26-29
        _fields_ = [("values", ctypes.POINTER(V)), ("nr_values", IndexType)]

    class csr_hw_matrix(ctypes.Structure):  # csr_hw.h:16-26
        _fields_ = [("submatrix", ctypes.POINTER(ctypes.POINTER(BusDataType))),
                    ("nr_rows", ctypes.POINTER(IndexType)), ("nr_cols", ctypes.POINTER(IndexType)),
                    ("nr_nzeros", ctypes.POINTER(IndexType)), ("nr_ci", ctypes.POINTER(IndexType)),
                    ("nr_val", ctypes.POINTER(IndexType)), ("blocks", ctypes.c_int)]

    class csr_hw_vector(ctypes.Structure):  # csr_hw.h:28-33
        _fields_ = [("values", ctypes.POINTER(ctypes.POINTER(BusDataType))),
                    ("nr_values", ctypes.POINTER(IndexType)), ("blocks", ctypes.c_int)]

    return csr_matrix, csr_vector, csr_hw_matrix, csr_hw_vector


class csr_header(ctypes.Structure):  # csr.h:7-13
    _fields_ = [("nr_rows", IndexType), ("nr_cols", IndexType), ("nr_nzeros", IndexType),
                ("blocks", ctypes.c_int)]


class spmv_plan_stats(ctypes.Structure):
    _fields_ = [("nr_rows", ctypes.c_uint64), ("nr_cols", ctypes.c_uint64),
                ("nr_nzeros", ctypes.c_uint64), ("nr_nonempty_rows", ctypes.c_uint64),
                ("nr_tiles", ctypes.c_uint64), ("tile_nnz", ctypes.c_uint64),
                ("device_bytes", ctypes.c_uint64), ("algorithmic_bytes", ctypes.c_uint64),
                ("device", ctypes.c_int32), ("kernel", ctypes.c_int32), ("blocks", ctypes.c_int32),
                ("format", ctypes.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every symbol include/csr_hw_wrapper.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "create_csr_hw_matrix", "create_csr_hw_y_vector", "create_csr_hw_x_vector", "spmv_hw",
    "delete_csr_hw_matrix", "delete_csr_hw_y_vector", "delete_csr_hw_x_vector",
    "storage_overhead", "verification",
    "spmv_hw_units", "spmv_hw_set_units", "spmv_hw_value_bytes", "spmv_hw_last_error",
    "spmv_plan_create_device", "spmv_plan_create_host", "spmv_plan_run", "spmv_plan_run_graph", "spmv_plan_get_stats",
    "spmv_plan_set_variant", "spmv_plan_set_timing", "spmv_plan_get_timing", "spmv_plan_destroy", "spmv_partition_rows",
    "spmv_gen_banded", "spmv_gen_powerlaw_row_ptr", "spmv_gen_fill", "spmv_gen_vector",
    "spmv_read_csr_header", "spmv_read_csr_matrix", "spmv_read_csr", "spmv_free_csr",
    "spmv_mgpu_create", "spmv_mgpu_set_x", "spmv_mgpu_run", "spmv_mgpu_get_y", "spmv_mgpu_get_timing",
    "spmv_mgpu_slice", "spmv_mgpu_destroy", "spmv_mgpu_unique_id", "spmv_mgpu_create_rank",
    "spmv_mgpu_set_x_device", "spmv_mgpu_set_x_device_on", "spmv_mgpu_y_device", "spmv_mgpu_run_pipelined",
    "spmv_mgpu_run_graph", "spmv_mgpu_comm_count", "spmv_mgpu_schedule",
]

MGPU_GATHER, MGPU_REDUCE, MGPU_ALLGATHER = 0, 1, 2  # include/csr_hw_wrapper.h SPMV_MGPU_*
# spmv_xop kinds and buffers (include/csr_hw_wrapper.h SPMV_XOP_* / SPMV_XBUF_*)
XOP_ZERO, XOP_COMPUTE, XOP_SEND, XOP_RECV, XOP_REDUCE, XOP_BCAST = range(6)
XOP_NAMES = {XOP_ZERO: "zero", XOP_COMPUTE: "compute", XOP_SEND: "send", XOP_RECV: "recv",
             XOP_REDUCE: "reduce", XOP_BCAST: "bcast"}
XBUF_Y, XBUF_SLICE, XBUF_PART, XBUF_XNEXT = range(4)


class spmv_xop(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("buf", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("out", ctypes.c_int32), ("offset", ctypes.c_uint32), ("count", ctypes.c_uint32)]


class Lib:
    """Typed handle on one precision of libspmv_hw."""

    def __init__(self, dtype=np.float64, ablations: bool | None = None):
        self.dtype = np.dtype(dtype)
        self.path = path = lib_path(self.dtype, ablations)
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is not built (run `make -C spmv-fpga_amd`); "
                               "the MI355X path has no CPU fallback")
        self.L = L = ctypes.CDLL(path)
        self.V = V = _value_ctype(self.dtype)
        (self.csr_matrix, self.csr_vector, self.csr_hw_matrix, self.csr_hw_vector) = _structs(self.dtype)
        PM = ctypes.POINTER(self.csr_hw_matrix)
        PV = ctypes.POINTER(self.csr_hw_vector)
        PB = ctypes.POINTER(ctypes.POINTER(ctypes.c_bool))
        vp, up = ctypes.c_void_p, ctypes.POINTER(IndexType)
        sig = {
            "create_csr_hw_matrix": (None, [ctypes.POINTER(self.csr_matrix), ctypes.POINTER(ctypes.POINTER(PM)),
                                            ctypes.POINTER(PB)]),
            "create_csr_hw_y_vector": (None, [ctypes.POINTER(PM), ctypes.POINTER(ctypes.POINTER(PV))]),
            "create_csr_hw_x_vector": (None, [ctypes.POINTER(PV), ctypes.POINTER(self.csr_vector), ctypes.c_int, up]),
            "spmv_hw": (None, [ctypes.POINTER(PM), PV, ctypes.POINTER(self.csr_vector), PB]),
            "delete_csr_hw_matrix": (None, [ctypes.POINTER(PM)]),
            "delete_csr_hw_y_vector": (None, [ctypes.POINTER(PV)]),
            "delete_csr_hw_x_vector": (None, [PV]),
            "storage_overhead": (V, [PM]),
            "verification": (ctypes.c_int, [IndexType, ctypes.POINTER(V), ctypes.POINTER(V), ctypes.c_int]),
            "spmv_hw_units": (ctypes.c_int, []),
            "spmv_hw_set_units": (ctypes.c_int, [ctypes.c_int]),
            "spmv_hw_value_bytes": (ctypes.c_int, []),
            "spmv_hw_last_error": (ctypes.c_char_p, []),
            "spmv_plan_create_device": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, IndexType, IndexType,
                                                       IndexType, vp, vp, vp, vp]),
            "spmv_plan_create_host": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int,
                                                     ctypes.POINTER(self.csr_matrix), IndexType, IndexType]),
            "spmv_plan_run": (ctypes.c_int, [vp, vp, vp, vp]),
            "spmv_plan_run_graph": (ctypes.c_int, [vp, vp, vp, ctypes.c_int, vp]),
            "spmv_plan_get_stats": (ctypes.c_int, [vp, ctypes.POINTER(spmv_plan_stats)]),
            "spmv_plan_set_timing": (ctypes.c_int, [vp, ctypes.c_int]),
            "spmv_plan_set_variant": (ctypes.c_int, [vp, ctypes.c_int]),
            "spmv_plan_get_timing": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double),
                                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
            "spmv_plan_destroy": (None, [vp]),
            "spmv_partition_rows": (ctypes.c_int, [up, IndexType, ctypes.c_int, up]),
            "spmv_gen_banded": (ctypes.c_int, [IndexType, IndexType, ctypes.c_uint64, vp, vp, vp, vp]),
            "spmv_gen_powerlaw_row_ptr": (ctypes.c_int, [IndexType, ctypes.c_uint64, IndexType, ctypes.c_uint64,
                                                         up, ctypes.POINTER(ctypes.c_double)]),
            "spmv_gen_fill": (ctypes.c_int, [IndexType, IndexType, ctypes.c_uint64, ctypes.c_uint64, vp, vp, vp, vp]),
            "spmv_gen_vector": (ctypes.c_int, [IndexType, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double,
                                               ctypes.c_double, vp, vp]),
            "spmv_read_csr_header": (ctypes.c_int, [ctypes.POINTER(csr_header), ctypes.c_char_p]),
            "spmv_read_csr_matrix": (ctypes.c_int, [ctypes.POINTER(self.csr_matrix), ctypes.c_char_p]),
            "spmv_read_csr": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(self.csr_matrix)]),
            "spmv_free_csr": (None, [ctypes.POINTER(self.csr_matrix)]),
            "spmv_mgpu_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                ctypes.POINTER(self.csr_matrix)]),
            "spmv_mgpu_set_x": (ctypes.c_int, [vp, ctypes.POINTER(V)]),
            "spmv_mgpu_run": (ctypes.c_int, [vp, ctypes.c_int]),
            "spmv_mgpu_get_y": (ctypes.c_int, [vp, ctypes.POINTER(V), ctypes.c_int]),
            "spmv_mgpu_get_timing": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double),
                                                    ctypes.POINTER(ctypes.c_double)]),
            "spmv_mgpu_slice": (ctypes.c_int, [vp, ctypes.c_int, up, up, ctypes.POINTER(ctypes.c_int)]),
            "spmv_mgpu_destroy": (None, [vp]),
            "spmv_mgpu_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
            "spmv_mgpu_create_rank": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                                     ctypes.c_int, up, IndexType, vp]),
            "spmv_mgpu_set_x_device": (ctypes.c_int, [vp, vp]),
            "spmv_mgpu_set_x_device_on": (ctypes.c_int, [vp, vp, vp]),
            "spmv_mgpu_run_pipelined": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
            "spmv_mgpu_run_graph": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]),
            "spmv_mgpu_y_device": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(vp)]),
            "spmv_mgpu_comm_count": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int)]),
            "spmv_mgpu_schedule": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, up,
                                                  ctypes.POINTER(spmv_xop), ctypes.c_int]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.spmv_hw_value_bytes() != self.dtype.itemsize:
            raise RuntimeError(f"{path} was built for a different precision")
        self._libc = ctypes.CDLL(None)
        self._libc.free.argtypes = [ctypes.c_void_p]

    # ---- error helper for Part-2 calls ----
    def _ok(self, rc: int, what: str) -> None:
        if rc != 0:
            raise RuntimeError(f"{what}: {self.L.spmv_hw_last_error().decode()}")

    # ---- host-side helpers ----
    def make_csr_matrix(self, row_ptr, col, val, nr_cols: int):
        """A csr_matrix (csr.h:15-24) viewing numpy arrays (kept alive on the struct)."""
        row_ptr = np.ascontiguousarray(row_ptr, np.uint32)
        col = np.ascontiguousarray(col, np.uint32)
        val = np.ascontiguousarray(val, self.dtype)
        m = self.csr_matrix()
        m.row_ptr = row_ptr.ctypes.data_as(ctypes.POINTER(IndexType))
        m.col_ind = col.ctypes.data_as(ctypes.POINTER(IndexType))
        m.values = val.ctypes.data_as(ctypes.POINTER(self.V))
        m.nr_nzeros = int(row_ptr[-1])
        m.nr_rows = len(row_ptr) - 1
        m.nr_cols = int(nr_cols)
        m.Filename = None
        m._keep = (row_ptr, col, val)
        return m

    def make_csr_vector(self, values):
        values = np.ascontiguousarray(values, self.dtype)
        v = self.csr_vector()
        v.values = values.ctypes.data_as(ctypes.POINTER(self.V))
        v.nr_values = len(values)
        v._keep = values
        return v

    # ---- Part 1: reference API (same names; failures exit the process like the C-ABI) ----
    def create_csr_hw_matrix(self, matrix):
        hw = ctypes.POINTER(ctypes.POINTER(self.csr_hw_matrix))()
        bm = ctypes.POINTER(ctypes.POINTER(ctypes.c_bool))()
        self.L.create_csr_hw_matrix(ctypes.byref(matrix), ctypes.byref(hw), ctypes.byref(bm))
        return hw, bm

    def create_csr_hw_x_vector(self, x_vec, blocks: int, nr_cols):
        hx = ctypes.POINTER(self.csr_hw_vector)()
        self.L.create_csr_hw_x_vector(ctypes.byref(hx), ctypes.byref(x_vec), blocks, nr_cols)
        return hx

    def create_csr_hw_y_vector(self, hw_matrix):
        hy = ctypes.POINTER(ctypes.POINTER(self.csr_hw_vector))()
        self.L.create_csr_hw_y_vector(hw_matrix, ctypes.byref(hy))
        return hy

    def spmv_hw(self, hw_matrix, hw_x, y_vec, bitmap) -> None:
        self.L.spmv_hw(hw_matrix, hw_x, ctypes.byref(y_vec), bitmap)

    def delete_csr_hw_matrix(self, hw_matrix) -> None:
        self.L.delete_csr_hw_matrix(hw_matrix)

    def delete_csr_hw_y_vector(self, hw_y) -> None:
        self.L.delete_csr_hw_y_vector(hw_y)

    def delete_csr_hw_x_vector(self, hw_x) -> None:
        self.L.delete_csr_hw_x_vector(hw_x)

    def free_bitmap(self, bitmap) -> None:
        """main.cpp:95 frees only the outer array; that releases the whole bitmap here."""
        self._libc.free(ctypes.cast(bitmap, ctypes.c_void_p))

    def storage_overhead(self, hw_matrix_unit) -> float:
        return float(self.L.storage_overhead(hw_matrix_unit))

    def verification(self, sw, hw, verbose: int = 0) -> int:
        sw = np.ascontiguousarray(sw, self.dtype)
        hw = np.ascontiguousarray(hw, self.dtype)
        return int(self.L.verification(len(sw), sw.ctypes.data_as(ctypes.POINTER(self.V)),
                                       hw.ctypes.data_as(ctypes.POINTER(self.V)), verbose))

    def units(self) -> int:
        return int(self.L.spmv_hw_units())

    def set_units(self, units: int) -> int:
        """spmv_hw_set_units: the caller's compile-time ComputeUnits (0 = env SPMV_NGPUS)."""
        return int(self.L.spmv_hw_set_units(int(units)))

    # ---- Part 3: fast reader (host only) ----
    def read_csr_header(self, path: str):
        """spmv_read_csr_header: (rc, csr_header) with read_csr_header's codes (csr.cpp:10-46)."""
        h = csr_header()
        rc = self.L.spmv_read_csr_header(ctypes.byref(h), os.fsencode(path))
        return rc, h

    def read_csr(self, path: str):
        """(row_ptr u32[n+1], col u32[nnz], val[nnz], nr_cols) copied out of spmv_read_csr."""
        m = self.csr_matrix()
        rc = self.L.spmv_read_csr(os.fsencode(path), ctypes.byref(m))
        if rc != 0:
            raise RuntimeError(f"spmv_read_csr({path}) = {rc}: {self.L.spmv_hw_last_error().decode()}")
        try:
            n, z = int(m.nr_rows), int(m.nr_nzeros)
            rp = np.ctypeslib.as_array(m.row_ptr, (n + 1,)).copy()
            col = np.ctypeslib.as_array(m.col_ind, (z,)).copy() if z else np.zeros(0, np.uint32)
            val = np.ctypeslib.as_array(m.values, (z,)).copy() if z else np.zeros(0, self.dtype)
            return rp.astype(np.uint32), col.astype(np.uint32), val, int(m.nr_cols)
        finally:
            self.L.spmv_free_csr(ctypes.byref(m))

    def partition_rows(self, row_ptr, units: int):
        row_ptr = np.ascontiguousarray(row_ptr, np.uint32)
        bounds = np.zeros(units + 1, np.uint32)
        self._ok(self.L.spmv_partition_rows(row_ptr.ctypes.data_as(ctypes.POINTER(IndexType)),
                                            len(row_ptr) - 1, units,
                                            bounds.ctypes.data_as(ctypes.POINTER(IndexType))),
                 "spmv_partition_rows")
        return bounds

    def mgpu_schedule(self, exchange: int, rank: int, nranks: int, bounds):
        """spmv_mgpu_schedule: the ops rank `rank` issues for one SpMV step (host only), as dicts
        {kind, buf, peer, out, offset, count} in issue order."""
        b = np.ascontiguousarray(bounds, np.uint32)
        assert len(b) == nranks + 1
        bp = b.ctypes.data_as(ctypes.POINTER(IndexType))
        n = self.L.spmv_mgpu_schedule(int(exchange), int(rank), int(nranks), bp, None, 0)
        if n < 0:
            raise RuntimeError(f"spmv_mgpu_schedule: {self.L.spmv_hw_last_error().decode()}")
        ops = (spmv_xop * max(n, 1))()
        assert self.L.spmv_mgpu_schedule(int(exchange), int(rank), int(nranks), bp, ops, n) == n
        return [{k: getattr(ops[i], k) for k, _ in spmv_xop._fields_} for i in range(n)]

    def powerlaw_row_ptr(self, n: int, nnz: int, max_len: int = 65536, seed: int = 4):
        rp = np.zeros(n + 1, np.uint32)
        s = ctypes.c_double()
        self._ok(self.L.spmv_gen_powerlaw_row_ptr(n, nnz, max_len, seed,
                                                  rp.ctypes.data_as(ctypes.POINTER(IndexType)),
                                                  ctypes.byref(s)), "spmv_gen_powerlaw_row_ptr")
        return rp, s.value


class Plan:
    """One unit's device-resident matrix slice (include/csr_hw_wrapper.h Part 2)."""

    def __init__(self, lib: Lib, handle: ctypes.c_void_p):
        self.lib = lib
        self.h = handle

    @classmethod
    def from_device(cls, lib: Lib, row_ptr, col, val, nr_cols: int, device: int = 0, stream=None):
        """row_ptr/col/val: torch tensors on `device` (uint32 viewed as int32, values of lib.dtype)."""
        h = ctypes.c_void_p()
        n = row_ptr.numel() - 1
        nnz = int(row_ptr[-1].item()) - int(row_ptr[0].item()) if n >= 0 else 0
        lib._ok(lib.L.spmv_plan_create_device(ctypes.byref(h), device, n, nr_cols, nnz & 0xFFFFFFFF,
                                              row_ptr.data_ptr(), col.data_ptr(), val.data_ptr(),
                                              _stream_ptr(stream)), "spmv_plan_create_device")
        return cls(lib, h)

    @classmethod
    def from_host(cls, lib: Lib, matrix, row_begin: int, row_end: int, device: int = 0):
        h = ctypes.c_void_p()
        lib._ok(lib.L.spmv_plan_create_host(ctypes.byref(h), device, ctypes.byref(matrix), row_begin, row_end),
                "spmv_plan_create_host")
        return cls(lib, h)

    def run(self, x, y, stream=None) -> None:
        self.lib._ok(self.lib.L.spmv_plan_run(self.h, x.data_ptr(), y.data_ptr(), _stream_ptr(stream)),
                     "spmv_plan_run")

    def run_graph(self, x, y, iters: int = 1, stream=None) -> None:
        """`iters` SpMVs y = A x replayed from a hipGraph captured on the first call."""
        self.lib._ok(self.lib.L.spmv_plan_run_graph(self.h, x.data_ptr(), y.data_ptr(), int(iters),
                                                    _stream_ptr(stream)), "spmv_plan_run_graph")

    def stats(self) -> dict:
        st = spmv_plan_stats()
        self.lib._ok(self.lib.L.spmv_plan_get_stats(self.h, ctypes.byref(st)), "spmv_plan_get_stats")
        return st.as_dict()

    def set_variant(self, variant: int) -> None:
        self.lib._ok(self.lib.L.spmv_plan_set_variant(self.h, int(variant)), "spmv_plan_set_variant")

    def set_timing(self, on: bool) -> None:
        self.lib._ok(self.lib.L.spmv_plan_set_timing(self.h, int(on)), "spmv_plan_set_timing")

    def timing(self):
        mean, tot, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        self.lib._ok(self.lib.L.spmv_plan_get_timing(self.h, ctypes.byref(mean), ctypes.byref(tot),
                                                     ctypes.byref(n)), "spmv_plan_get_timing")
        return mean.value, tot.value, n.value

    def destroy(self) -> None:
        if self.h:
            self.lib.L.spmv_plan_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.destroy()
        except Exception:
            pass


def mgpu_unique_id(lib: "Lib") -> bytes:
    """spmv_mgpu_unique_id: the 128-byte RCCL id rank 0 shares with the other ranks."""
    buf = ctypes.create_string_buffer(128)
    lib._ok(lib.L.spmv_mgpu_unique_id(buf), "spmv_mgpu_unique_id")
    return buf.raw


class MultiGpu:
    """Part 4 of the C-ABI (spmv_mgpu_*): RCCL exchange of y between GPUs -- one process driving
    `ndev` GPUs (MultiGpu(lib, matrix, ndev=...)), or one process per GPU
    (MultiGpu.rank(lib, rank, nranks, uid, device, bounds, nr_cols, plan))."""

    def __init__(self, lib: Lib, matrix=None, devices=None, ndev: int = None, _handle=None, _dims=None):
        self.lib = lib
        if _handle is not None:
            self.h = _handle
            self.ndev, self.nr_rows, self.nr_cols = _dims
            return
        devs = list(devices) if devices is not None else list(range(ndev or 1))
        arr = (ctypes.c_int * len(devs))(*devs)
        h = ctypes.c_void_p()
        lib._ok(lib.L.spmv_mgpu_create(ctypes.byref(h), len(devs), arr, ctypes.byref(matrix)), "spmv_mgpu_create")
        self.h, self.ndev, self.nr_rows, self.nr_cols = h, len(devs), int(matrix.nr_rows), int(matrix.nr_cols)

    @classmethod
    def rank(cls, lib: Lib, rank: int, nranks: int, uid: bytes, device: int, bounds, nr_cols: int, plan):
        b = np.ascontiguousarray(bounds, np.uint32)
        h = ctypes.c_void_p()
        lib._ok(lib.L.spmv_mgpu_create_rank(ctypes.byref(h), int(rank), int(nranks), uid, int(device),
                                            b.ctypes.data_as(ctypes.POINTER(IndexType)), int(nr_cols), plan.h),
                "spmv_mgpu_create_rank")
        obj = cls(lib, _handle=h, _dims=(1, int(b[-1]), int(nr_cols)))
        obj._plan = plan  # borrowed by the handle: keep it alive
        return obj

    def set_x_device(self, x, stream=None) -> None:
        """Every rank calls it; x (a device tensor) is read on rank 0 only. The copy is ordered
        after the torch stream that produced x (`stream`, default: the current stream) by an
        event, with no host wait."""
        if x is not None:
            # the C side records the producer event on rank 0's device: x must live there
            dev0 = self.slice(0)[2]
            if dev0 >= 0 and x.device.index != dev0:
                raise ValueError(f"set_x_device: x is on cuda:{x.device.index}, rank 0 of this handle on cuda:{dev0}")
        if stream is None and x is not None:
            import torch
            stream = torch.cuda.current_stream(x.device)
        sp = ctypes.c_void_p(stream.cuda_stream if stream is not None else 0)
        self.lib._ok(self.lib.L.spmv_mgpu_set_x_device_on(self.h, ctypes.c_void_p(x.data_ptr() if x is not None else 0),
                                                          sp), "spmv_mgpu_set_x_device_on")

    def run_pipelined(self, exchange: int = MGPU_GATHER, steps: int = 8) -> float:
        """`steps` SpMVs, each exchange overlapping the next SpMV's kernels; ms per step."""
        ms = ctypes.c_double()
        self.lib._ok(self.lib.L.spmv_mgpu_run_pipelined(self.h, int(exchange), int(steps), ctypes.byref(ms)),
                     "spmv_mgpu_run_pipelined")
        return float(ms.value)

    def run_graph(self, exchange: int = MGPU_ALLGATHER, iters: int = 8) -> float:
        """`iters` steps (SpMV + exchange) replayed from one hipGraph (one device per handle);
        ms per step. The all-gather form leaves A^iters x as x."""
        ms = ctypes.c_double()
        self.lib._ok(self.lib.L.spmv_mgpu_run_graph(self.h, int(exchange), int(iters), ctypes.byref(ms)),
                     "spmv_mgpu_run_graph")
        return float(ms.value)

    def comm_count(self) -> int:
        """Ranks in the handle's RCCL communicator (ncclCommCount)."""
        c = ctypes.c_int()
        self.lib._ok(self.lib.L.spmv_mgpu_comm_count(self.h, ctypes.byref(c)), "spmv_mgpu_comm_count")
        return int(c.value)

    def y_device_ptr(self, exchange: int = MGPU_GATHER) -> int:
        p = ctypes.c_void_p()
        self.lib._ok(self.lib.L.spmv_mgpu_y_device(self.h, int(exchange), ctypes.byref(p)), "spmv_mgpu_y_device")
        return int(p.value or 0)

    def set_x(self, x) -> None:
        x = np.ascontiguousarray(x, self.lib.dtype)
        self.lib._ok(self.lib.L.spmv_mgpu_set_x(self.h, x.ctypes.data_as(ctypes.POINTER(self.lib.V))),
                     "spmv_mgpu_set_x")

    def run(self, exchange: int = MGPU_GATHER) -> None:
        self.lib._ok(self.lib.L.spmv_mgpu_run(self.h, int(exchange)), "spmv_mgpu_run")

    def y(self, exchange: int = MGPU_GATHER):
        out = np.empty(self.nr_rows, self.lib.dtype)
        self.lib._ok(self.lib.L.spmv_mgpu_get_y(self.h, out.ctypes.data_as(ctypes.POINTER(self.lib.V)),
                                                int(exchange)), "spmv_mgpu_get_y")
        return out

    def timing(self):
        c, e = ctypes.c_double(), ctypes.c_double()
        self.lib._ok(self.lib.L.spmv_mgpu_get_timing(self.h, ctypes.byref(c), ctypes.byref(e)), "spmv_mgpu_get_timing")
        return c.value, e.value

    def slice(self, d: int):
        b, e, dev = IndexType(), IndexType(), ctypes.c_int()
        self.lib._ok(self.lib.L.spmv_mgpu_slice(self.h, d, ctypes.byref(b), ctypes.byref(e), ctypes.byref(dev)),
                     "spmv_mgpu_slice")
        return b.value, e.value, dev.value

    def destroy(self) -> None:
        if self.h:
            self.lib.L.spmv_mgpu_destroy(self.h)
            self.h = None


def _stream_ptr(stream):
    if stream is None:
        if torch is not None and torch.cuda.is_available():
            return torch.cuda.current_stream().cuda_stream
        return None
    return getattr(stream, "cuda_stream", stream)


def gen_banded(lib: Lib, n: int, width: int = 16, seed: int = 2, device: str = "cuda"):
    """Config 2 matrix on the GPU: returns (row_ptr, col, val) torch tensors."""
    rp = torch.empty(n + 1, dtype=torch.int32, device=device)
    col = torch.empty(n * width, dtype=torch.int32, device=device)
    val = torch.empty(n * width, dtype=_torch_dtype(lib.dtype), device=device)
    lib._ok(lib.L.spmv_gen_banded(n, width, seed, rp.data_ptr(), col.data_ptr(), val.data_ptr(),
                                  _stream_ptr(None)), "spmv_gen_banded")
    return rp, col, val


def gen_powerlaw(lib: Lib, n: int, m: int, nnz: int, seed: int = 4, max_len: int = 65536,
                 row_begin: int = 0, row_end: int | None = None, device: str = "cuda"):
    """Config 3 matrix (or rows [row_begin,row_end) of it) on the GPU.
    Row lengths come from seed, columns/values from seed+1 (seeds 4, 5)."""
    rp_full, scale = lib.powerlaw_row_ptr(n, nnz, min(max_len, m), seed)
    row_end = n if row_end is None else row_end
    rp_h = (rp_full[row_begin:row_end + 1].astype(np.int64) - int(rp_full[row_begin])).astype(np.uint32)
    z = int(rp_h[-1])
    rp = torch.from_numpy(rp_h.view(np.int32)).to(device)
    col = torch.empty(max(z, 1), dtype=torch.int32, device=device)
    val = torch.empty(max(z, 1), dtype=_torch_dtype(lib.dtype), device=device)
    lib._ok(lib.L.spmv_gen_fill(row_end - row_begin, m, seed + 1, row_begin, rp.data_ptr(), col.data_ptr(),
                                val.data_ptr(), _stream_ptr(None)), "spmv_gen_fill")
    return rp, col[:z], val[:z], scale


def gen_vector(lib: Lib, n: int, seed: int = 6, lo: float = 0.0, hi: float = 1.0, offset: int = 0,
               device: str = "cuda"):
    x = torch.empty(max(n, 1), dtype=_torch_dtype(lib.dtype), device=device)
    lib._ok(lib.L.spmv_gen_vector(n, seed, offset, lo, hi, x.data_ptr(), _stream_ptr(None)), "spmv_gen_vector")
    return x[:n]


def _torch_dtype(dtype):
    return torch.float64 if np.dtype(dtype) == np.float64 else torch.float32


def load(dtype=np.float64, ablations: bool | None = None) -> Lib:
    """The library of `dtype`; the tools build when ablations (default: env SPMV_HW_ABLATIONS=1)."""
    abl = ablations_requested() if ablations is None else bool(ablations)
    key = (np.dtype(dtype).str, abl)
    if key not in _LIBS:
        _LIBS[key] = Lib(dtype, abl)
    return _LIBS[key]
