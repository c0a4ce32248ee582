"""Traces spmv_hw's streamed copy-back on the 10M/160M fp64 matrix (one unit, host merge,
SPMV_HW_TRACE=1): four calls, each printing when every piece of y was released (by its panels'
flags or by the end of the kernel) and its copy enqueued, and when the panel flags were first
seen (profiles/r06f_spmv_hw_stream_trace.txt). Measurement tool, not product code."""
import os, sys
sys.path.insert(0, "spmv-fpga_amd")
import numpy as np, torch, spmv_hw
os.environ.update(SPMV_NGPUS="1", SPMV_HW_MERGE="host", SPMV_HW_TRACE="1")
lib = spmv_hw.load(np.float64)
n, z = 10_000_000, 160_000_000
rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
x = spmv_hw.gen_vector(lib, n, seed=6)
h = [rp.cpu().numpy().view(np.uint32), col.cpu().numpy().view(np.uint32), val.cpu().numpy(), x.cpu().numpy()]
m = lib.make_csr_matrix(h[0], h[1], h[2], n)
hw, bm = lib.create_csr_hw_matrix(m)
hx = lib.create_csr_hw_x_vector(lib.make_csr_vector(h[3]), 1, hw[0].contents.nr_cols)
yv = lib.make_csr_vector(np.zeros(n))
for _ in range(4):
    lib.spmv_hw(hw, hx, yv, bm)
