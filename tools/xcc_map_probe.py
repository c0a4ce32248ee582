#!/usr/bin/env python3
"""Which XCC runs sweep workgroup b? (measurement build, SPMV_HW_ABLATIONS=1.) For 40 launches of a
2M-row and of the 10M-row power-law sweep plan, reads each workgroup's HW_REG_XCC_ID (stamped by
k_spmv_sweep_packed, see tools/wg_timeline.py) and prints the set of (xcc - b) mod 8 per launch: a
single 0 means block b ran on XCC b % 8, the assumption of the sweep's XCC bias.
Measurement tool, not product code."""
import ctypes, os, sys, json
os.environ["SPMV_HW_ABLATIONS"] = "1"
sys.path.insert(0, "spmv-fpga_amd")
import numpy as np, torch, spmv_hw
lib = spmv_hw.load(np.float64)
for n, m, z in ((2_000_000, 2_000_000, 32_000_000), (10_000_000, 10_000_000, 160_000_000)):
    rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, m, z, seed=4)
    x = spmv_hw.gen_vector(lib, m, seed=6)
    os.environ["SPMV_HW_KERNEL"] = "sweep"
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, m)
    U = plan.stats()["nr_tiles"]
    y = torch.empty(n, dtype=torch.float64, device="cuda")
    offs = []
    for it in range(40):
        plan.run(x, y); torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (4 * min(U, 4096)))()
        lib.L.spmv_abl_wg_times(buf, ctypes.c_uint(4 * min(U, 4096)))
        a = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 4)
        xcc = (a[:, 3] >> np.uint64(32)).astype(np.int64)
        b = np.arange(len(xcc))
        c = (xcc - b) % 8
        offs.append(sorted(set(c.tolist())))
    print(json.dumps({"rows": n, "units": U, "offsets_per_launch": [o if len(o) > 1 else o[0] for o in offs]}), flush=True)
    plan.destroy(); del rp, col, val, x, y; torch.cuda.empty_cache()
