#!/usr/bin/env python3
"""Device -> pinned host copy rate against the size of each copy: 80 MB of y copied as back-to-back
pieces of one size on one stream (hipMemcpyAsync through torch's copy_, timed with HIP events on
that stream), the form spmv_hw's copy-back issues. Also the rate of pieces in a tapering sequence
(the streamed copy-back's bounds at 8 pieces). One JSON line per form. Measurement tool, not
product code."""
import json

import torch


def timed(stream, fn, reps=7):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            a.record()
            fn()
            b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    total = 80 << 20
    dev = torch.empty(total // 4, dtype=torch.float32, device="cuda").uniform_()
    host = torch.empty(total // 4, dtype=torch.float32, pin_memory=True)
    s = torch.cuda.Stream()
    n = dev.numel()
    host.copy_(dev)  # warm the path
    torch.cuda.synchronize()
    for mb in (0.3125, 0.625, 1.25, 2.5, 5, 10, 20, 40, 80):
        k = int(round(80 / mb))
        step = n // k

        def run():
            for j in range(k):
                b, e = j * step, (j + 1) * step if j < k - 1 else n
                host[b:e].copy_(dev[b:e], non_blocking=True)

        ms = timed(s, run)
        print(json.dumps({"form": "equal", "piece_mb": mb, "pieces": k, "ms": round(ms, 4),
                          "GBps": round(total / ms / 1e6, 1)}), flush=True)
    w = [16, 16, 16, 8, 4, 2, 1, 1]
    for tot_mb in (80, 40):
        m = n * tot_mb // 80
        bounds = [0]
        for x in w:
            bounds.append(bounds[-1] + m * x // 64)
        bounds[-1] = m

        def run_t():
            for j in range(len(w)):
                host[bounds[j]:bounds[j + 1]].copy_(dev[bounds[j]:bounds[j + 1]], non_blocking=True)

        ms = timed(s, run_t)
        print(json.dumps({"form": "tapered", "total_mb": tot_mb, "ms": round(ms, 4),
                          "GBps": round(m * 4 / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
