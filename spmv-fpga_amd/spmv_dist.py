"""Multi-GPU layout of the SpMV path: one process per GPU, torch.distributed over RCCL/xGMI.

The reference's only parallelism is ComputeUnits pipelines that each own a contiguous,
nnz-balanced row slice of every column block (csr_hw.cpp:459-468) with x replicated into every
CU (spmv.cpp:280-294); the host then merges the per-CU y (accum_results, csr_hw.cpp:1531-1565,
loop csr_hw_wrapper.cpp:276-281). Here a CU is a GPU rank:

  * row_slice(): the nnz-balanced contiguous slice of rank r (spmv_partition_rows in the C-ABI,
    S1 rule without the FPGA alignment rules S2/S3);
  * x is replicated: broadcast once from rank 0 (broadcast_x) or generated on every rank;
  * the y merge is a real exchange step, done three ways over RCCL:
      - "reduce": every rank contributes a full-length partial y (zeros outside its slice) to
        an RCCL reduce(SUM) on rank 0 -- the literal accum_results '+=' mapping;
      - "gather": ranks send only their disjoint slices to rank 0 (bandwidth-optimal);
      - "allgather" (iterative solvers): equal padded slices all-gathered so
        every rank holds the full y as its next x (one RCCL all_gather_into_tensor).
    reduce and gather return the full y on rank 0 and None elsewhere.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def _staged(t: torch.Tensor) -> torch.Tensor:
    """gloo collectives run on host tensors (used by the CPU tests and the single-GPU
    multi-process rehearsal); RCCL ('nccl') works on the device tensor directly."""
    if dist.get_backend() == "gloo" and t.is_cuda:
        return t.cpu()
    return t


def row_slice(bounds, rank: int):
    return int(bounds[rank]), int(bounds[rank + 1])


def exchange_reduce(y_slice: torch.Tensor, row_begin: int, n_rows: int, dst: int = 0):
    """accum_results semantics: full-length partials summed into rank `dst`."""
    full = torch.zeros(n_rows, dtype=y_slice.dtype, device=y_slice.device)
    full[row_begin:row_begin + y_slice.numel()] = y_slice
    full = _staged(full)
    dist.reduce(full, dst=dst, op=dist.ReduceOp.SUM)
    return full if dist.get_rank() == dst else None


def exchange_gather(y_slice: torch.Tensor, counts, dst: int = 0):
    """Disjoint slices to rank `dst` (each rank sends only its own rows)."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    maxc = int(max(counts))
    buf = torch.zeros(maxc, dtype=y_slice.dtype, device=y_slice.device)
    buf[:y_slice.numel()] = y_slice
    buf = _staged(buf)
    if rank == dst:
        parts = [torch.empty(maxc, dtype=buf.dtype, device=buf.device) for _ in range(world)]
        dist.gather(buf, gather_list=parts, dst=dst)
        return torch.cat([parts[r][:int(counts[r])] for r in range(world)])
    dist.gather(buf, dst=dst)
    return None


def exchange_allgather(y_slice: torch.Tensor, counts, out: torch.Tensor | None = None):
    """Every rank receives the full y (e.g. as the next x of an iterative solver). Slices are
    padded to the longest one so the collective is a single all_gather_into_tensor."""
    world = dist.get_world_size()
    maxc = int(max(counts))
    buf = torch.zeros(maxc, dtype=y_slice.dtype, device=y_slice.device)
    buf[:y_slice.numel()] = y_slice
    buf = _staged(buf)
    gathered = torch.empty(world * maxc, dtype=buf.dtype, device=buf.device)
    dist.all_gather_into_tensor(gathered, buf)
    parts = gathered.view(world, maxc)
    n = int(np.sum(counts))
    if out is None:
        out = torch.empty(n, dtype=y_slice.dtype, device=y_slice.device)
    off = 0
    for r in range(world):
        c = int(counts[r])
        out[off:off + c].copy_(parts[r, :c])
        off += c
    return out


def pipelined_gather(run_step, y_bufs, counts, steps: int, dst: int = 0):
    """`steps` independent SpMVs whose y exchange overlaps the next SpMV.

    One SpMV's gather cannot overlap its own compute: the N = 8 slice is a single round of
    workgroups whose rows all finish at the end. A stream of SpMVs (right-hand
    sides, time steps) can: step k's y goes to rank `dst` on the collective's own stream while
    step k + 1 computes into the other buffer of `y_bufs` (double buffering; a buffer is reused
    only once its previous gather completed). run_step(k, y) enqueues SpMV k into y[:count] on the
    current stream. y_bufs are two device tensors of max(counts) values (equal-size gather). On
    rank `dst` returns the last step's full y; None elsewhere."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    maxc = int(max(counts))
    assert len(y_bufs) == 2 and all(b.numel() == maxc for b in y_bufs)
    gloo = dist.get_backend() == "gloo"
    parts = [[torch.empty(maxc, dtype=y_bufs[0].dtype, device="cpu" if gloo else y_bufs[0].device)
              for _ in range(world)] for _ in range(2)] if rank == dst else [None, None]
    works = [None, None]
    for k in range(steps):
        b = k % 2
        if works[b] is not None:
            works[b].wait()  # this buffer's previous gather is done before it is overwritten
        run_step(k, y_bufs[b])
        src = _staged(y_bufs[b])
        if rank == dst:
            works[b] = dist.gather(src, gather_list=parts[b], dst=dst, async_op=True)
        else:
            works[b] = dist.gather(src, dst=dst, async_op=True)
    for w in works:
        if w is not None:
            w.wait()
    if rank != dst or steps == 0:
        return None
    last = parts[(steps - 1) % 2]
    return torch.cat([last[r][:int(counts[r])] for r in range(world)])


def execute_schedule(ops, bufs, compute):
    """Runs one rank's step schedule (spmv_mgpu_schedule: the list every RCCL call of the
    library's exchange iterates over, mgpu.cpp issue_local / issue_exchange) over
    torch.distributed, op for op: ZERO and COMPUTE locally (compute(view) writes this rank's rows
    of A x into `view`), then SEND / RECV as posted point-to-point operations (the RCCL group posts
    them together), REDUCE and BCAST as collectives in list order (every rank lists them in the
    same order). `bufs` maps an SPMV_XBUF_* id to this rank's 1-D tensor of that role. gloo runs it
    on host tensors: the CPU replay of the multi-GPU merge (tests/test_exchange_schedule.py)."""
    import spmv_hw as hw
    for o in ops:
        view = bufs[o["buf"]][o["offset"]:o["offset"] + o["count"]] if o["buf"] in bufs else None
        if o["kind"] == hw.XOP_ZERO:
            view.zero_()
        elif o["kind"] == hw.XOP_COMPUTE:
            compute(view)
    pending = []
    for o in ops:
        k = o["kind"]
        if k < hw.XOP_SEND:
            continue
        view = bufs[o["buf"]][o["offset"]:o["offset"] + o["count"]]
        if k == hw.XOP_SEND:
            pending.append((dist.isend(_staged(view).contiguous(), dst=o["peer"]), None, None))
        elif k == hw.XOP_RECV:
            tmp = torch.empty(o["count"], dtype=view.dtype, device="cpu" if dist.get_backend() == "gloo" else view.device)
            pending.append((dist.irecv(tmp, src=o["peer"]), tmp, view))
        elif k == hw.XOP_REDUCE:
            tmp = _staged(view).clone()
            dist.reduce(tmp, dst=o["peer"], op=dist.ReduceOp.SUM)
            if o["out"] >= 0:
                bufs[o["out"]][o["offset"]:o["offset"] + o["count"]].copy_(tmp)
        elif k == hw.XOP_BCAST:
            tmp = _staged(view).clone()
            dist.broadcast(tmp, src=o["peer"])
            view.copy_(tmp)
    for work, tmp, view in pending:
        work.wait()
        if tmp is not None:
            view.copy_(tmp)


def broadcast_x(x: torch.Tensor, src: int = 0) -> torch.Tensor:
    """x replicated from rank `src` to every rank (broadcast once, then resident)."""
    buf = _staged(x)
    dist.broadcast(buf, src=src)
    if buf is not x:
        x.copy_(buf)
    return x


def max_over_ranks(value: float, device) -> float:
    t = torch.tensor([value], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        t = _staged(t)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device):
    t = torch.tensor(values, dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        t = _staged(t)
        dist.all_reduce(t)
    return [float(v) for v in t.tolist()]


_RANK0_CALLS = [0]


def rank0_only(fn, timeout_s: float, passed=lambda r: True):
    """fn() on rank 0 while every other rank waits on the process group's store -- host only, so
    no collective kernel spins on the GPUs fn may drive itself (bench.py's N-unit drop-in child
    uses every GPU of the node). Returns (fn's result on rank 0, None elsewhere; status), status
    the same on every rank that saw it: "ok", "fail" (passed(result) is false), "error" (fn
    raised on rank 0; the result is then {"error": ...}) or, on a waiting rank, "timeout" when
    rank 0 gave no status within timeout_s."""
    import datetime
    _RANK0_CALLS[0] += 1
    key = f"spmv_rank0_only_{_RANK0_CALLS[0]}"
    store = dist.distributed_c10d._get_default_store()
    if dist.get_rank() == 0:
        try:
            res = fn()
            status = "ok" if passed(res) else "fail"
        except Exception as e:
            res, status = {"error": f"{type(e).__name__}: {str(e)[:300]}"}, "error"
        store.set(key, status)
        return res, status
    try:
        store.wait([key], datetime.timedelta(seconds=timeout_s))
        return None, store.get(key).decode()
    except Exception:
        return None, "timeout"


def slice_counts(bounds) -> np.ndarray:
    b = np.asarray(bounds, np.int64)
    return np.diff(b)
