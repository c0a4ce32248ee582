#!/usr/bin/env python3
"""SpMV benchmark on MI355X — BASELINE.json metric "SpMV GFLOP/s + effective HBM GB/s
(% roofline), fp64, 1/2/4/8 MI355X".

A step = one y = A*x over the workload's matrix, through the C-ABI plan (the automatically chosen
kernel: the panel sweep for the power-law matrix, the flagged tiles for the banded one), with A,
x and y resident in HBM before the timed region. The K timed steps are replayed from one hipGraph
(spmv_plan_run_graph, captured and warmed before the timed region); the same K steps with one
host launch each are timed first (graph.eager_ms_per_step), and their HIP-event kernel times give
the roofline. For a split plan (the N >= 4 strong-scaling slices: panels cut into pieces whose
partial sums a second kernel adds) the graph carries the combine of step k as extra blocks of step
k + 1's sweep launch, which run in that sweep's tail, and one combine kernel after the last step
(DESIGN.md §6): every step still computes all of y, but a step's time can then fall below the
eager sweep + combine time of one SpMV.

Workloads:
  powerlaw (default, config 3): n = m = 10,000,000, nnz = 160,000,000, Pareto(2) row lengths
      (mean 16, max ~2e4), columns spread over [0,m), fp64. BASELINE's target is quoted here.
  banded   (config 2): n = m = 1,000,000, 16 nnz/row.
  --dtype f32 (config 5): the power-law matrix in fp32.
Multi-GPU (--gpus N, one process per GPU, torch.distributed over RCCL):
  --scaling strong (default for N > 1; config 4): the single 10M/160M matrix split into N
      nnz-balanced row slices (csr_hw.cpp:459-468), x replicated; value = 2 * 160M / the
      max-over-ranks time of one SpMV (compute-only: every rank's slice, no collective inside
      the timed step). The y exchange (RCCL gather of the disjoint slices, RCCL reduce of
      full-length partials = accum_results' +=, and the all-gather of the iterative form) is
      timed separately in "exchange", with the end-to-end rate beside it.
  --scaling weak: rank r owns its own 10M-row / 160M-nnz row partition of an (N*10M) x 10M
      matrix; value = total nnz of all ranks * 2 / max-over-ranks time. A strong run reports the
      weak measurement as the side field "weak_companion" (and a weak run the strong one as
      "strong_companion").

Extra JSON fields: roofline (dominant kernel of the plan: k_spmv_sweep_packed for the power-law
matrix, k_spmv_tiles for the banded one; HIP events on its launch stream),
cpu_baseline (the oracle's restatement of spmv_gold, 1 thread, on the host of the GPU box),
parity (full-size componentwise-scaled error vs that oracle run; mandatory at every N: a failed
or missing check prints value null / valid false and exits 3), dropin (the drop-in boundary
itself: create_csr_hw_matrix -> spmv_hw -> verification in a child process, the reference's
"Matrix read", "Hardware execution", "Result accumulation" and "Total" times; at N > 1 rank 0
runs it with N units merged by the library's RCCL reduce, then with the default host merge,
dropin.host_merge), value_e2e (2 nnz / (SpMV step +
the exchange that completes y); = value at N = 1),
lds_xtiles (power-law, 1 GPU: the same matrix through kernel 4, the reference's dataflow with a
block of x in LDS per workgroup -- the technique BASELINE configs 3/5 name -- timed beside the
headline kernel), binned (power-law, 1 GPU: the same matrix through kernel 6, the two-pass
gather-free alternative), deterministic (power-law, 1 GPU: the same matrix with SPMV_SWEEP_DETERMINISTIC=1,
bitwise reproducible y, timed the same way), side_configs (1 GPU: BASELINE config 2, banded
1M x 16 fp64, and config 5, the power-law matrix in fp32, each timed the same way with its own
roofline and oracle parity).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "spmv-fpga_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
DRIVER_LIMIT_S = 600.0  # the driver's limit on one bench run (BENCH_r05.json run.timeout_s)
RUN_TIMEOUT_DEFAULT = 480.0  # the run's own deadline: below DRIVER_LIMIT_S with --spawn-grace to spare


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["powerlaw", "banded"], default="powerlaw")
    ap.add_argument("--dtype", choices=["f64", "f32"], default="f64")
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--nnz", type=int, default=None)
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="default: strong (config 4) when --gpus > 1, weak (= single GPU) otherwise")
    ap.add_argument("--no-cpu", action="store_true",
                    help="skip the CPU baseline timing (the full-size parity check always runs)")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in boundary measurement (create_csr_hw_matrix -> spmv_hw -> "
                         "verification in a child process, the reference's run.elf timings)")
    ap.add_argument("--dropin-reps", type=int, default=5, help="spmv_hw calls of the drop-in measurement")
    ap.add_argument("--extras-timeout", type=float, default=None,
                    help="seconds the reported-only fields after the verified measurement may take before "
                         "the line is printed without them (default: half the run timeout at N = 1, 3/8 of "
                         "it at N > 1)")
    ap.add_argument("--extras-timeout-status", type=int, default=0,
                    help="exit status after the watchdog printed the line (the line stays valid: it "
                         "carries `extras_timeout`, and at N > 1 its parity already passed; set e.g. 3 to "
                         "make a hang visible to an exit-code check)")
    ap.add_argument("--no-det", action="store_true",
                    help="skip the deterministic-sweep side line (SPMV_SWEEP_DETERMINISTIC=1)")
    ap.add_argument("--no-xtiles", action="store_true",
                    help="skip the LDS x-tile (kernel 4, blocked) measurement beside the headline")
    ap.add_argument("--no-strong-companion", action="store_true",
                    help="N > 1 weak runs: skip the config-4 strong-scaling companion measurement")
    ap.add_argument("--no-weak-companion", action="store_true",
                    help="N > 1 strong runs: skip the weak-scaling companion measurement")
    ap.add_argument("--no-native-exchange", action="store_true",
                    help="N > 1: skip the library's own RCCL exchange (spmv_mgpu_create_rank)")
    ap.add_argument("--no-side-configs", action="store_true",
                    help="1 GPU: skip the config-2 (banded fp64) and config-5 (power-law fp32) side lines")
    ap.add_argument("--dist-rehearsal", action="store_true",
                    help="1 GPU: run the N > 1 code path as the one rank of an RCCL ('nccl') process "
                         "group -- its collectives, parity gather, exchange fields and the library's "
                         "own clique on the hardware (the path of the 8-GPU run, at world size 1)")
    ap.add_argument("--slice-of", type=int, default=None,
                    help="with --dist-rehearsal: the one rank holds rank 0's slice of an N-way strong cut "
                         "(e.g. 8: the split plan, serial chain and behind form of an 8-GPU rank, over RCCL)")
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the row-parallel CPU line (the box's CPU share is 16)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC traffic summary written by tools/pmc_traffic.py")
    ap.add_argument("--spawn-grace", type=float, default=60.0,
                    help="self-launch: seconds the other ranks may run on after one rank failed (non-zero "
                         "status), or after a rank finished cleanly (for rank 0 only once it printed its "
                         "line: it alone does work after the last collective); ranks still running then "
                         "are hung, killed, and the run fails")
    ap.add_argument("--run-timeout", type=float, default=RUN_TIMEOUT_DEFAULT,
                    help="seconds the whole run may take (below the driver's 600 s limit): then every rank "
                         "is killed and one JSON error line names each rank's last stage; exit status 124")
    ap.add_argument("--collective-timeout", type=float, default=None,
                    help="N > 1: timeout of every torch.distributed collective (init_process_group; "
                         "default min(120, run timeout / 4))")
    ap.add_argument("--dry-launch", action="store_true",
                    help="every rank prints its launch environment as JSON and exits before any GPU call")
    ap.add_argument("--dry-launch-rc", default="",
                    help="with --dry-launch: RANK:RC[,RANK:RC] exit codes of those ranks (launcher tests; "
                         "RC < 0 kills the rank with signal -RC, 'hang' makes it sleep before its line, "
                         "'teardown-hang' after it)")
    a = ap.parse_args(argv)
    if a.dist_rehearsal and a.gpus != 1:
        ap.error("--dist-rehearsal is the one-GPU form of the N > 1 path")
    if a.slice_of is not None and not (a.dist_rehearsal and a.slice_of >= 1):
        ap.error("--slice-of N needs --dist-rehearsal (and N >= 1)")
    if a.scaling is None:
        a.scaling = "strong" if a.gpus > 1 or a.slice_of else "weak"
    if a.slice_of and a.scaling != "strong":
        ap.error("--slice-of is a slice of the strong-scaling cut")
    a.multi = a.gpus > 1 or a.dist_rehearsal  # the N > 1 path: a process group, slices, exchange
    # every deadline derives from --run-timeout, which stays below the driver's limit (VERDICT r5
    # item 2): a run that reaches its extras by run/2 (N = 1) or 5/8 of it (N > 1) still prints
    # its line from the extras watchdog before the run deadline, and a hung collective gives up
    # well before either
    if a.extras_timeout is None:
        a.extras_timeout = a.run_timeout * (0.375 if a.multi else 0.5)
    if a.collective_timeout is None:
        a.collective_timeout = min(120.0, a.run_timeout / 4)
    return a


# ---- self-launch: `bench.py --gpus N` with no torchrun around it ---------------------------------
# The driver may start the N-GPU bench as `python bench.py --gpus N` (no launcher). Then this
# process starts N workers itself -- one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
# MASTER_ADDR / MASTER_PORT set as torch.distributed.run would -- before torch is even imported here
# (no HIP call happens in the parent), relays rank 0's JSON line (rank 0 writes to this stdout,
# the other ranks to stderr) and exits with the workers' worst status.

def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _status(rc):
    """A worker's exit status as a shell would report it (a signal k -> 128 + k)."""
    return 128 - rc if rc is not None and rc < 0 else (rc or 0)


STAGE_FD_ENV = "SPMV_BENCH_STAGE_FD"


def _die_with_parent():
    """preexec of a self-launched rank: SIGKILL when the parent dies (Linux prctl
    PR_SET_PDEATHSIG), so a killed parent leaves no rank behind on the GPU."""
    try:
        import ctypes
        ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGKILL, 0, 0, 0)
    except Exception:
        pass


def error_line(args, error, stages, rc):
    """The one JSON line of a run that produced no measurement: what failed and each rank's last
    stage (init, build, warmup, timed, parity, extras, emitted)."""
    return json.dumps({"metric": "SpMV GFLOP/s + effective HBM GB/s (% roofline), fp64, 1/2/4/8 MI355X",
                       "value": None, "unit": "GFLOP/s", "n_gpus": args.gpus, "error": error, "rc": rc,
                       "stage": {str(r): st for r, st in sorted(stages.items())}})


def spawn_ranks(args, argv):
    """Starts the N ranks and supervises them (csr_hw_wrapper.cpp:193-288 is
    synchronous and always reports). Every rank writes "rank:stage" lines into one pipe. The
    parent kills every rank and fails (status 124) when --run-timeout expires; once any rank has
    exited, the others get --spawn-grace seconds, then they are killed as hung. When rank 0 never
    printed its line, the parent prints one JSON error line with each rank's last stage."""
    n = args.gpus
    port = _free_port()
    r_fd, w_fd = os.pipe()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SPMV_BENCH_LAUNCHER="bench.py",
                   **{STAGE_FD_ENV: str(w_fd)})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else sys.stderr, pass_fds=(w_fd,),
                                      preexec_fn=_die_with_parent))
    os.close(w_fd)
    os.set_blocking(r_fd, False)

    def kill_all():
        for p in procs:
            if p.poll() is None:
                p.kill()
        for p in procs:
            p.wait()

    def stop(signum, _frame):  # the parent is being stopped: take the workers with it
        kill_all()
        sys.exit(128 + signum)

    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, stop)
    stages = {r: "launched" for r in range(n)}
    finished_at = {}  # rank -> when it reached "emitted" / "done" (its line is out; teardown only)
    pending = b""

    def read_stages():
        nonlocal pending
        while True:
            try:
                chunk = os.read(r_fd, 65536)
            except BlockingIOError:
                return
            if not chunk:
                return
            pending += chunk
            *lines, pending = pending.split(b"\n")
            for ln in lines:
                rank, _, st = ln.decode(errors="replace").partition(":")
                if rank.isdigit() and int(rank) in stages:
                    stages[int(rank)] = st
                    if st in ("emitted", "done"):
                        finished_at.setdefault(int(rank), time.monotonic())

    def grace_start(r, failed_at, clean_at):
        """When rank r's --spawn-grace starts: at the first failed rank; after a clean exit, at
        once for ranks > 0 (rank 0 still owes the line, the others only the collectives rank 0
        has passed), but for rank 0 only once it printed its line -- it alone does work after
        the last collective (the drop-in child, the CPU baseline), bounded by the run deadline."""
        if failed_at is not None:
            return failed_at
        if clean_at is None:
            return None
        if r != 0:
            return clean_at
        return max(clean_at, finished_at[0]) if 0 in finished_at else None

    t0 = time.monotonic()
    failed_at, clean_at, error, hung = None, None, None, []
    while any(p.poll() is None for p in procs):
        read_stages()
        now = time.monotonic()
        for p in procs:
            rc = p.poll()
            if rc is not None and rc != 0 and failed_at is None:
                failed_at = now
            if rc == 0 and clean_at is None:
                clean_at = now
        late = [r for r, p in enumerate(procs) if p.poll() is None
                and (grace_start(r, failed_at, clean_at) or now) + args.spawn_grace < now]
        if now - t0 > args.run_timeout or late:
            read_stages()
            hung = [r for r, p in enumerate(procs) if p.poll() is None]
            error = (f"run timeout: ranks {hung} still running after {args.run_timeout:g} s, killed"
                     if now - t0 > args.run_timeout else
                     f"ranks {hung} still running {args.spawn_grace:g} s after another rank exited, killed as hung")
            kill_all()
            break
        time.sleep(0.2)
    read_stages()
    os.close(r_fd)
    status = [_status(p.returncode) for p in procs]
    # a rank killed after it passed emit() ("emitted" / "done": the line is out, parity included at
    # N > 1) hung in its teardown (plan / process-group destruction): the measurement is complete,
    # so that kill is reported but does not fail the run
    teardown = [r for r in hung if stages.get(r) in ("emitted", "done")]
    for r in teardown:
        status[r] = 0
    if hung and len(teardown) == len(hung) and stages.get(0) == "emitted" and max(status) == 0:
        print(f"bench.py: {error}; every killed rank had finished (teardown hang), stages {stages}",
              file=sys.stderr, flush=True)
        return 0
    rc = 124 if error and error.startswith("run timeout") else max(status)
    if error or rc != 0:
        if stages.get(0) != "emitted":
            print(error_line(args, error or f"rank exit statuses {[_status(p.returncode) for p in procs]}",
                             stages, rc), flush=True)
        print(f"bench.py: {error or 'a rank failed'}; stages {stages}", file=sys.stderr, flush=True)
        rc = rc or 1
    return rc


def dry_launch(args):
    """--dry-launch: this rank's launch environment, before any GPU call; rank 0 on stdout."""
    env = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                          "MASTER_ADDR", "MASTER_PORT", "SPMV_BENCH_LAUNCHER")}
    rank = int(os.environ.get("RANK", "0"))
    deadlines = {k: getattr(args, k) for k in ("run_timeout", "extras_timeout", "collective_timeout", "spawn_grace")}
    print(json.dumps({"dry_launch": True, "gpus": args.gpus, "pid": os.getpid(), "deadlines": deadlines,
                      "driver_limit_s": DRIVER_LIMIT_S, **env}), flush=True)
    codes = dict(kv.split(":") for kv in args.dry_launch_rc.split(",") if kv)
    code = codes.get(str(rank), "0")
    stage("init")
    if code == "hang":
        stage("timed")  # a rank stuck where a collective would hold it
        time.sleep(3600)
    if code in ("0", "teardown-hang"):
        stage("emitted" if rank == 0 else "done")
    if code == "teardown-hang":
        time.sleep(3600)  # finished, then stuck in teardown (e.g. destroying a process group)
    if int(code) < 0:
        os.kill(os.getpid(), -int(code))
    return int(code)


_STAGE = ["start"]
_CHILDREN = []  # child processes of this rank (the drop-in run), ended with it


def _kill_children():
    for p in list(_CHILDREN):
        try:
            p.kill()
        except OSError:
            pass


def stage(name):
    """This rank's progress: kept for the run watchdog's error line and, under the self-launch
    parent, written to its pipe as "rank:stage"."""
    _STAGE[0] = name
    fd = os.environ.get(STAGE_FD_ENV)
    if fd:
        try:
            os.write(int(fd), f"{os.environ.get('RANK', '0')}:{name}\n".encode())
        except (OSError, ValueError):
            pass


def arm_run_watchdog(args):
    """Without the self-launch parent (N = 1, or ranks started by torch.distributed.run): the
    run's own deadline. After --run-timeout seconds rank 0 prints one JSON error line with its
    stage and every rank exits 124 -- a hang (rendezvous, barrier, a collective, a kernel that
    never ends) costs minutes, not the driver's whole limit."""
    if os.environ.get("SPMV_BENCH_LAUNCHER") == "bench.py":
        return None  # the parent supervises (spawn_ranks)

    def expire():
        if int(os.environ.get("RANK", "0")) == 0 and _STAGE[0] != "emitted":
            print(error_line(args, f"run timeout after {args.run_timeout:g} s", {0: _STAGE[0]}, 124), flush=True)
        sys.stdout.flush()
        _kill_children()
        os._exit(124)

    t = threading.Timer(args.run_timeout, expire)
    t.daemon = True
    t.start()
    return t


if __name__ == "__main__":
    _args = parse()
    if _args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(_args, sys.argv[1:]))
    if _args.dry_launch:
        arm_run_watchdog(_args)
        sys.exit(dry_launch(_args))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import spmv_dist  # noqa: E402
import spmv_hw  # noqa: E402


def setup_dist(args):
    """One process per GPU. RCCL ('nccl') by default; SPMV_BENCH_BACKEND=gloo with fewer GPUs than
    ranks is the single-GPU rehearsal of the multi-process path (ranks share device r % ndev)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:  # (without WORLD_SIZE, --gpus N > 1 self-launches N ranks: spawn_ranks)
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    backend = os.environ.get("SPMV_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks but only {ndev} GPUs (use SPMV_BENCH_BACKEND=gloo to rehearse)")
    dev_index = local % ndev
    torch.cuda.set_device(dev_index)
    if args.dist_rehearsal:  # one rank, its own rendezvous (no launcher around it)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
    if args.multi:
        import datetime
        # every collective (rendezvous, barriers, max-over-ranks, the exchange) gives up after
        # --collective-timeout instead of waiting forever for a rank that is gone or stuck
        tmo = datetime.timedelta(seconds=args.collective_timeout)
        stage("init")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
    return world, rank, dev_index


def barrier(world):
    if dist.is_initialized():
        dist.barrier()


def build_workload(lib, args, world, rank):
    """Returns (row_ptr, col, val, x, nr_cols, desc, rows_begin) on this rank's GPU."""
    if args.workload == "banded":
        n = args.rows or 1_000_000
        rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2 + 1000 * rank)
        x = spmv_hw.gen_vector(lib, n, seed=3)
        desc = {"workload": "banded", "rows": n, "cols": n, "nnz_per_row": 16, "nnz": n * 16}
        return rp, col, val, x, n, desc
    n = args.rows or 10_000_000
    z = args.nnz or 160_000_000
    if args.multi and args.scaling == "strong":
        rp_full, _ = lib.powerlaw_row_ptr(n, z, 65536, 4)
        b = lib.partition_rows(rp_full, args.slice_of or world)
        r0, r1 = spmv_dist.row_slice(b, rank)
        rp, col, val, scale = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4, row_begin=r0, row_end=r1)
        desc = {"workload": "powerlaw", "rows": n, "cols": n, "nnz": z, "slice_rows": [r0, r1]}
    else:
        # weak: rank r's own 10M-row partition (row-length seed 4 + 1000r, columns of global rows)
        rp, col, val, scale = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4 + 1000 * rank)
        desc = {"workload": "powerlaw", "rows": n, "cols": n, "nnz": z}
    x = spmv_hw.gen_vector(lib, n, seed=6)
    desc.update({"alpha": 2.0, "scale": round(scale, 4), "mean_nnz_per_row": z / n})
    return rp, col, val, x, n, desc


def host_csr(rp, col, val, x, y):
    """The measured matrix, x and the GPU's y in host memory (numpy), for the checks after the
    timed region."""
    return {"rp": rp.cpu().numpy().view(np.uint32), "col": col.cpu().numpy().view(np.uint32),
            "val": val.cpu().numpy(), "x": x.cpu().numpy(), "y": y.cpu().numpy()}


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    return oracle


def full_parity(h):
    """N = 1: the measured y against the oracle's restatement of spmv_gold (csr.cpp:184-194) on the
    whole matrix -- the check main.cpp:77-82 makes after every spmv_hw. Part of the measurement,
    not an extra: it runs before the extras watchdog, and a failed or missing check fails the
    run (status 3). Returns (parity, the oracle's y, its 1-thread time in ms)."""
    oracle = _oracle()
    n = len(h["rp"]) - 1
    ref = np.zeros(n, h["val"].dtype)
    t0 = time.perf_counter()
    oracle.spmv_gold_rows(h["rp"], h["col"], h["val"], h["x"], 0, n, out=ref)
    sw_ms = (time.perf_counter() - t0) * 1e3
    yg = h["y"]
    err = oracle.scaled_error(h["rp"], h["col"], h["val"], h["x"], ref, yg)
    abs_errors = oracle.verification_errors(ref, yg.astype(ref.dtype))
    yr, yg64 = ref.astype(np.float64), yg.astype(np.float64)
    nz = yr != 0
    rel = float(np.max(np.abs(yg64[nz] - yr[nz]) / np.abs(yr[nz]))) if nz.any() else 0.0
    tol = 1e-6 if ref.dtype == np.float64 else 1e-4
    # the north star's gate is the componentwise-scaled error; in fp64 the reference's own check
    # (verification: |dy| < 1e-5 absolute, csr_hw.cpp:1571-1590) must pass too. In fp32 that
    # absolute bound is below the rounding of |y| ~ 1e2 (spmv_gold sums in fp32, the kernels in
    # fp64), so its count is reported only
    parity = {"scope": f"full matrix ({n} rows) vs spmv_gold", "rows_checked": n, "max_scaled_err": err, "tol": tol,
              "max_rel_err": rel, "ref_abs_1e-5_errors": abs_errors,
              "pass": bool(err <= tol and (abs_errors == 0 or ref.dtype != np.float64))}
    return parity, ref, sw_ms


def cpu_baseline(lib, h, ref, reps, args_threads=16):
    """Times the oracle's restatement of spmv_gold (1 thread, -O2 -ffp-contract=off) on the
    same matrix in host memory; every run must give the parity check's y bit for bit."""
    oracle = _oracle()
    n = len(h["rp"]) - 1
    y = np.zeros(n, h["val"].dtype)
    times = []
    for _ in range(max(1, reps)):
        t0 = time.perf_counter()
        oracle.spmv_gold_rows(h["rp"], h["col"], h["val"], h["x"], 0, n, out=y)
        times.append(time.perf_counter() - t0)
    assert np.array_equal(y.view(np.uint8), ref.view(np.uint8))
    t = float(np.median(times))
    nnz = int(h["rp"][-1])
    try:
        model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
    except Exception:
        model = "unknown"
    base = {"value": round(2.0 * nnz / t / 1e9, 4), "unit": "GFLOP/s", "cores": 1, "kind": "port",
            "sample": f"full matrix ({n} rows, {nnz} nnz), median of {len(times)} runs, "
                      f"{t * 1e3:.1f} ms/SpMV, oracle/csr_ref.c spmv_gold, host {model}, "
                      f"nproc {os.cpu_count()}"}
    # second line: the same restatement row-parallel on host threads (ctypes
    # releases the GIL; nnz-balanced row slices), labelled as such
    from concurrent.futures import ThreadPoolExecutor
    nt = max(1, min(args_threads, os.cpu_count() or 1))
    bounds = lib.partition_rows(h["rp"], nt)
    y_mt = np.zeros(n, h["val"].dtype)

    def part(t):
        r0, r1 = int(bounds[t]), int(bounds[t + 1])
        if r1 > r0:
            oracle.spmv_gold_rows(h["rp"], h["col"], h["val"], h["x"], r0, r1, out=y_mt[r0:r1])

    times_mt = []
    with ThreadPoolExecutor(nt) as ex:
        for _ in range(max(1, reps)):
            t0 = time.perf_counter()
            list(ex.map(part, range(nt)))
            times_mt.append(time.perf_counter() - t0)
    t_mt = float(np.median(times_mt))
    assert np.array_equal(y_mt.view(np.uint8), ref.view(np.uint8))  # same rows, same order
    base["threads_line"] = {"value": round(2.0 * nnz / t_mt / 1e9, 4), "unit": "GFLOP/s", "cores": nt,
                            "kind": "port", "sample": f"same matrix, row-parallel restatement: {nt} threads "
                                                      f"over nnz-balanced row slices, median of {len(times_mt)} "
                                                      f"runs, {t_mt * 1e3:.1f} ms/SpMV"}
    return base


def _ref_lines(text, prefix):
    """The values of the reference's timing lines "<prefix> : <ms> ms elapsed" (csr_hw_wrapper.cpp:
    274,284-285, main.cpp:72) in the order printed."""
    out = []
    for ln in text.splitlines():
        if ln.startswith(prefix):
            try:
                out.append(float(ln.split(":", 1)[1].split()[0]))
            except (IndexError, ValueError):
                pass
    return out


def run_dropin(args, units, merge, ref, sw_ms, timeout):
    """The drop-in boundary itself: the reference's run.elf flow -- the host
    CSR through create_csr_hw_matrix + create_csr_hw_x_vector ("Matrix read time", main.cpp:67-72),
    spmv_hw ("Hardware execution time", "Result accumulation time", "Total time",
    csr_hw_wrapper.cpp:272-285) and verification against spmv_gold's y (main.cpp:77-82) -- in a
    child process (spmv-fpga_amd/dropin_main.py) on the same synthetic matrix, `units` units
    ("ComputeUnits", one per GPU) merged by `merge`. The first call's times are the reference's
    single-run numbers; the median over --dropin-reps calls is beside them. Every call is
    verified; `pass` is false when any call's verification is not 0."""
    import tempfile
    n = ref.shape[0]
    z = (args.nnz or 160_000_000) if args.workload == "powerlaw" else 16 * n
    fd, path = tempfile.mkstemp(suffix=".npy", prefix="spmv_dropin_ref_")
    os.close(fd)
    t0 = time.perf_counter()
    try:
        np.save(path, ref)
        cmd = [sys.executable, os.path.join(ROOT, "spmv-fpga_amd", "dropin_main.py"), "--workload", args.workload,
               "--dtype", args.dtype, "--rows", str(n), "--nnz", str(z), "--units", str(units), "--merge", merge,
               "--reps", str(max(1, args.dropin_reps)), "--ref", path, "--ab-unstreamed", str(max(1, args.dropin_reps))]
        env = {k: v for k, v in os.environ.items()
               if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR",
                            "MASTER_PORT", STAGE_FD_ENV, "SPMV_NGPUS", "SPMV_HW_MERGE")}
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=ROOT)
        _CHILDREN.append(p)  # killed by the watchdogs if the run ends while it works
        try:
            out, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            p.communicate()
            return {"error": f"drop-in child still running after {timeout:g} s, killed", "pass": None}
        finally:
            _CHILDREN.remove(p)
    finally:
        try:
            os.unlink(path)
        except OSError:
            pass
    js = [ln[len("DROPIN_JSON "):] for ln in out.splitlines() if ln.startswith("DROPIN_JSON ")]
    if p.returncode != 0 or not js:
        return {"error": f"drop-in child exit status {p.returncode}: {(err or out)[-400:]}", "pass": None}
    d = json.loads(js[-1])
    main_out, _, ab_out = out.partition("DROPIN_AB_UNSTREAMED")
    hw = _ref_lines(main_out, "Hardware execution time")
    ra = _ref_lines(main_out, "Result accumulation time")
    tot = _ref_lines(main_out, "Total time")
    ab_tot = _ref_lines(ab_out, "Total time")
    calls = d["calls"]
    if not (len(hw) == len(ra) == len(tot) == len(calls) >= 1):
        return {"error": f"drop-in child printed {len(hw)}/{len(ra)}/{len(tot)} timing lines for "
                         f"{len(calls)} spmv_hw calls", "pass": None}
    tol = 1e-6 if args.dtype == "f64" else 1e-4
    med = lambda v: round(float(np.median(v)), 4)  # noqa: E731
    res = {"api": "create_csr_hw_matrix + create_csr_hw_x_vector -> spmv_hw -> verification "
                  "(main.cpp:67-82 over the Part-1 C-ABI, child process spmv-fpga_amd/dropin_main.py)",
           "units": d["units"], "merge": merge, "rows": d["rows"], "nnz": d["nnz"],
           "matrix_read_ms": d["matrix_read_ms"],
           "hardware_execution_ms": hw[0], "result_accumulation_ms": ra[0], "total_ms": tot[0],
           "calls": len(calls),
           "median": {"hardware_execution_ms": med(hw), "result_accumulation_ms": med(ra), "total_ms": med(tot)},
           "per_call_ms": {"hardware_execution": hw, "result_accumulation": ra, "total": tot,
                           "spmv_hw_wall": [c["wall_ms"] for c in calls]},
           "total_gflops_median": round(2.0 * d["nnz"] / (med(tot) * 1e-3) / 1e9, 3) if med(tot) > 0 else None,
           "software_execution_ms": round(sw_ms, 3) if sw_ms else None,
           # the same matrix's calls with SPMV_HW_STREAM=0 (y copied back after the kernel; the
           # streamed copy-back applies to one-piece-per-panel sweep and binned plans with the host merge)
           "unstreamed_total_ms": {"median": med(ab_tot), "calls": ab_tot} if ab_tot else None,
           "verification": [c["verification"] for c in calls],
           "max_rel_diff_vs_spmv_gold": max(c["max_rel_diff"] for c in calls), "tol": tol,
           "storage_mb": d["storage_mb"], "csr_mb": d["csr_mb"],
           "child_wall_s": round(time.perf_counter() - t0, 2)}
    # fp64: every call's verification is 0 (main.cpp:77-82); fp32: the normwise difference only
    # (the absolute 1e-5 bound is below fp32 rounding of this y; see full_parity)
    res["pass"] = bool(res["max_rel_diff_vs_spmv_gold"] <= tol
                       and (args.dtype != "f64" or all(v == 0 for v in res["verification"])))
    if os.environ.get("SPMV_BENCH_INJECT") == "dropin":
        res["verification"][0], res["pass"] = 1, False  # test hook: a failed drop-in verification
    return res


def lds_xtiles(lib, args, rp, col, val, x, y_ref, ncols, dev_index, stream):
    """BASELINE configs 3/5 name LDS-staged x tiles with the reference's 2-D column blocking: the
    same matrix through kernel 4 (blocked.hip: a block of x in LDS per workgroup, per-block
    partials, block-ordered merge; VF = 1; blocks of 32768 fp32 / 16384 fp64 columns = 128 KiB
    of LDS), timed like the headline (HIP events over K launches) and checked against the
    headline's y. Reported beside `value`, which stays the automatic (fastest) kernel."""
    saved = {k: os.environ.get(k) for k in ("SPMV_HW_KERNEL", "SPMV_FPGA_BLOCK", "SPMV_FPGA_VF")}
    os.environ.update({"SPMV_HW_KERNEL": "blocked", "SPMV_FPGA_VF": "1",
                       "SPMV_FPGA_BLOCK": "32768" if args.dtype == "f32" else "16384"})
    try:
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, ncols, device=dev_index, stream=stream)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    st = plan.stats()
    y = torch.empty_like(y_ref)
    for _ in range(args.warmup):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    plan.set_timing(True)
    for _ in range(args.steps):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    ms, _, launches = plan.timing()
    plan.set_timing(False)
    diff = float(((y.double() - y_ref.double()).abs().max() / y_ref.double().abs().max().clamp_min(1e-300)).item())
    res = {"kernel": "k_blocked_partials + k_blocked_merge",
           "block_columns": 32768 if args.dtype == "f32" else 16384, "blocks": st["blocks"], "units": st["nr_tiles"],
           "ms_per_step": round(ms, 5), "launches": launches,
           "gflops": round(2.0 * st["nr_nzeros"] / (ms * 1e-3) / 1e9, 3),
           "alg_GBps": round(st["algorithmic_bytes"] / (ms * 1e-3) / 1e9, 2),
           "device_bytes": st["device_bytes"], "max_rel_diff_vs_value_kernel": diff}
    plan.destroy()
    del y
    torch.cuda.empty_cache()
    return res


def binned_side(lib, args, rp, col, val, x, y_ref, ncols, dev_index, stream):
    """The same matrix through the two-pass binned kernel (SPMV_HW_KERNEL=binned: products per
    column window, summed per row panel; 16 B per non-zero in fp32, 28 B in fp64), timed like
    the headline: the gather-free alternative to the sweep, measured beside it."""
    saved = os.environ.get("SPMV_HW_KERNEL")
    os.environ["SPMV_HW_KERNEL"] = "binned"
    try:
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, ncols, device=dev_index, stream=stream)
    finally:
        if saved is None:
            os.environ.pop("SPMV_HW_KERNEL", None)
        else:
            os.environ["SPMV_HW_KERNEL"] = saved
    y = torch.empty_like(y_ref)
    for _ in range(args.warmup):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    plan.set_timing(True)
    for _ in range(args.steps):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    ms, _, launches = plan.timing()
    plan.set_timing(False)
    diff = float(((y.double() - y_ref.double()).abs().max() / y_ref.double().abs().max().clamp_min(1e-300)).item())
    st = plan.stats()
    streamed = st["nr_nzeros"] * (2 * (2 * y_ref.element_size() + 2) - y_ref.element_size())
    res = {"kernel": "k_bin_mul + k_bin_acc", "env": "SPMV_HW_KERNEL=binned", "ms_per_step": round(ms, 5),
           "launches": launches, "gflops": round(2.0 * st["nr_nzeros"] / (ms * 1e-3) / 1e9, 3),
           "alg_GBps": round(st["algorithmic_bytes"] / (ms * 1e-3) / 1e9, 2),
           "streamed_bytes_per_launch": streamed,
           "streamed_GBps": round(streamed / (ms * 1e-3) / 1e9, 2),
           "max_rel_diff_vs_value_kernel": diff}
    plan.destroy()
    del y
    torch.cuda.empty_cache()
    return res


def deterministic_side(lib, args, rp, col, val, x, y_ref, ncols, dev_index, stream):
    """The same matrix with SPMV_SWEEP_DETERMINISTIC=1 (k_spmv_sweep_turn: LDS adds in a fixed
    (iteration, wave, lane) order on the default layout), timed like the headline; y must be the
    same bits over the timed runs and a fresh run, and within 1e-13 of the headline's y."""
    saved = os.environ.get("SPMV_SWEEP_DETERMINISTIC")
    os.environ["SPMV_SWEEP_DETERMINISTIC"] = "1"
    try:
        plan = spmv_hw.Plan.from_device(lib, rp, col, val, ncols, device=dev_index, stream=stream)
    finally:
        if saved is None:
            os.environ.pop("SPMV_SWEEP_DETERMINISTIC", None)
        else:
            os.environ["SPMV_SWEEP_DETERMINISTIC"] = saved
    y0 = torch.empty_like(y_ref)
    plan.run(x, y0, stream)
    y = torch.empty_like(y_ref)
    for _ in range(args.warmup):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    plan.set_timing(True)
    for _ in range(args.steps):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    ms, _, launches = plan.timing()
    plan.set_timing(False)
    itype = torch.int64 if y.element_size() == 8 else torch.int32
    bitwise = bool(torch.equal(y.view(itype), y0.view(itype)))
    diff = float(((y.double() - y_ref.double()).abs().max() / y_ref.double().abs().max().clamp_min(1e-300)).item())
    st = plan.stats()
    res = {"kernel": "k_spmv_sweep_turn", "env": "SPMV_SWEEP_DETERMINISTIC=1", "ms_per_step": round(ms, 5),
           "launches": launches, "gflops": round(2.0 * st["nr_nzeros"] / (ms * 1e-3) / 1e9, 3),
           "alg_GBps": round(st["algorithmic_bytes"] / (ms * 1e-3) / 1e9, 2),
           "bitwise_over_runs": bitwise, "max_rel_diff_vs_value_kernel": diff}
    plan.destroy()
    del y, y0
    torch.cuda.empty_cache()
    return res


def side_config(args, name, dev, stream):
    """BASELINE configs 2 and 5 beside the headline (1 GPU): the matrix built by the same
    generator, the automatically chosen kernel timed like the headline (HIP events over K eager
    launches after W warm-ups give kernel_ms; K steps replayed from one hipGraph give
    ms_per_step), and y checked against the oracle's spmv_gold on the full matrix."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    dtype = np.float32 if name == "config5" else np.float64
    lib = spmv_hw.load(dtype)
    if name == "config2":
        n = 1_000_000
        rp, col, val = spmv_hw.gen_banded(lib, n, 16, seed=2)
        x = spmv_hw.gen_vector(lib, n, seed=3)
        desc = {"workload": "banded", "rows": n, "cols": n, "nnz_per_row": 16, "nnz": 16 * n, "dtype": "f64"}
    else:
        n, z = 10_000_000, 160_000_000
        rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4)
        x = spmv_hw.gen_vector(lib, n, seed=6)
        desc = {"workload": "powerlaw", "rows": n, "cols": n, "nnz": z, "dtype": "f32"}
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, n, device=dev.index, stream=stream)
    st = plan.stats()
    y = torch.empty(n, dtype=x.dtype, device=dev)
    # the side configs run after the CPU baseline, i.e. after seconds of an idle GPU: W launches
    # (a few ms) do not bring the clocks back up (config 5 measured 0.478 ms after the idle
    # spell, 0.450 ms in the same build without it, profiles/r03d_*), so the untimed warm-up also
    # lasts at least 0.2 s of back-to-back launches
    tw = time.perf_counter()
    k = 0
    while k < args.warmup or time.perf_counter() - tw < 0.2:
        plan.run(x, y, stream)
        k += 1
        if k % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    plan.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - t0) * 1e3 / args.steps
    kernel_ms, _, _ = plan.timing()
    plan.set_timing(False)
    # ms_per_step as for the headline: the K steps replayed from one hipGraph (captured and warmed
    # once, untimed), so a short kernel (config 2: ~27 us) is not measured through its host
    # launch gaps; the eager wall time stays beside it
    plan.run_graph(x, y, args.steps, stream)
    torch.cuda.synchronize()
    tg = time.perf_counter()
    plan.run_graph(x, y, args.steps, stream)
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - tg) * 1e3 / args.steps
    h = [t.cpu().numpy() for t in (rp, col, val, x)]
    r, c = h[0].view(np.uint32), h[1].view(np.uint32)
    ref = oracle.spmv_gold(r, c, h[2], h[3])
    err = oracle.scaled_error(r, c, h[2], h[3], ref, y.cpu().numpy())
    tol = 1e-6 if dtype == np.float64 else 1e-4
    alg = st["algorithmic_bytes"]
    names = {0: "k_spmv_tiles", 2: "k_spmv_sweep_packed" if st["format"] & 2 else "k_spmv_sweep", 5: "k_spmv_slices",
             6: "k_bin_mul + k_bin_acc"}
    res = {"config": desc, "ms_per_step": round(wall_ms, 5), "eager_ms_per_step": round(eager_ms, 5),
           "kernel_ms": round(kernel_ms, 5),
           "gflops": round(2.0 * st["nr_nzeros"] / (wall_ms * 1e-3) / 1e9, 3),
           "effective_GBps": round(alg / (wall_ms * 1e-3) / 1e9, 2),
           "roofline": {"bound": "hbm", "kernel": names.get(st["kernel"], str(st["kernel"])),
                        "achieved": round(alg / (kernel_ms * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBPS,
                        "frac": round(alg / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                        "alg_bytes_per_launch": alg},
           "parity": {"max_scaled_err": err, "tol": tol, "pass": bool(err <= tol)}}
    res["roofline"]["traffic"] = None
    if st["kernel"] == 6 and name == "config5":
        # PMC traffic of the two binned passes on this matrix: the latest summary
        # (profiles/binned_pmc.json, tools/pmc_binned.py), else round 2's
        for fn in ("binned_pmc.json", "r02_binned_pmc.json"):
            try:
                pmc = json.load(open(os.path.join(ROOT, "profiles", fn)))
                res["roofline"]["traffic"] = pmc["f32"]["hbm_bytes_per_spmv"]
                res["roofline"]["traffic_src"] = "profiles/" + fn
                break
            except Exception:
                continue
    elif name == "config2":
        # PMC traffic of this kernel on this matrix (profiles/traffic.json, key banded_f64), used
        # only when it was recorded for the kernel the plan chose
        try:
            tr = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))["banded_f64"]
            if tr.get("nnz") == st["nr_nzeros"] and tr["kernel"].split("<")[0] == names.get(st["kernel"]):
                res["roofline"]["traffic"] = tr["hbm_bytes_per_launch"]
        except Exception:
            pass
    # the fraction of HBM peak the kernel's MEASURED bytes move at: the algorithmic `frac` charges
    # compulsory CSR bytes (12 B/nnz fp64), which a compressed layout (e.g. 9 B/nnz narrow tiles)
    # does not read, so `frac` can exceed what the memory system did; `frac_traffic` cannot
    if res["roofline"]["traffic"]:
        res["roofline"]["achieved_traffic"] = round(res["roofline"]["traffic"] / (kernel_ms * 1e-3) / 1e9, 2)
        res["roofline"]["frac_traffic"] = round(res["roofline"]["achieved_traffic"] / HBM_PEAK_GBPS, 4)
    plan.destroy()
    del rp, col, val, x, y
    torch.cuda.empty_cache()
    return res


def native_exchange(lib, plan, x, ncols, counts, world, rank, dev, y_parity=None, reps=5):
    """The y exchange through the library's own RCCL path (Part 4 of the C-ABI,
    spmv_mgpu_create_rank): rank 0's RCCL id is shared over torch.distributed, every rank joins
    with its plan, and spmv_mgpu_run times the SpMV plus each exchange form with HIP events
    (compute / exchange, max over ranks).

    Every form's result is verified, against this SpMV's slices all-gathered
    through torch.distributed (independent of the library's clique) -- itself held, on rank 0, to
    the parity gather `y_parity` that was checked against the oracle: rank 0's gathered y and
    its reduced y (the ncclReduce of full-length partials, accum_results' += ), and every rank's
    all-gathered next x. `verified.pass` is false on any mismatch; the caller then fails the run."""
    ok = torch.tensor([1.0], device=dev)
    uid = b"\0" * 128
    try:
        uid = spmv_hw.mgpu_unique_id(lib)  # every rank: RCCL loads here
    except Exception:
        ok.fill_(0.0)
    t = spmv_dist._staged(torch.tensor(list(uid), dtype=torch.uint8, device=dev))
    dist.broadcast(t, src=0)
    uid = bytes(t.cpu().tolist())
    okt = spmv_dist._staged(ok)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    if float(okt.item()) < 1.0:
        return {"error": "RCCL could not be loaded on every rank"}
    bounds = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    mg, err = None, None
    try:
        mg = spmv_hw.MultiGpu.rank(lib, rank, world, uid, dev.index, bounds, ncols, plan)
    except Exception as e:  # the clique is formed; agree before any collective
        err = str(e)[:300]
    ok.fill_(0.0 if mg is None else 1.0)
    okt = spmv_dist._staged(ok)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    if float(okt.item()) < 1.0:
        if mg is not None:
            mg.destroy()
        return {"error": err or "spmv_mgpu_create_rank failed on another rank"}
    res = {"api": "spmv_mgpu_create_rank + spmv_mgpu_run (library RCCL clique, one rank per GPU)",
           "rccl_comm_count": mg.comm_count()}
    # the reference y of every form: this SpMV's slices, all-gathered over torch.distributed
    y_loc = torch.empty(int(counts[rank]), dtype=x.dtype, device=dev)
    plan.run(x, y_loc, torch.cuda.current_stream())
    torch.cuda.synchronize()
    y_all = spmv_dist.exchange_allgather(y_loc, counts).to(dev).double()
    del y_loc
    scale = float(y_all.abs().max().clamp_min(1e-300).item())
    tol = 1e-12 if x.element_size() == 8 else 1e-5  # two SpMVs differ in the LDS adds' order only
    inject = os.environ.get("SPMV_BENCH_INJECT")

    def rel(y_n):
        return float((y_n.to(dev).double() - y_all).abs().max().item()) / scale

    diffs = {"torch_allgather_vs_parity_gather": rel(y_parity) if (rank == 0 and y_parity is not None) else 0.0}
    mg.set_x_device(x)
    square = int(counts.sum()) == int(ncols)  # (--slice-of: the slices do not cover x; no all-gather)
    forms = [("gather", spmv_hw.MGPU_GATHER), ("reduce", spmv_hw.MGPU_REDUCE)]
    for name, mode in forms + ([("allgather", spmv_hw.MGPU_ALLGATHER)] if square else []):
        if mode == spmv_hw.MGPU_ALLGATHER:
            mg.set_x_device(x)
        for _ in range(2):
            mg.run(mode)
        cs, es = [], []
        for _ in range(reps):
            if mode == spmv_hw.MGPU_ALLGATHER:
                mg.set_x_device(x)  # every run computes A x, not A^k x
            mg.run(mode)
            c, e = mg.timing()
            cs.append(c)
            es.append(e)
        res[f"{name}_compute_ms"] = round(spmv_dist.max_over_ranks(float(np.median(cs)), dev), 5)
        res[f"{name}_exchange_ms"] = round(spmv_dist.max_over_ranks(float(np.median(es)), dev), 5)
        if mode == spmv_hw.MGPU_ALLGATHER:  # every rank's next x = A x
            x_next = torch.from_numpy(mg.y(spmv_hw.MGPU_ALLGATHER))
            if inject == "allgather" and rank == world - 1:
                x_next[-1] += 1.0  # test hook: a wrong all-gather result on the last rank
            diffs["allgather"] = rel(x_next)
        else:  # a stream of SpMVs, each exchange under the next kernels; rank 0 keeps the last y
            mg.run_pipelined(mode, 2)
            res[f"{name}_pipelined_ms_per_step"] = round(
                spmv_dist.max_over_ranks(mg.run_pipelined(mode, max(reps, 8)), dev), 5)
            diffs[name] = 0.0
            if rank == 0:
                y_n = torch.from_numpy(mg.y(mode))
                if inject == name:
                    y_n[0] += 1.0  # test hook (tests/test_gpu_bench.py): a wrong reduce / gather result
                diffs[name] = rel(y_n)
    diffs = {k: spmv_dist.max_over_ranks(v, dev) for k, v in diffs.items()}
    res["gather_max_rel_diff_vs_torch"] = diffs["gather"]
    res["verified"] = {"against": "this SpMV's slices all-gathered over torch.distributed; on rank 0 "
                                  "within tol of the oracle-checked parity gather",
                       "tol": tol, "max_rel_diff": diffs,
                       **{k: bool(v <= tol) for k, v in diffs.items()}}
    res["verified"]["pass"] = all(v <= tol for v in diffs.values())
    # iterative use: SpMV + all-gather of y into every rank's next x, steps
    # replayed from one hipGraph per rank (spmv_mgpu_run_graph; capture outside the timing)
    if square:
        mg.set_x_device(x)
        mg.run_graph(spmv_hw.MGPU_ALLGATHER, max(reps, 8))
        mg.set_x_device(x)
        res["allgather_graph_ms_per_step"] = round(
            spmv_dist.max_over_ranks(mg.run_graph(spmv_hw.MGPU_ALLGATHER, max(reps, 8)), dev), 5)
    mg.destroy()
    return res


def weak_companion(lib, args, world, rank, dev, stream):
    """Beside a strong-scaling run: every rank's own 10M-row / 160M-nnz partition (the weak
    workload), timed like the headline; value = total nnz of all ranks * 2 / max-over-ranks."""
    import copy
    a = copy.copy(args)
    a.scaling = "weak"
    rp, col, val, x, ncols, desc = build_workload(lib, a, world, rank)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, ncols, device=dev.index, stream=stream)
    st = plan.stats()
    del rp, col, val
    y = torch.empty(st["nr_rows"], dtype=x.dtype, device=dev)
    for _ in range(args.warmup):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    barrier(world)
    ms = spmv_dist.max_over_ranks((time.perf_counter() - t0) * 1e3 / args.steps, dev)
    nnz_all = spmv_dist.sum_over_ranks([float(st["nr_nzeros"])], dev)[0]
    res = {"n_gpus": world, "value": round(2.0 * nnz_all / (ms * 1e-3) / 1e9, 3), "unit": "GFLOP/s",
           "ms_per_step": round(ms, 5), "scaling": "weak", "nnz_per_rank": st["nr_nzeros"],
           "kernel": st["kernel"]}
    plan.destroy()
    del x, y
    torch.cuda.empty_cache()
    return res


def strong_companion(lib, args, world, rank, dev, stream):
    """Config 4 beside a weak-scaling run: the SAME 10M/160M matrix cut into `world` nnz-balanced
    row slices (one per rank), timed like the headline (warm-up, barrier-bracketed K steps, max
    over ranks), plus the RCCL y exchange of its slices: reduce of full-length partials (the
    accum_results '+=' mapping) and gather of the disjoint slices."""
    import copy
    a = copy.copy(args)
    a.scaling = "strong"
    rp, col, val, x, ncols, desc = build_workload(lib, a, world, rank)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, ncols, device=dev.index, stream=stream)
    st = plan.stats()
    del rp, col, val
    y = torch.empty(st["nr_rows"], dtype=x.dtype, device=dev)
    for _ in range(args.warmup):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    barrier(world)
    ms = spmv_dist.max_over_ranks((time.perf_counter() - t0) * 1e3 / args.steps, dev)
    nnz_all = spmv_dist.sum_over_ranks([float(st["nr_nzeros"])], dev)[0]
    cnt = [0.0] * world
    cnt[rank] = float(st["nr_rows"])
    counts = np.array(spmv_dist.sum_over_ranks(cnt, dev), dtype=np.int64)
    row_begin, n_total = int(counts[:rank].sum()), int(counts.sum())
    res = {"n_gpus": world, "value": round(2.0 * nnz_all / (ms * 1e-3) / 1e9, 3), "unit": "GFLOP/s",
           "ms_per_step": round(ms, 5), "slice_rows": desc.get("slice_rows"), "kernel": st["kernel"],
           "units": st["nr_tiles"]}
    for mode in ("reduce", "gather"):
        def exchange():
            return (spmv_dist.exchange_reduce(y, row_begin, n_total) if mode == "reduce"
                    else spmv_dist.exchange_gather(y, counts))
        exchange()
        torch.cuda.synchronize()
        barrier(world)
        te0 = time.perf_counter()
        for _ in range(3):
            exchange()
        torch.cuda.synchronize()
        barrier(world)
        res[f"{mode}_ms"] = round(spmv_dist.max_over_ranks((time.perf_counter() - te0) * 1e3 / 3, dev), 4)
    res["e2e_gflops_with_reduce"] = round(2.0 * nnz_all / ((ms + res["reduce_ms"]) * 1e-3) / 1e9, 2)
    res["e2e_gflops_with_gather"] = round(2.0 * nnz_all / ((ms + res["gather_ms"]) * 1e-3) / 1e9, 2)
    plan.destroy()
    return res


def distributed_parity(lib, args, world, rank, dev, y, st, held=None):
    """N > 1: the reference checks every spmv_hw result (main.cpp:77-82); so does this line.
    Strong scaling (config 4): every rank's y slice is gathered on rank 0 (spmv_dist.exchange_gather)
    and the assembled 10M-row y is checked against the oracle's spmv_gold of the whole matrix,
    regenerated on rank 0 by the same generator. Weak scaling (and the banded workload): every
    rank checks its own partition; the worst error over ranks is reported. Runs after the timed
    region, never inside it."""
    oracle = _oracle()
    dtype = np.float64 if args.dtype == "f64" else np.float32
    tol = 1e-6 if dtype == np.float64 else 1e-4

    def check(rp, col, val, x, y_test):
        h = [t.cpu().numpy() for t in (rp, col, val, x)]
        r, c = h[0].view(np.uint32), h[1].view(np.uint32)
        ref = oracle.spmv_gold(r, c, h[2], h[3])
        if held is not None:
            held["ref"] = ref  # (rank 0, strong: spmv_gold's y of the whole matrix, for the drop-in run)
        yt = y_test.cpu().numpy() if hasattr(y_test, "cpu") else y_test
        return oracle.scaled_error(r, c, h[2], h[3], ref, yt), oracle.verification_errors(ref, yt.astype(ref.dtype))

    if args.scaling == "strong" and args.workload == "powerlaw":
        cnt = [0.0] * world
        cnt[rank] = float(st["nr_rows"])
        counts = np.array(spmv_dist.sum_over_ranks(cnt, dev), dtype=np.int64)
        y_full = spmv_dist.exchange_gather(y, counts)
        if held is not None:
            held["y_full"] = y_full  # rank 0: the assembled y (the dependent form's check)
        res = {"scope": f"y of all {world} row slices gathered on rank 0 vs spmv_gold of the whole matrix"
                        if not args.slice_of else f"rank 0's slice of a {args.slice_of}-way cut vs spmv_gold of its rows",
               "rows_checked": int(counts.sum())}
        if rank == 0:
            n, z = args.rows or 10_000_000, args.nnz or 160_000_000
            r0 = held.get("row_begin", 0) if held is not None else 0  # (--slice-of: rank 0's slice)
            rp, col, val, _ = spmv_hw.gen_powerlaw(lib, n, n, z, seed=4, row_begin=r0,
                                                   row_end=r0 + int(counts.sum()))
            x = spmv_hw.gen_vector(lib, n, seed=6)
            err, nerr = check(rp, col, val, x, y_full)
            del rp, col, val, x
            torch.cuda.empty_cache()
        else:
            err, nerr = 0.0, 0
    else:
        rp, col, val, x, _, _ = build_workload(lib, args, world, rank)
        err, nerr = check(rp, col, val, x, y)
        del rp, col, val, x
        torch.cuda.empty_cache()
        res = {"scope": f"every rank's own partition vs spmv_gold (worst of {world} ranks)",
               "rows_checked": int(spmv_dist.sum_over_ranks([float(st["nr_rows"])], dev)[0])}
    err = spmv_dist.max_over_ranks(err, dev)
    nerr = int(spmv_dist.sum_over_ranks([float(nerr)], dev)[0])
    res.update({"max_scaled_err": err, "tol": tol, "ref_abs_1e-5_errors": nerr, "pass": bool(err <= tol)})
    return res


def serial_chain_ms(plan, x, y, steps, world, dev):
    """The K steps as a serial chain: K spmv_plan_run calls captured into one graph by the
    caller (torch.cuda.graph), so every step -- a split plan's sweep and its combine -- ends
    before the next begins, as one spmv_hw call is one complete SpMV (csr_hw_wrapper.cpp:200-285).
    Replayed once untimed, then timed; max over ranks."""
    g = torch.cuda.CUDAGraph()
    # thread_local: a process-group watchdog thread polling its events does not void the capture
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(steps):
            plan.run(x, y)
    g.replay()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    barrier(world)
    ms = spmv_dist.max_over_ranks((time.perf_counter() - t0) * 1e3 / steps, dev)
    del g
    return ms


def dependent_iteration(plan, x, y, st, steps, world, rank, dev, y_full, row0=0):
    """The dependent form (x <- A x): every step is this rank's SpMV into its
    slice and the all-gather of the slices into every rank's next x (spmv_dist.exchange_allgather),
    so step k + 1 cannot start before step k's exchange has ended. Timed over K steps from the
    headline's x, max over ranks. Checked: one step from that x gives, on every rank, the y the
    parity gather assembled on rank 0 (within 1e-12 relative in fp64, 1e-5 in fp32: the LDS adds'
    order)."""
    cnt = [0.0] * world
    cnt[rank] = float(st["nr_rows"])
    counts = np.array(spmv_dist.sum_over_ranks(cnt, dev), dtype=np.int64)
    nloc = int(st["nr_rows"])
    total = int(counts.sum())
    ys = torch.empty(nloc, dtype=y.dtype, device=dev)
    bufs = [x.clone(), x.clone()]

    def step(k):  # (row0 > 0 only for --slice-of: the gathered rows land at their own offset)
        src, dst = bufs[k % 2], bufs[(k + 1) % 2]
        plan.run(src, ys)
        spmv_dist.exchange_allgather(ys, counts, out=dst[row0:row0 + total])

    step(0)  # warm (communicator, staging buffers)
    bufs[0].copy_(x)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize()
    barrier(world)
    ms = spmv_dist.max_over_ranks((time.perf_counter() - t0) * 1e3 / steps, dev)
    bufs[0].copy_(x)
    step(0)  # x1 = A x on every rank
    torch.cuda.synchronize()
    diff = 0.0
    if rank == 0 and y_full is not None:
        ref = y_full.to(dev).double()
        diff = float(((bufs[1][row0:row0 + total].double() - ref).abs().max()
                      / ref.abs().max().clamp_min(1e-300)).item())
    diff = spmv_dist.max_over_ranks(diff, dev)
    tol = 1e-12 if y.element_size() == 8 else 1e-5  # two runs of the sweep differ in the LDS adds' order
    del bufs, ys
    return {"ms_per_step": round(ms, 5), "steps": steps,
            "form": "SpMV into the rank's slice, then all-gather of the slices into every rank's next x",
            "x1_max_rel_diff_vs_parity_y": diff, "tol": tol, "pass": bool(diff <= tol)}


def value_e2e(out, ms, nnz_all):
    """value_e2e: 2 nnz / (the serial SpMV step + the exchange that completes y), beside the
    compute-only `value` -- the reference's "Total time" is hardware + accumulation
    (csr_hw_wrapper.cpp:276-285). At N > 1 the exchange is the library's own RCCL reduce of
    full-length partials (spmv_mgpu_run MGPU_REDUCE: accum_results' +=, exchange only, median
    of 5, max over ranks, verified), else torch.distributed's reduce; at N = 1 there is none. The
    form also gives the rate with the library's gather of the disjoint slices (with_gather)."""
    if out["n_ranks"] == 1 and not out["dist_rehearsal"]:
        return out["value"], {"form": "one GPU: the SpMV is the whole job (no exchange)"}
    ex = out.get("exchange") if isinstance(out.get("exchange"), dict) else {}
    nat = ex.get("native") if isinstance(ex.get("native"), dict) else {}
    if "reduce_exchange_ms" in nat:
        ex_ms, src = nat["reduce_exchange_ms"], "exchange.native.reduce_exchange_ms (library RCCL reduce)"
    elif "reduce_ms" in ex:
        ex_ms, src = ex["reduce_ms"], "exchange.reduce_ms (torch.distributed reduce)"
    else:
        return None, {"form": "no exchange was measured"}
    form = {"form": "serial SpMV step (ms_per_step) + the y reduce onto rank 0, per SpMV", "ms_per_step": ms,
            "exchange_ms": ex_ms, "exchange_src": src,
            "value_is": "compute-only: max-over-ranks SpMV step, no collective inside the timed step"}
    if "gather_exchange_ms" in nat:  # the bandwidth-optimal form beside it (disjoint slices to rank 0)
        g = nat["gather_exchange_ms"]
        form["with_gather"] = {"value": round(2.0 * nnz_all / ((ms + g) * 1e-3) / 1e9, 3), "exchange_ms": g,
                               "exchange_src": "exchange.native.gather_exchange_ms (library RCCL gather, verified)"}
    return round(2.0 * nnz_all / ((ms + ex_ms) * 1e-3) / 1e9, 3), form


def main():
    args = parse()
    run_watchdog = arm_run_watchdog(args)
    world, rank, local = setup_dist(args)
    dtype = np.float64 if args.dtype == "f64" else np.float32
    lib = spmv_hw.load(dtype)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream()

    t_setup = time.perf_counter()
    stage("build")
    rp, col, val, x, ncols, desc = build_workload(lib, args, world, rank)
    plan = spmv_hw.Plan.from_device(lib, rp, col, val, ncols, device=local, stream=stream)
    st = plan.stats()
    y = torch.empty(st["nr_rows"], dtype=x.dtype, device=dev)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t_setup
    keep_csr = not args.multi  # N = 1: the full-size parity check reads the matrix after the timed region
    want_xtiles = not args.multi and args.workload == "powerlaw" and not args.no_xtiles
    if not keep_csr and not want_xtiles:
        del rp, col, val
        torch.cuda.empty_cache()

    stage("warmup")
    for _ in range(args.warmup):
        plan.run(x, y, stream)
    torch.cuda.synchronize()

    stage("timed")
    if os.environ.get("SPMV_BENCH_INJECT") == "hang" and rank == world - 1:
        time.sleep(3600)  # test hook (tests/test_gpu_bench.py): a rank that never reaches the barrier
    # 1) eager: one host launch per step, the main kernel timed with HIP events on its stream
    #    (roofline.achieved; rocprofv3 sees the same launches)
    barrier(world)
    torch.cuda.synchronize()
    plan.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(x, y, stream)
    torch.cuda.synchronize()
    barrier(world)
    t1 = time.perf_counter()
    kernel_ms, _, launches = plan.timing()
    plan.set_timing(False)
    eager_ms = spmv_dist.max_over_ranks((t1 - t0) * 1e3 / args.steps, dev)
    kernel_ms_max = spmv_dist.max_over_ranks(kernel_ms, dev)
    per_rank = [0.0] * world  # every rank's dominant-kernel time (load balance of the slices)
    per_rank[rank] = kernel_ms
    kernel_ms_ranks = spmv_dist.sum_over_ranks(per_rank, dev) if args.multi else [kernel_ms]

    # 2) the headline: the same K steps replayed from one hipGraph (spmv_plan_run_graph, captured
    #    and warmed once, untimed) -- no host launch gap between steps
    plan.run_graph(x, y, args.steps, stream)  # capture + warm-up
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    tg0 = time.perf_counter()
    plan.run_graph(x, y, args.steps, stream)
    torch.cuda.synchronize()
    barrier(world)
    product_ms = spmv_dist.max_over_ranks((time.perf_counter() - tg0) * 1e3 / args.steps, dev)
    product_form = ("behind" if st["format"] & 256 else "dag" if st["format"] & 512 else "serial")
    # 3) step semantics. spmv_plan_run_graph pipelines a split plan's steps
    #    (the N >= 4 slices: step k's combine rides in step k + 1's sweep launch), which only
    #    independent SpMVs of the same x allow. `value` is the serial chain -- every step complete
    #    before the next starts, like the one-GPU headline, whose plan has no combine (its replay
    #    IS the serial chain) -- so the driver's N-GPU / 1-GPU ratio compares like with like.
    if product_form == "serial":
        ms = product_ms
    else:
        ms = serial_chain_ms(plan, x, y, args.steps, world, dev)
    graph = {"iters": args.steps, "ms_per_step": round(ms, 5), "timed": "headline (value, ms_per_step)",
             "eager_ms_per_step": round(eager_ms, 5),
             "value_form": "serial: each SpMV (sweep, then the combine of a split plan) ends before the next begins",
             # how spmv_plan_run_graph orders the steps (plan stats format bits 8 / 9)
             "run_graph_form": product_form, "run_graph_ms_per_step": round(product_ms, 5)}
    step_forms = {"value_form": "serial", "serial_ms_per_step": round(ms, 5),
                  "behind_ms_per_step": round(product_ms, 5) if product_form == "behind" else None,
                  "independent_pipelined_ms_per_step": round(product_ms, 5),
                  "dependent_ms_per_step": None,
                  "note": "serial = value (K SpMVs of one x, each complete before the next); behind = "
                          "spmv_plan_run_graph on a split plan (step k's combine inside step k + 1's sweep: "
                          "independent SpMVs only); dependent = x <- A x with the all-gather exchange in every "
                          "step (compute + exchange)"}

    xtiles = det = binned = None
    if want_xtiles:  # reported beside the headline, never fatal to it
        try:
            xtiles = lds_xtiles(lib, args, rp, col, val, x, y, ncols, local, stream)
        except Exception as e:
            xtiles = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
        if st["kernel"] != 6:
            try:
                binned = binned_side(lib, args, rp, col, val, x, y, ncols, local, stream)
            except Exception as e:
                binned = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
        if not args.no_det:
            try:
                det = deterministic_side(lib, args, rp, col, val, x, y, ncols, local, stream)
            except Exception as e:
                det = {"error": f"{type(e).__name__}: {str(e)[:300]}"}
        if not keep_csr:
            del rp, col, val
            torch.cuda.empty_cache()

    # the Part-1 boundary (spmv_hw) hands over host buffers: PCIe cost of x in and y out,
    # pinned host memory (reported only; never part of `value`)
    host = {}
    for name, t in (("x_h2d_ms", x), ("y_d2h_ms", y)):
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        reps = 3
        torch.cuda.synchronize()
        th0 = time.perf_counter()
        dst = torch.empty_like(t) if name == "x_h2d_ms" else h  # x itself stays intact
        src = h if name == "x_h2d_ms" else t
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        host[name] = round((time.perf_counter() - th0) * 1e3 / reps, 4)
        del h, dst

    nnz_local = st["nr_nzeros"]
    alg_local = st["algorithmic_bytes"]
    nnz_all, alg_all = spmv_dist.sum_over_ranks([float(nnz_local), float(alg_local)], dev)
    if args.multi and args.scaling == "strong":
        # one matrix: x and the row_ptr sentinel count once, not once per rank
        alg_all -= (world - 1) * (st["nr_cols"] * np.dtype(dtype).itemsize + 4)

    gflops = 2.0 * nnz_all / (ms * 1e-3) / 1e9
    graph["eager_gflops"] = round(2.0 * nnz_all / (eager_ms * 1e-3) / 1e9, 3)
    eff_gbps = alg_all / (ms * 1e-3) / 1e9
    # roofline of the dominant kernel: algorithmic bytes of one launch / mean launch duration
    # (max over ranks: every rank's dominant kernel has the same per-launch algorithmic bytes)
    kernel_ms = kernel_ms_max
    achieved = alg_local / (kernel_ms * 1e-3) / 1e9 if kernel_ms > 0 else 0.0
    # the dominant kernel of this plan; its PMC traffic is taken from profiles/traffic.json only
    # when that summary was recorded for the same workload, size and kernel
    if st["kernel"] == 2:
        kname = "k_spmv_sweep_packed" if st["format"] & 2 else "k_spmv_sweep"
    elif st["kernel"] == 1:
        kname = "k_spmv_gold"
    elif st["kernel"] == 3:
        kname = "k_spmv_fpga"
    elif st["kernel"] == 4:
        kname = "k_blocked_partials"
    elif st["kernel"] == 5:
        kname = "k_spmv_slices"
    elif st["kernel"] == 6:
        kname = "k_bin_mul + k_bin_acc"
    else:
        kname = "k_spmv_tiles"
    traffic = None
    l2_requests = None  # TCC_HIT_sum + TCC_MISS_sum per launch, same PMC passes
    if os.path.exists(args.traffic):
        try:
            tr = json.load(open(args.traffic))
            key = f"{desc['workload']}_{args.dtype}"
            if (key in tr and tr[key].get("nnz") == nnz_local
                    and tr[key].get("kernel", "").split("<")[0] == kname
                    and tr[key].get("format", st["format"]) == st["format"]  # same entry layout
                    and (kname != "k_spmv_tiles"  # template arg CB: bytes per stored column
                         or tr[key]["kernel"].endswith(
                             ", %d>" % (1 if st["format"] & 8 else 2 if st["format"] & 1 else 4)))):
                traffic = tr[key]["hbm_bytes_per_launch"]
                cnt = next(iter(tr[key].get("counters", {}).values()), {})
                if "TCC_HIT_sum" in cnt and "TCC_MISS_sum" in cnt:
                    l2_requests = cnt["TCC_HIT_sum"] + cnt["TCC_MISS_sum"]
        except Exception:
            traffic = None

    # the achievable HBM read rate measured on MI355X by tools/hbm_calib (dwordx4 stream read,
    # SURVEY §8d "report both"); the roofline fraction stays against the 8 TB/s spec
    # and the L2 request ceiling measured by the same tool (L2-resident random gathers): the bound
    # of the sweep kernel, whose x gathers hit L2
    stream_peak, l2_peak = None, None
    try:
        for line in open(os.path.join(ROOT, "profiles", "r01_hbm_calib.jsonl")):
            rec = json.loads(line)
            if rec.get("test") == "stream_read":
                stream_peak = rec["GBps"]
            if str(rec.get("test", "")).startswith("gather_table_") and rec["test"].endswith("KB") \
                    and int(rec["test"][13:-2]) <= 4096:
                l2_peak = max(l2_peak or 0.0, rec["Greq_per_s"])
    except (OSError, ValueError):
        stream_peak, l2_peak = None, None
    l2 = None
    if l2_requests and kernel_ms > 0:
        rate = l2_requests / (kernel_ms * 1e-3) / 1e9
        l2 = {"requests_per_launch": int(l2_requests), "achieved_G_per_s": round(rate, 1),
              "peak_G_per_s": l2_peak, "frac": round(rate / l2_peak, 4) if l2_peak else None,
              "src": "TCC_HIT_sum+TCC_MISS_sum (profiles/traffic.json) / kernel_ms; peak = "
                     "L2-resident gather rate (profiles/r01_hbm_calib.jsonl)"}

    out = {
        "metric": "SpMV GFLOP/s + effective HBM GB/s (% roofline), fp64, 1/2/4/8 MI355X",
        "value": round(gflops, 3),
        "unit": "GFLOP/s",
        "n_gpus": world,
        "n_ranks": dist.get_world_size() if dist.is_initialized() else 1,
        "launcher": os.environ.get("SPMV_BENCH_LAUNCHER") or ("torch.distributed.run" if world > 1 else None),
        "dist_rehearsal": bool(args.dist_rehearsal),
        "slice_of": args.slice_of,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 5),
        "higher_is_better": True,
        "scaling": args.scaling if args.multi else "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (splitmix64 generator, SURVEY.md §8d)",
        "config": dict(desc, parallelism=f"row-slice x{world}", dtype=args.dtype),
        "effective_GBps": round(eff_gbps, 2),
        "roofline_pct": round(100.0 * eff_gbps / (HBM_PEAK_GBPS * world), 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                     "peak_measured": stream_peak,
                     "frac_of_measured": round(achieved / stream_peak, 4) if stream_peak else None,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "frac_traffic": (round(traffic / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                                      if traffic and kernel_ms > 0 else None),
                     "kernel": kname, "kernel_ms": round(kernel_ms, 5), "l2": l2,
                     "kernel_ms_per_rank": [round(v, 5) for v in kernel_ms_ranks],
                     "kernel_launches": launches, "alg_bytes_per_launch": alg_local},
        "cpu_baseline": None,
        "parity": None,
        "exchange": None,
        "graph": graph,
        "step_forms": step_forms,
        "strong_companion": None,
        "weak_companion": None,
        "lds_xtiles": xtiles,
        "binned": binned,
        "deterministic": det,
        "side_configs": None,
        "host_copy": host,
        "plan": {k: st[k] for k in ("nr_tiles", "tile_nnz", "device_bytes", "kernel", "format", "nr_nonempty_rows")},
        "setup_s": round(setup_s, 2),
    }
    emitted = threading.Event()

    def emit(note=None):
        if rank == 0 and not emitted.is_set():
            emitted.set()
            line = dict(out, extras_timeout=note) if note else out
            print(json.dumps(line), flush=True)
        stage("emitted" if rank == 0 else "done")

    def fail_run(what, detail):
        """A check of what the line reports did not pass: the line is printed as an invalid
        measurement (value null, the measured number kept as value_unverified) and the run ends
        with status 3 on every rank -- an rc-blind reader cannot take it for a result."""
        out.update(valid=False, error=what, value_unverified=out["value"], value=None)
        emit()
        print(f"bench.py rank {rank}: {what}: {detail}", file=sys.stderr, flush=True)
        os._exit(3)

    # parity is part of the measurement, not an extra (main.cpp:77-82 verifies every spmv_hw
    # result), at every N. It runs under the run deadline and the collective timeout only, before
    # the extras watchdog; a parity that errors or fails ends the run with status 3.
    held = {"row_begin": (desc.get("slice_rows") or [0])[0] if args.slice_of else 0}
    if os.environ.get("SPMV_BENCH_INJECT") == "parity" and rank == world - 1:
        y[0] += 1.0  # test hook (tests/test_gpu_bench.py): a wrong y must fail the run
    stage("parity")
    hcsr = ref = sw_ms = None
    try:
        if args.multi:
            out["parity"] = distributed_parity(lib, args, world, rank, dev, y, st, held)
        else:  # N = 1: the whole matrix against spmv_gold (the CSR was kept for this)
            hcsr = host_csr(rp, col, val, x, y)
            del rp, col, val
            torch.cuda.empty_cache()
            out["parity"], ref, sw_ms = full_parity(hcsr)
    except Exception as e:
        out["parity"] = {"error": f"{type(e).__name__}: {str(e)[:300]}", "pass": False}
    if not out["parity"].get("pass"):
        fail_run("parity did not pass", out["parity"])

    # what follows adds reported-only fields, except that every result they report is verified
    # too (the library's RCCL forms, the drop-in's y): a mismatch fails the run (status 3). Each
    # runs under a try (an error is reported, never fatal), and a watchdog prints the line as it
    # stands and ends the process if they take longer than --extras-timeout seconds (a hung
    # collective on an 8-GPU node must not cost the measured, verified value)
    stage("extras")

    def on_timeout():
        emit(f"extras still running after {args.extras_timeout} s; line printed without them")
        sys.stdout.flush()
        _kill_children()
        os._exit(args.extras_timeout_status)

    watchdog = threading.Timer(args.extras_timeout, on_timeout)
    watchdog.daemon = True
    watchdog.start()
    t_extras = time.monotonic()

    def guarded(field, fn):
        try:
            out[field] = fn()
        except Exception as e:  # reported, never fatal to the bench line
            out[field] = {"error": f"{type(e).__name__}: {str(e)[:300]}"}

    def exchange_fields():
        cnt = [0.0] * world
        cnt[rank] = float(st["nr_rows"])
        counts = np.array(spmv_dist.sum_over_ranks(cnt, dev), dtype=np.int64)
        row_begin = int(counts[:rank].sum())
        n_total = int(counts.sum())
        res = {}
        for mode in ("gather", "reduce", "allgather"):
            def exchange():
                if mode == "gather":
                    return spmv_dist.exchange_gather(y, counts)
                if mode == "allgather":
                    return spmv_dist.exchange_allgather(y, counts)
                return spmv_dist.exchange_reduce(y, row_begin, n_total)

            for _ in range(2):  # warm the communicator
                exchange()
            torch.cuda.synchronize()
            barrier(world)
            reps = 5
            te0 = time.perf_counter()
            for _ in range(reps):
                exchange()
            torch.cuda.synchronize()
            barrier(world)
            res[f"{mode}_ms"] = round(spmv_dist.max_over_ranks((time.perf_counter() - te0) * 1e3 / reps, dev), 4)
        # x replication (done once per matrix; the bench generates x on every rank instead)
        xb = x.clone()
        spmv_dist.broadcast_x(xb)
        torch.cuda.synchronize()
        barrier(world)
        tb0 = time.perf_counter()
        for _ in range(3):
            spmv_dist.broadcast_x(xb)
        torch.cuda.synchronize()
        barrier(world)
        res["x_broadcast_ms"] = round(spmv_dist.max_over_ranks((time.perf_counter() - tb0) * 1e3 / 3, dev), 4)
        assert torch.equal(xb, x)  # every rank generates the same x
        del xb
        # a stream of SpMVs (right-hand sides, time steps): step k's gather runs on the
        # collective's stream while step k + 1 computes (spmv_dist.pipelined_gather, double-
        # buffered y). One SpMV's own gather cannot overlap its compute
        maxc = int(counts.max())
        bufs = [torch.zeros(maxc, dtype=y.dtype, device=dev) for _ in range(2)]
        nloc = int(st["nr_rows"])

        def step(k, yb):
            plan.run(x, yb[:nloc], stream)

        psteps = max(args.steps, 4)
        spmv_dist.pipelined_gather(step, bufs, counts, 2)  # warm
        torch.cuda.synchronize()
        barrier(world)
        tp0 = time.perf_counter()
        yp = spmv_dist.pipelined_gather(step, bufs, counts, psteps)
        torch.cuda.synchronize()
        barrier(world)
        res["pipelined_gather_ms_per_step"] = round(
            spmv_dist.max_over_ranks((time.perf_counter() - tp0) * 1e3 / psteps, dev), 4)
        res["pipelined_steps"] = psteps
        res["e2e_gflops_pipelined_gather"] = round(2.0 * nnz_all / (res["pipelined_gather_ms_per_step"] * 1e-3) / 1e9, 2)
        if rank == 0:  # the last step's gathered y against a plain gather of the same SpMV
            y_chk = spmv_dist.exchange_gather(bufs[(psteps - 1) % 2][:nloc], counts)
            res["pipelined_max_rel_diff"] = float(((yp.double() - y_chk.double()).abs().max()
                                                   / y_chk.double().abs().max().clamp_min(1e-300)).item())
        else:
            spmv_dist.exchange_gather(bufs[(psteps - 1) % 2][:nloc], counts)
        del bufs
        res["y_bytes"] = n_total * y.element_size()
        res["e2e_gflops_with_gather"] = round(2.0 * nnz_all / ((ms + res["gather_ms"]) * 1e-3) / 1e9, 2)
        res["e2e_gflops_with_reduce"] = round(2.0 * nnz_all / ((ms + res["reduce_ms"]) * 1e-3) / 1e9, 2)
        res["e2e_gflops_with_allgather"] = round(2.0 * nnz_all / ((ms + res["allgather_ms"]) * 1e-3) / 1e9, 2)
        res["backend"] = dist.get_backend()
        if world > torch.cuda.device_count():  # the single-GPU rehearsal: ranks share a device
            res["native"] = {"skipped": "ranks share one GPU; RCCL refuses two ranks on one device"}
        elif not args.no_native_exchange:
            try:
                res["native"] = native_exchange(lib, plan, x, st["nr_cols"], counts, world, rank, dev,
                                                held.get("y_full"))
            except Exception as e:  # reported, never fatal to the bench line
                res["native"] = {"error": str(e)[:300]}
        return res

    if args.multi and args.scaling == "strong" and args.workload == "powerlaw":
        # the dependent form x <- A x (square matrix): compute + all-gather in every step
        def dependent():
            res = dependent_iteration(plan, x, y, st, args.steps, world, rank, dev, held.get("y_full"),
                                      held.get("row_begin", 0))
            step_forms["dependent_ms_per_step"] = res["ms_per_step"]
            return res
        guarded("dependent", dependent)
        step_forms["dependent"] = out.pop("dependent")
    if args.multi:
        guarded("exchange", exchange_fields)
        nat = out["exchange"].get("native") if isinstance(out["exchange"], dict) else None
        if isinstance(nat, dict) and "allgather_graph_ms_per_step" in nat:
            # the same dependent form through the library's own RCCL clique, steps in one hipGraph
            step_forms["dependent_native_graph_ms_per_step"] = nat["allgather_graph_ms_per_step"]
        if isinstance(nat, dict) and nat.get("verified", {}).get("pass") is False:  # (same on every rank)
            fail_run("the library's RCCL exchange gave a wrong y", nat["verified"])
    held.pop("y_full", None)
    if args.multi and args.scaling == "weak" and args.workload == "powerlaw" and not args.no_strong_companion:
        guarded("strong_companion", lambda: strong_companion(lib, args, world, rank, dev, stream))
    if args.multi and args.scaling == "strong" and args.workload == "powerlaw" and not args.no_weak_companion:
        guarded("weak_companion", lambda: weak_companion(lib, args, world, rank, dev, stream))
    if hcsr is not None and not args.no_cpu:
        guarded("cpu_baseline", lambda: cpu_baseline(lib, hcsr, ref, args.cpu_reps, args.cpu_threads))
    hcsr = None
    # the drop-in boundary (create_csr_hw_matrix -> spmv_hw -> verification) in a child process:
    # N = 1 one unit, host merge (the reference's CU = 1 build); N > 1 (strong, the whole matrix)
    # rank 0 runs it with N units, one per GPU, merged by the library's RCCL reduce over xGMI --
    # the north star's mapping of accum_results -- while the other ranks wait on the store (no
    # GPU collective spinning on the GPUs the child uses)
    left = args.extras_timeout - (time.monotonic() - t_extras)
    child_timeout = max(30.0, min(240.0, left - 60.0))
    if not args.no_dropin and not args.slice_of and (not args.multi or args.scaling == "strong"):
        if not args.multi:
            guarded("dropin", lambda: run_dropin(args, 1, "host", ref, sw_ms, child_timeout))
        elif torch.cuda.device_count() < world:
            out["dropin"] = {"skipped": f"{world} units need {world} GPUs ({torch.cuda.device_count()} here)"}
        else:
            def both_merges():
                # the north star's RCCL reduce, then the library's default host merge (each GPU's
                # slice over its own PCIe link), each in its own child with the budget left
                red = run_dropin(args, world, "reduce", held["ref"], None, child_timeout)
                left2 = args.extras_timeout - (time.monotonic() - t_extras) - 60.0
                red["host_merge"] = (run_dropin(args, world, "host", held["ref"], None, min(240.0, left2))
                                     if left2 >= 30.0 else {"skipped": f"{left2 + 60:.0f} s of the extras budget left"})
                if red["host_merge"].get("pass") is False:
                    red["pass"] = False
                return red

            res, status = spmv_dist.rank0_only(both_merges, 2 * child_timeout + 60,
                                               passed=lambda r: r.get("pass") is not False)
            if rank == 0:
                out["dropin"] = res
            if status == "fail":
                fail_run("the drop-in boundary's y failed verification", res or "see rank 0")
            if status == "timeout":  # rank 0's line reports the drop-in; this rank only waited
                print(f"bench.py rank {rank}: no drop-in status from rank 0", file=sys.stderr, flush=True)
        if isinstance(out.get("dropin"), dict) and out["dropin"].get("pass") is False:
            fail_run("the drop-in boundary's y failed verification", out["dropin"])
    held.clear()
    ref = None
    if not args.multi and args.workload == "powerlaw" and args.dtype == "f64" and not args.no_side_configs:
        guarded("side_configs", lambda: {name: side_config(args, name, dev, stream) for name in ("config2", "config5")})
    # the end-to-end rate beside the compute-only value: one SpMV plus the
    # exchange that completes y, as the reference's "Total time" is hardware + accumulation
    # (csr_hw_wrapper.cpp:276-285)
    out["value_e2e"], out["value_e2e_form"] = value_e2e(out, ms, nnz_all)
    watchdog.cancel()
    emit()
    # the line is out and verified: a teardown that hangs (plan or process-group destruction) must
    # not hold the run (under torch.distributed.run no parent would end it before --run-timeout)
    teardown = threading.Timer(args.spawn_grace, lambda: os._exit(0))
    teardown.daemon = True
    teardown.start()
    plan.destroy()
    if dist.is_initialized():
        dist.destroy_process_group()
    if run_watchdog is not None:
        run_watchdog.cancel()


if __name__ == "__main__":
    main()
