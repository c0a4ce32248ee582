"""bench.py --gpus N without a launcher: the parent starts N ranks itself
before any GPU call, with the environment torch.distributed.run would give them, relays rank 0's
JSON line and exits with the workers' worst status. --dry-launch makes every rank print its launch
environment and exit before touching the GPU, so the plumbing runs here on the CPU."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(*extra, env=None, timeout=120):
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *extra], capture_output=True, text=True, timeout=timeout, env=e)


def _lines(text):
    return [json.loads(ln) for ln in text.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("n", [2, 3, 8])
def test_self_launch_gives_every_rank_its_environment(n):
    p = _run("--gpus", str(n), "--dry-launch")
    assert p.returncode == 0, p.stderr
    out = _lines(p.stdout)
    assert len(out) == 1 and out[0]["RANK"] == "0"  # only rank 0's line on stdout
    ranks = out + _lines(p.stderr)
    assert sorted(int(r["RANK"]) for r in ranks) == list(range(n))
    for r in ranks:
        assert r["LOCAL_RANK"] == r["RANK"] and r["WORLD_SIZE"] == str(n) and r["LOCAL_WORLD_SIZE"] == str(n)
        assert r["MASTER_ADDR"] == "127.0.0.1" and r["MASTER_PORT"] == ranks[0]["MASTER_PORT"]
        assert r["SPMV_BENCH_LAUNCHER"] == "bench.py" and r["gpus"] == n
    assert len({r["pid"] for r in ranks}) == n  # one process per rank


@pytest.mark.parametrize("codes,want", [("2:3", 3), ("1:7,2:3", 7), ("1:-9", 137), ("0:4", 4)])
def test_self_launch_exits_with_the_worst_status(codes, want):
    p = _run("--gpus", "3", "--dry-launch", "--dry-launch-rc", codes)
    assert p.returncode == want, (p.returncode, p.stderr)


def test_self_launch_stops_a_hung_rank_after_another_failed():
    """A rank that fails leaves the others possibly waiting in a collective: after --spawn-grace
    seconds the parent kills them (status 128 + 9)."""
    p = _run("--gpus", "3", "--dry-launch", "--dry-launch-rc", "1:hang,2:5", "--spawn-grace", "1", timeout=60)
    assert p.returncode == 137, (p.returncode, p.stderr)


def test_self_launch_all_ranks_hung_end_at_the_run_timeout():
    """every rank stuck (e.g. in one collective) -- no rank ever exits. The
    parent's --run-timeout kills them all, prints one JSON error line naming each rank's last
    stage, and exits 124, well before the driver's own limit."""
    p = _run("--gpus", "3", "--dry-launch", "--dry-launch-rc", "0:hang,1:hang,2:hang", "--run-timeout", "3",
             timeout=60)
    assert p.returncode == 124, (p.returncode, p.stderr)
    (line,) = [ln for ln in _lines(p.stdout) if "error" in ln]  # (rank 0's dry-launch line aside)
    assert line["value"] is None and "run timeout" in line["error"] and line["rc"] == 124
    assert line["stage"] == {"0": "timed", "1": "timed", "2": "timed"}, line


def test_self_launch_rank0_done_others_hung():
    """rank 0 finished (its line printed, status 0) but a peer never exits: after
    --spawn-grace the parent kills it and fails; rank 0's line stays the only stdout line."""
    p = _run("--gpus", "3", "--dry-launch", "--dry-launch-rc", "2:hang", "--spawn-grace", "1", timeout=60)
    assert p.returncode == 137, (p.returncode, p.stderr)
    (line,) = _lines(p.stdout)
    assert line["RANK"] == "0" and "dry_launch" in line
    assert "killed as hung" in p.stderr


def test_self_launch_teardown_hang_after_the_line_is_not_a_failure():
    """A rank that finished (past its line, parity included) but hangs in teardown is killed after
    --spawn-grace; the run keeps status 0, since the measurement is complete."""
    p = _run("--gpus", "3", "--dry-launch", "--dry-launch-rc", "1:teardown-hang", "--spawn-grace", "1", timeout=60)
    assert p.returncode == 0, (p.returncode, p.stderr)
    assert "teardown hang" in p.stderr
    p = _run("--gpus", "3", "--dry-launch", "--dry-launch-rc", "1:teardown-hang,2:hang", "--spawn-grace", "1",
             timeout=60)
    assert p.returncode == 137, (p.returncode, p.stderr)  # rank 2 never finished


def test_self_launch_failed_rank0_gets_an_error_line():
    """Rank 0 failed before printing its line: the parent prints the error line (stages, statuses)."""
    p = _run("--gpus", "2", "--dry-launch", "--dry-launch-rc", "0:5", timeout=60)
    assert p.returncode == 5, (p.returncode, p.stderr)
    lines = _lines(p.stdout)
    err = [ln for ln in lines if "error" in ln]
    assert len(err) == 1 and err[0]["value"] is None and err[0]["stage"]["0"] == "init", lines


def test_under_a_launcher_the_rank_has_its_own_deadline():
    """torch.distributed.run starts the ranks (no bench.py parent): each rank's own --run-timeout
    ends a hang with status 124, rank 0 printing the error line."""
    p = _run("--gpus", "2", "--dry-launch", "--dry-launch-rc", "0:hang", "--run-timeout", "2",
             env={"RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1",
                  "MASTER_PORT": "29999"}, timeout=60)
    assert p.returncode == 124, (p.returncode, p.stderr)
    lines = _lines(p.stdout)
    assert lines[-1]["value"] is None and lines[-1]["stage"] == {"0": "timed"}, lines


def test_under_a_launcher_no_second_spawn():
    """With WORLD_SIZE set (torch.distributed.run), bench.py is one rank and starts nothing."""
    p = _run("--gpus", "2", "--dry-launch",
             env={"RANK": "1", "LOCAL_RANK": "1", "WORLD_SIZE": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29999"})
    assert p.returncode == 0, p.stderr
    (line,) = _lines(p.stdout)
    assert line["RANK"] == "1" and line["SPMV_BENCH_LAUNCHER"] is None


def test_one_gpu_runs_in_process():
    p = _run("--dry-launch")
    assert p.returncode == 0, p.stderr
    (line,) = _lines(p.stdout)
    assert line["gpus"] == 1 and line["WORLD_SIZE"] is None


def test_dist_rehearsal_is_one_gpu_only():
    """--dist-rehearsal runs the N > 1 path as one rank of an RCCL group (tests/test_gpu_bench.py);
    it is refused with --gpus > 1, where the real process group takes its place."""
    p = _run("--gpus", "2", "--dist-rehearsal", "--dry-launch")
    assert p.returncode == 2 and "one-GPU form" in p.stderr, p.stderr
    p = _run("--dist-rehearsal", "--dry-launch")
    assert p.returncode == 0, p.stderr


def test_slice_of_needs_the_rehearsal_and_the_strong_cut():
    """--slice-of N is the one-rank RCCL rehearsal of an N-GPU rank's slice: refused without
    --dist-rehearsal and with --scaling weak (argparse status 2); accepted with both."""
    p = _run("--slice-of", "8", "--dry-launch")
    assert p.returncode == 2 and "--dist-rehearsal" in p.stderr
    p = _run("--dist-rehearsal", "--slice-of", "8", "--scaling", "weak", "--dry-launch")
    assert p.returncode == 2 and "strong-scaling cut" in p.stderr
    p = _run("--dist-rehearsal", "--slice-of", "8", "--dry-launch")
    assert p.returncode == 0, p.stderr


@pytest.mark.parametrize("extra,multi", [((), False), (("--gpus", "8"), True), (("--dist-rehearsal",), True)])
def test_default_deadlines_fit_the_driver_limit(extra, multi):
    """the run's own deadline (and the self-launch parent's kill after it) ends
    before the driver's 600 s limit, so a hung run still prints its stage line; a collective gives
    up long before the run deadline; the extras watchdog fires before it even when the extras
    start late (N = 1 by half the deadline, N > 1 by 5/8 of it)."""
    p = _run(*extra, "--dry-launch")
    assert p.returncode == 0, p.stderr
    d = _lines(p.stdout)[0]["deadlines"]
    limit = _lines(p.stdout)[0]["driver_limit_s"]
    assert limit == 600
    assert d["run_timeout"] <= 480 and d["run_timeout"] + d["spawn_grace"] < limit
    assert d["collective_timeout"] <= d["run_timeout"] / 4
    frac = 0.625 if multi else 0.5
    assert d["extras_timeout"] + frac * d["run_timeout"] <= d["run_timeout"]
    # explicit deadlines derive the others
    p = _run(*extra, "--dry-launch", "--run-timeout", "200")
    d = _lines(p.stdout)[0]["deadlines"]
    assert d["run_timeout"] == 200 and d["collective_timeout"] == 50 and d["extras_timeout"] == (75 if multi else 100)


def test_self_launch_rank0_alone_after_the_others_finished_is_not_hung():
    """ranks 1 and 2 finished cleanly ("done", status 0) while rank 0 still works after
    the last collective (the drop-in child, the CPU baseline): it is not killed at --spawn-grace,
    only the run deadline bounds it (here: killed at --run-timeout, status 124)."""
    p = _run("--gpus", "3", "--dry-launch", "--dry-launch-rc", "0:hang", "--spawn-grace", "1", "--run-timeout", "6",
             timeout=60)
    assert p.returncode == 124, (p.returncode, p.stderr)
    assert "run timeout" in p.stderr
