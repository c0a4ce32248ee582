"""The bench contract on the GPU (bench.py is what the driver runs at N = 1 and N = 2/4/8):
small power-law matrices through `python bench.py` exactly as the driver calls it, checking the
JSON line's fields, its own parity, and -- for N = 2 -- the self-launch (no torchrun) with the
slices gathered on rank 0 and checked against the oracle (main.cpp:77-82 checks every result).
The two ranks share the box's one GPU over gloo (the rehearsal of the driver's SCALE runs); the
RCCL side of the same path runs as the one rank of an 'nccl' group (--dist-rehearsal): torch's
collectives on device tensors, the parity gather and the library's own clique."""
import json
import os
import signal
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SMALL = ["--rows", "400000", "--nnz", "6400000", "--steps", "3", "--warmup", "1", "--extras-timeout", "150"]


def _bench(*args, env=None, want_rc=0):
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    e.update(env or {})
    # its own process group: on a timeout the self-launched ranks go with the parent
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, *args], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True, env=e, cwd=ROOT, start_new_session=True)
    try:
        out, err = p.communicate(timeout=280)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        pytest.fail("bench.py timed out: " + err[-4000:])
    assert p.returncode == want_rc, out[-2000:] + err[-4000:]
    lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return lines[0]


def test_bench_one_gpu_line():
    d = _bench("--no-side-configs", "--no-xtiles", "--no-det", "--cpu-reps", "1")
    assert d["metric"] == "SpMV GFLOP/s + effective HBM GB/s (% roofline), fp64, 1/2/4/8 MI355X"
    assert d["n_gpus"] == 1 and d["n_ranks"] == 1 and d["steps"] == 3 and d["value"] > 0
    assert d["config"]["workload"] == "powerlaw" and d["config"]["nnz"] == 6_400_000
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] < 1.2 and r["kernel_ms"] > 0
    assert r["kernel_ms_per_rank"] == [r["kernel_ms"]]
    assert d["cpu_baseline"]["cores"] == 1 and d["cpu_baseline"]["kind"] == "port"
    assert d["parity"]["pass"] and d["parity"]["max_scaled_err"] <= 1e-12
    sf = d["step_forms"]  # value is the serial chain (each SpMV complete before the next)
    assert sf["value_form"] == "serial" and sf["serial_ms_per_step"] == d["ms_per_step"]
    assert d["graph"]["run_graph_ms_per_step"] > 0
    assert d["value_e2e"] == d["value"]  # one GPU: no exchange
    # the drop-in boundary: the reference's run.elf figures, verified
    di = d["dropin"]
    assert di["pass"] and di["units"] == 1 and di["merge"] == "host", di
    assert di["calls"] == 5 and di["verification"] == [0] * 5 and di["max_rel_diff_vs_spmv_gold"] <= 1e-12
    assert di["rows"] == 400_000 and di["nnz"] == 6_400_000
    for k in ("matrix_read_ms", "hardware_execution_ms", "result_accumulation_ms", "total_ms"):
        assert di[k] > 0, (k, di)
    assert abs(di["total_ms"] - di["hardware_execution_ms"] - di["result_accumulation_ms"]) < 1e-3
    assert di["software_execution_ms"] > 0 and di["storage_mb"] > 0
    assert len(di["unstreamed_total_ms"]["calls"]) == 5 and di["unstreamed_total_ms"]["median"] > 0


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_two_ranks_self_launched(scaling):
    d = _bench("--gpus", "2", "--scaling", scaling, "--no-weak-companion", "--no-strong-companion",
               "--no-native-exchange", env={"SPMV_BENCH_BACKEND": "gloo"})
    assert d["n_gpus"] == 2 and d["n_ranks"] == 2 and d["launcher"] == "bench.py" and d["scaling"] == scaling
    p = d["parity"]
    assert p["pass"] and p["max_scaled_err"] <= 1e-12 and p["ref_abs_1e-5_errors"] == 0
    assert p["rows_checked"] == (400_000 if scaling == "strong" else 800_000)
    assert len(d["roofline"]["kernel_ms_per_rank"]) == 2
    if scaling == "strong":
        assert d["config"]["slice_rows"][0] == 0
        assert d["exchange"]["backend"] == "gloo" and d["exchange"]["pipelined_max_rel_diff"] == 0.0
        sf = d["step_forms"]
        assert sf["value_form"] == "serial" and sf["serial_ms_per_step"] == d["ms_per_step"]
        assert sf["dependent"]["pass"] and sf["dependent_ms_per_step"] > 0, sf


def test_bench_parity_failure_fails_the_run():
    """at N > 1 parity is not an extra. A wrong y on the last rank (test hook
    SPMV_BENCH_INJECT=parity) prints the line with the failed parity and exits 3."""
    d = _bench("--gpus", "2", "--no-weak-companion", "--no-native-exchange",
               env={"SPMV_BENCH_BACKEND": "gloo", "SPMV_BENCH_INJECT": "parity"}, want_rc=3)
    assert d["n_ranks"] == 2 and d["parity"]["pass"] is False and d["parity"]["max_scaled_err"] > 1e-6


@pytest.mark.parametrize("scaling", ["strong", "weak"])
def test_bench_one_rank_rccl_rehearsal(scaling):
    d = _bench("--dist-rehearsal", "--scaling", scaling, "--no-weak-companion", "--no-strong-companion")
    assert d["dist_rehearsal"] and d["n_gpus"] == 1 and d["n_ranks"] == 1 and d["scaling"] == scaling
    p = d["parity"]
    assert p["pass"] and p["max_scaled_err"] <= 1e-12 and p["rows_checked"] == 400_000
    if scaling == "strong":
        assert d["config"]["slice_rows"] == [0, 400_000]
        ex = d["exchange"]
        assert ex["backend"] == "nccl" and ex["pipelined_max_rel_diff"] == 0.0, ex
        assert all(ex[k] > 0 for k in ("gather_ms", "reduce_ms", "allgather_ms", "x_broadcast_ms"))
        nat = ex["native"]
        assert "error" not in nat, nat
        assert nat["rccl_comm_count"] == 1 and nat["gather_max_rel_diff_vs_torch"] <= 1e-12  # two SpMVs (LDS adds)
        v = nat["verified"]  # every form of the library's exchange is checked
        assert v["pass"] and v["gather"] and v["reduce"] and v["allgather"], v
        assert v["max_rel_diff"]["torch_allgather_vs_parity_gather"] <= 1e-12
        # the north star's literal mapping at world 1: spmv_hw with one unit, RCCL reduce merge
        di = d["dropin"]
        assert di["pass"] and di["units"] == 1 and di["merge"] == "reduce", di
        hm = di["host_merge"]  # then the library's default merge (each GPU's slice over PCIe)
        assert hm["pass"] and hm["merge"] == "host" and hm["units"] == 1 and hm["verification"] == [0] * hm["calls"], hm
        e2e = d["value_e2e_form"]
        assert d["value_e2e"] < d["value"] and e2e["exchange_ms"] == nat["reduce_exchange_ms"], e2e
        assert all(nat[k] > 0 for k in ("gather_compute_ms", "reduce_exchange_ms", "allgather_graph_ms_per_step"))
        sf = d["step_forms"]
        assert sf["dependent"]["pass"] and sf["dependent_ms_per_step"] > 0
        assert sf["dependent_native_graph_ms_per_step"] == nat["allgather_graph_ms_per_step"]


def test_bench_rccl_rehearsal_of_a_split_slice():
    """--dist-rehearsal --slice-of 4: the one RCCL rank holds rank 0's slice of a 4-way cut of a
    4M-row / 64M-nnz power-law matrix (~1M rows: a split sweep plan, like an 8-GPU rank's slice
    of the 10M/160M matrix), so the line carries all three step forms over 'nccl': the serial
    chain (value, a torch graph captured with the process group up), the behind form of
    spmv_plan_run_graph and the dependent form, with parity on the slice's rows and the
    dependent step checked against it."""
    d = _bench("--dist-rehearsal", "--slice-of", "4", "--no-weak-companion", "--rows", "4000000",
               "--nnz", "64000000")
    assert d["slice_of"] == 4 and d["n_ranks"] == 1 and d["exchange"]["backend"] == "nccl"
    r0, r1 = d["config"]["slice_rows"]
    assert r0 == 0 and 900_000 < r1 < 1_100_000
    p = d["parity"]
    assert p["pass"] and p["rows_checked"] == r1 - r0
    sf = d["step_forms"]
    assert sf["value_form"] == "serial" and sf["serial_ms_per_step"] == d["ms_per_step"]
    assert d["graph"]["run_graph_form"] == "behind" and sf["behind_ms_per_step"] > 0
    assert sf["dependent"]["pass"] and sf["dependent_ms_per_step"] > 0
    nat = d["exchange"]["native"]
    assert "error" not in nat and nat["gather_compute_ms"] > 0, nat


def test_bench_hung_rank_ends_at_the_run_timeout():
    """VERDICT r4 item 1 on the GPU: rank 1 never reaches the timed region's barrier (test hook
    SPMV_BENCH_INJECT=hang), so rank 0 waits in the collective. The self-launch parent kills both
    at --run-timeout, prints one error line naming each rank's stage ("timed") and exits 124."""
    e = {k: v for k, v in os.environ.items()
         if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    e.update(SPMV_BENCH_BACKEND="gloo", SPMV_BENCH_INJECT="hang")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL, "--gpus", "2", "--run-timeout", "40"],
                       capture_output=True, text=True, env=e, cwd=ROOT, timeout=110)
    assert p.returncode == 124, p.stdout[-2000:] + p.stderr[-3000:]
    (line,) = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert line["value"] is None and "run timeout" in line["error"]
    assert line["stage"] == {"0": "timed", "1": "timed"}, line


def test_bench_one_gpu_parity_failure_fails_the_run():
    """at N = 1 the full-size parity check is part of the measurement. A wrong
    y (SPMV_BENCH_INJECT=parity) gives an invalid line -- value null, the measured number kept as
    value_unverified -- and exit status 3, before any extra runs."""
    d = _bench("--no-side-configs", "--no-xtiles", "--no-det", "--cpu-reps", "1",
               env={"SPMV_BENCH_INJECT": "parity"}, want_rc=3)
    assert d["parity"]["pass"] is False and d["value"] is None and d["valid"] is False
    assert d["value_unverified"] > 0 and d["cpu_baseline"] is None and "dropin" not in d


def test_bench_one_gpu_extras_timeout_keeps_the_verified_parity():
    """An N = 1 run whose extras outlast --extras-timeout prints the line from the watchdog (exit
    --extras-timeout-status, 0 by default) and still carries the passed full-size parity."""
    d = _bench("--no-xtiles", "--no-det", "--extras-timeout", "0.5", "--cpu-reps", "50")
    assert d["extras_timeout"] and d["parity"]["pass"] and d["value"] > 0
    assert d["parity"]["rows_checked"] == 400_000


def test_bench_failed_dropin_verification_fails_the_run():
    """A drop-in call whose verification is not 0 (test hook SPMV_BENCH_INJECT=dropin) is a
    result the line would report wrong: status 3, value null."""
    d = _bench("--no-side-configs", "--no-xtiles", "--no-det", "--cpu-reps", "1", "--dropin-reps", "1",
               env={"SPMV_BENCH_INJECT": "dropin"}, want_rc=3)
    assert d["dropin"]["pass"] is False and d["value"] is None and d["parity"]["pass"]


@pytest.mark.parametrize("form", ["reduce", "allgather"])
def test_bench_wrong_library_exchange_fails_the_run(form):
    """the library's RCCL reduce (rank 0's y) and all-gather (every rank's
    next x) are verified, not only timed. A wrong result (SPMV_BENCH_INJECT=reduce / allgather)
    fails the run with status 3 and names the form."""
    d = _bench("--dist-rehearsal", "--scaling", "strong", "--no-weak-companion", "--no-dropin",
               env={"SPMV_BENCH_INJECT": form}, want_rc=3)
    v = d["exchange"]["native"]["verified"]
    assert v["pass"] is False and v[form] is False and d["value"] is None, v
    assert all(v[k] for k in ("gather", "reduce", "allgather") if k != form)


def test_bench_one_gpu_fp32_line():
    """--dtype f32 (config 5's precision): the mandatory parity gates on the scaled error (1e-4);
    the reference's absolute 1e-5 count is reported, not gated, in fp32 (it is below fp32
    rounding of |y| ~ 1e2), and the drop-in run passes on its normwise difference."""
    d = _bench("--dtype", "f32", "--no-xtiles", "--no-det", "--cpu-reps", "1", "--dropin-reps", "2")
    assert d["dtype"] == "f32" and d["value"] > 0 and d["parity"]["pass"], d["parity"]
    assert d["parity"]["max_scaled_err"] <= 1e-4 and "ref_abs_1e-5_errors" in d["parity"]
    assert d["dropin"]["pass"] and d["dropin"]["calls"] == 2, d["dropin"]
