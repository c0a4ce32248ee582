#!/usr/bin/env bash
# One gpurun session: each GPU step under its own time limit; stop at the first step that
# faults, aborts, segfaults or times out (exit 124/134/137/139), keep going after plain test
# failures so the bench and profile still run. Usage: tools/gpu_session.sh <tag> [steps...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
STEPS=${*:-"tests smoke bench prof"}
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  # heartbeat: a step that prints nothing for minutes (a bench before its one line) still shows life
  ( while sleep 30; do date +%T >> "$OUT/heartbeat"; done ) & local hb=$!
  local t0=$(date +%s%N)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  local wall=$(( ($(date +%s%N) - t0) / 1000000 ))
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "== $name rc=$rc wall_ms=$wall" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL step $name rc=$rc; stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    tests_sel) run pytest_sel 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -rf -x --timeout 120 --timeout-method thread ;;
    selflaunch) SPMV_BENCH_BACKEND=gloo run selflaunch_strong 600 python bench.py --gpus 2 --steps 5 --warmup 2 ;;
    selflaunch4) SPMV_BENCH_BACKEND=gloo run selflaunch4_strong 900 python bench.py --gpus 4 --steps 5 --warmup 2 --no-weak-companion ;;
    selflaunch8) SPMV_BENCH_BACKEND=gloo run selflaunch8_strong 1000 python bench.py --gpus 8 ${SCALE_ARGS:-} ;;
    selflaunch_weak) SPMV_BENCH_BACKEND=gloo run selflaunch_weak 600 python bench.py --gpus 2 --steps 5 --warmup 2 --scaling weak ;;
    abmirror) run abmirror 900 python tools/ab_variants.py --workload powerlaw --dtype f32 --rounds ${AB_ROUNDS:-7} --reps 10 \
                --variants binned#1:0,binned#1:7,binned#2:0,binned#2:7,binned#3:0,binned#3:7,binned#4:0,binned#4:7 ;;
    absteal) run absteal 900 python tools/strong_slices.py --ns ${STEAL_NS:-4,8} --slices all --variants ${STEAL_VARIANTS:-28,36,37,38} --rounds ${AB_ROUNDS:-5} --reps 20 ;;
    abgraph) run abgraph 900 python tools/strong_slices.py --ns ${GRAPH_NS:-4,8} --slices all --graph-ab ${GRAPH_K:-20} --graph-modes ${GRAPH_MODES:-product,dag,serial} --rounds ${AB_ROUNDS:-5} ;;
    tests_all) run pytest_gpu 1000 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    bench32) run bench_f32 600 python bench.py --dtype f32 --no-cpu ;;
    banded) run bench_banded 300 python bench.py --workload banded ;;
    prof) run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --no-cpu --no-dropin --steps 20 ;;
    calib) [ -x tools/hbm_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/hbm_calib.hip -o tools/hbm_calib
           run calib 300 tools/hbm_calib ;;
    strong) run strong 600 python tools/strong_slices.py ${STRONG_ARGS:-} ;;
    profstrong) run rocprof_strong 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_strong" -o run -- python tools/strong_slices.py ${STRONG_ARGS:---ns 4,8} ;;
    skew) run skew 600 python tools/skew_probe.py ${SKEW_ARGS:-} ;;
    e2e) run reader 600 python tools/bench_reader.py --dir /tmp --threads 1,8,16
         run run_elf_16m 600 ./tests/run_elf/run.elf /tmp/reader_1000000_16000000.mtx --fast-reader ;;
    tracegraph) run trace_graph 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_graph" -o run -- python tools/strong_slices.py --ns 8 --slices ends --graph-ab 20 --graph-modes ${GRAPH_MODES:-product,dag,serial} --rounds 1 ;;
    wgcons) run wgcons 600 python tools/wg_timeline.py --slices ${WG_SLICES:-0/8,7/8,0/4,0/1} --consistency ${WG_K:-20} ;;
    abbias) for i in $(seq 1 ${AB_ITERS:-3}); do
              SPMV_SWEEP_XCC_BIAS=0 run abbias0_$i 400 python tools/strong_slices.py --ns 8,4 --slices all --graph-ab 20 --graph-modes product --rounds 3 --tag xcc_bias_0
              SPMV_SWEEP_XCC_BIAS=0.02 run abbiasd_$i 400 python tools/strong_slices.py --ns 8,4 --slices all --graph-ab 20 --graph-modes product --rounds 3 --tag xcc_bias_0.02
            done ;;
    rccl1) run rccl1_strong 600 python bench.py --dist-rehearsal --scaling strong --no-weak-companion ;;
    rccl1s8) run rccl1_slice8 600 python bench.py --dist-rehearsal --slice-of 8 --no-weak-companion ;;
    rehearse) SPMV_BENCH_BACKEND=gloo run rehearse_weak 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --scaling weak
              SPMV_BENCH_BACKEND=gloo run rehearse_strong 600 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --scaling strong ;;
    ab) run ab 600 python tools/ab_variants.py ;;
    absweep) run absweep 600 python tools/ab_variants.py ${AB_ARGS:---workload powerlaw --variants sweep:20,sweep:28,sweep:30 --rounds 5} ;;
    counters) run counters 120 rocprofv3 -L ;;
    pmc) for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
           tagc=$(echo $c | tr ' ' '_')
           run pmc_$tagc 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$tagc" -o run -- python tools/ab_variants.py --workload powerlaw --variants sweep:3,sweep:11 --rounds 1 --reps 3
         done ;;
    pmcw) for wl in powerlaw banded; do for dt in f64 f32; do for c in FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum; do
           run pmc_${wl}_${dt}_$c 600 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${wl}_${dt}_$c" -o run -- python bench.py --workload $wl --dtype $dt --no-cpu --no-dropin --no-xtiles --no-side-configs --steps 5 --warmup 1
         done; done; done
         python tools/pmc_traffic.py "$OUT" --out "$OUT/traffic.json" > /dev/null ;;
    pmcw64) for wl in powerlaw banded; do for c in FETCH_SIZE WRITE_SIZE TCC_HIT_sum TCC_MISS_sum; do
           run pmc_${wl}_f64_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${wl}_f64_$c" -o run -- python bench.py --workload $wl --dtype f64 --no-cpu --no-dropin --no-xtiles --no-side-configs --no-det --steps 5 --warmup 1
         done; done
         python tools/pmc_traffic.py "$OUT" --out "$OUT/traffic.json" > /dev/null ;;
    pmcbin) for c in FETCH_SIZE WRITE_SIZE; do
           run pmcbin_f32_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmcbin_f32_$c" -o run -- python bench.py --dtype f32 --no-cpu --no-dropin --no-xtiles --no-side-configs --no-det --steps 5 --warmup 1
         done
         python tools/pmc_binned.py "$OUT" --out "$OUT/binned_pmc.json" --session "$(basename $OUT)" ;;
    pmcx) i=0; for c in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM" \
                    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_BUSY_avr" \
                    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD"; do
           i=$((i+1)); run pmcx_$i 240 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmcx_$i" -o run -- python tools/ab_variants.py --workload powerlaw ${PMCX_ARGS:-} --variants ${PMCX_VARIANTS:-sweep:28} --rounds 1 --reps 3
         done ;;
    pmc_calib) for c in FETCH_SIZE WRITE_SIZE; do
           run pmccal_$c 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmccal_$c" -o run -- tools/hbm_calib
         done ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "session done" | tee -a "$OUT/session.log"
