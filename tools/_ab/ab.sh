#!/usr/bin/env bash
# A/B of two builds of libspmv_hw_f64.so on one box (the headline bench line, interleaved).
# libspmv_hw_f64_old.so (not tracked) is the product library built from another commit's sources:
#   git archive <commit> spmv-fpga_amd include | tar -x -C /tmp/old && make -C /tmp/old/spmv-fpga_amd all
#   cp /tmp/old/spmv-fpga_amd/lib/libspmv_hw_f64.so tools/_ab/libspmv_hw_f64_old.so
# (./tools/_ab is in .gpurunignore: drop that line to send the copies to the box again)
set -u
OUT=gpurun_out/${1:-r06u}; mkdir -p "$OUT"
cp spmv-fpga_amd/lib/libspmv_hw_f64.so tools/_ab/libspmv_hw_f64_new.so
for i in 1 2 3 4; do
  for v in old new; do
    cp tools/_ab/libspmv_hw_f64_$v.so spmv-fpga_amd/lib/libspmv_hw_f64.so
    timeout -k 10 150 python bench.py --no-cpu --no-dropin --no-side-configs --no-xtiles --steps 50 > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open('$OUT/$v$i.json').read().strip().splitlines()[-1]); print('$v', $i, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
cp tools/_ab/libspmv_hw_f64_new.so spmv-fpga_amd/lib/libspmv_hw_f64.so
