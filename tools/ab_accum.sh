mkdir -p gpurun_out/r01k
for r in 1000000 10000000; do
 for pf in 1 0 1 0; do
  echo "== rows=$r prefault=$pf" >> gpurun_out/r01k/accum_ab.log
  SPMV_HW_PREFAULT=$pf timeout -k 10 200 python tools/part1_accum.py --rows $r --calls 5 >> gpurun_out/r01k/accum_ab.log 2>&1 || exit 1
 done
done
