#!/usr/bin/env bash
# r03t: the round-3 final product: bench, rocprofv3 kernel trace + PMC passes
# for both policies (separate counter passes), summarised on the box (the counter CSVs of the
# burn-in's dispatches are too large to bring back), then the CSVs are removed
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
run bench 600 python bench.py
for pol in uniform masked; do
  if [ $pol = uniform ]; then B=3000; else B=1500; fi
  A="--policy $pol --steps 20 --warmup 5 --burn-in $B --cpu-seconds 0 --secondary-steps 0 --episode-envs 0 --progress"
  # counters for the step kernels' dispatches around the timed steps only (the burn-in's
  # thousands of serialised counter dispatches are slow and their CSVs too large)
  K="--kernel-include-regex k_classify|k_run --kernel-iteration-range [$((B - 20))-$((B + 40))]"
  T=${TAGP:-r03t}$pol
  run trace_$pol 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_fetch_$pol 300 rocprofv3 $K --pmc FETCH_SIZE -d $OUT/pmc_fetch_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_write_$pol 300 rocprofv3 $K --pmc WRITE_SIZE -d $OUT/pmc_write_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_sq1_$pol 300 rocprofv3 $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_sq1_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_sq2_$pol 300 rocprofv3 $K --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_sq2_$T -o run --output-format csv -- python3 bench.py $A
  # k_regen runs once per 16 steps: its own dispatch range
  R="--kernel-include-regex k_regen --kernel-iteration-range [$((B / 16 - 2))-$((B / 16 + 6))]"
  run pmc_regen_fetch_$pol 300 rocprofv3 $R --pmc FETCH_SIZE -d $OUT/pmc_regen_fetch_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_regen_write_$pol 300 rocprofv3 $R --pmc WRITE_SIZE -d $OUT/pmc_regen_write_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_regen_sq1_$pol 300 rocprofv3 $R --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_regen_sq1_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_regen_sq2_$pol 300 rocprofv3 $R --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_regen_sq2_$T -o run --output-format csv -- python3 bench.py $A
  run summary_$pol 120 python scripts/prof_summary.py --tag $T --policy $pol --dest $OUT/summ
  rm -rf $OUT/pmc_*_$T
  rm -f $OUT/trace_$T/run_kernel_trace.csv.gz; gzip -f $OUT/trace_$T/run_kernel_trace.csv
done
du -sh $OUT
echo "== all done"
