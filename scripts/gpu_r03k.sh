#!/usr/bin/env bash
# r03k: the product with the 8 + 8 generation ring: GPU tests, bench, rocprofv3 kernel trace + PMC passes
# for both policies (separate counter passes, as MI355X_MICROARCH.md prescribes)
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu
run bench 600 python bench.py --steps 30 --warmup 5
for pol in uniform masked; do
  if [ $pol = uniform ]; then B=3000; else B=1500; fi
  A="--policy $pol --steps 20 --warmup 5 --burn-in $B --cpu-seconds 0 --secondary-steps 0 --episode-envs 0"
  T=r03k$pol
  run trace_$pol 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_fetch_$pol 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_write_$pol 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_sq1_$pol 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_sq1_$T -o run --output-format csv -- python3 bench.py $A
  run pmc_sq2_$pol 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_sq2_$T -o run --output-format csv -- python3 bench.py $A
done
echo "== all done"
