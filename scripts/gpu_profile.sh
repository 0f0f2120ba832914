#!/usr/bin/env bash
# GPU session: tests, bench, rocprofv3 kernel trace of the SAME bench command, PMC passes.
# A test failure (rc 1) does not stop the session; any other failure ends it.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r02}
BENCH_ARGS=${BENCH_ARGS:---steps 100 --warmup 10}
PROF_ARGS=${PROF_ARGS:---steps 30 --warmup 5 --cpu-seconds 0 --secondary-steps 0}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
fi
step bench 600 python bench.py $BENCH_ARGS
step trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$TAG" -o run --output-format csv -- python3 bench.py $PROF_ARGS
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_$TAG" -o run --output-format csv -- python3 bench.py $PROF_ARGS
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_$TAG" -o run --output-format csv -- python3 bench.py $PROF_ARGS
step pmc_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/pmc_sq1_$TAG" -o run --output-format csv -- python3 bench.py $PROF_ARGS
step pmc_sq2 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/pmc_sq2_$TAG" -o run --output-format csv -- python3 bench.py $PROF_ARGS
if [ "${C5:-0}" = 1 ]; then  # config C5: the same passes over the render workload
  C5_ARGS="--workload c5 --steps 10 --warmup 2 --cpu-seconds 0"
  step bench_c5 600 python bench.py --workload c5 --steps 30 --warmup 3
  step trace_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_${TAG}c5" -o run --output-format csv -- python3 bench.py $C5_ARGS
  step pmc_fetch_c5 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_${TAG}c5" -o run --output-format csv -- python3 bench.py $C5_ARGS
  step pmc_write_c5 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_${TAG}c5" -o run --output-format csv -- python3 bench.py $C5_ARGS
fi
echo "== all done"
