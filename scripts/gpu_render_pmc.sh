#!/usr/bin/env bash
# PMC passes over the render A/B driver (one variant): HBM bytes and L2 hit rate of k_render.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r01r}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export VARIANTS=${VARIANTS:-g16:} REPS=${REPS:-3} NOBUILD=1
run() {  # name, counters...
  local name=$1; shift
  echo "== $name"
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$OUT/pmc_${name}_$TAG" -o run --output-format csv -- python3 scripts/diag_render.py > "$OUT/pmc_${name}.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -n 2 "$OUT/pmc_${name}.log"
  [ $rc -eq 0 ] || exit $rc
}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$TAG" -o run --output-format csv -- python3 scripts/diag_render.py > "$OUT/trace_render.log" 2>&1 || exit $?
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum
echo "== all done"
