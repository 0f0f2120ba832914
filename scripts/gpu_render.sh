#!/usr/bin/env bash
# GPU session for the renderer (config C5): render parity tests, the c5 bench, and a
# rocprofv3 kernel trace of the same bench command.  A test failure (rc 1) does not stop the
# session; any other failure ends it.
set -u
OUT=${OUT:-gpurun_out}
TAG=${TAG:-r01r}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log" | cut -c1-3000
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_render 600 python -u -m pytest tests/test_gpu_render.py -m gpu -x -v --timeout 300 --timeout-method thread
fi
step bench_c5 600 python bench.py --workload c5 --steps ${STEPS:-30} --warmup ${WARMUP:-3} ${EXTRA:-}
if [ -n "${TRACE:-}" ]; then
  step trace_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$TAG" -o run --output-format csv -- python3 bench.py --workload c5 --steps ${STEPS:-30} --warmup ${WARMUP:-3} --cpu-seconds 0
fi
echo "== all done"
