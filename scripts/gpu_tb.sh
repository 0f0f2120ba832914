#!/usr/bin/env bash
# GPU session: the gpu tests, then the bench (BENCH_ARGS).  A test failure (rc 1) does not stop
# the session; any other failure ends it.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 4 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:-}
fi
step bench 600 python bench.py ${BENCH_ARGS:---steps 100 --warmup 10}
echo "== all done"
