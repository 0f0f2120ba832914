#!/usr/bin/env bash
# Quick GPU session: gpu tests + bench in each mode (+ optional trace). rc 1 (test failure)
# does not stop the session; any other failure ends it.
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
  tail -n 4 "$OUT/$name.log" | cut -c1-1500
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then step pytest_gpu 900 python -m pytest tests -m gpu -q -x; fi
for m in ${MODES:-compact direct}; do
  step bench_$m 600 python bench.py --mode $m --steps ${STEPS:-100} --warmup ${WARMUP:-10} --cpu-seconds 0 ${EXTRA:-}
done
if [ -n "${TRACE:-}" ]; then
  step trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$TRACE" -o run --output-format csv -- python3 bench.py --steps ${STEPS:-100} --warmup ${WARMUP:-10} --cpu-seconds 0
fi
echo "== all done"
