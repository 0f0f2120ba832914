#!/usr/bin/env bash
# r03b: the refill queue: GPU tests, bench, stamps
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu
run bench 600 python bench.py --steps 30 --warmup 5 --cpu-seconds 0
TAG=Q NOBUILD=1 POLICY=masked STEPS=60 run stampsQ_masked 200 python scripts/diag_stamps.py
TAG=Q NOBUILD=1 POLICY=uniform STEPS=300 run stampsQ_uniform 200 python scripts/diag_stamps.py
echo "== all done"
