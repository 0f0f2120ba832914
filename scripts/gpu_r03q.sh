#!/usr/bin/env bash
# r03q: stamps of every k_run wave (option and idle) at steady state
set -u
OUT=gpurun_out
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
TAG=R NOBUILD=1 POLICY=uniform STEPS=3000 run stampsR2_uniform 300 python scripts/diag_stamps.py
TAG=R NOBUILD=1 POLICY=masked STEPS=1500 run stampsR2_masked 300 python scripts/diag_stamps.py
echo "== all done"
