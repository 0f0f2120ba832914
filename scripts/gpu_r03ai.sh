#!/usr/bin/env bash
# r03ai: per-wave k_run stamps of the final build (refills in k_regen): which waves end k_run
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
TAG=Z NOBUILD=1 POLICY=uniform STEPS=3000 run stampsZ_uniform 300 python scripts/diag_stamps.py
TAG=Z NOBUILD=1 POLICY=masked STEPS=1500 run stampsZ_masked 300 python scripts/diag_stamps.py
echo "== all done"
