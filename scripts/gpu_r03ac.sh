#!/usr/bin/env bash
# r03ac: k_regen draw codes from the top 27 bits (FAST): GPU suite, A/B against HEAD (rg1) and
# round-3 start (p1), bench
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
run pytest_gpu 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
V="p1=gym-treasure-game_amd/libtg_amd_p1.so,rg1=gym-treasure-game_amd/libtg_amd_rg1.so,fast=gym-treasure-game_amd/libtg_amd.so"
VARIANTS="$V" ROUNDS=3 STEPS=64 run ab_fast 900 python scripts/ab.py
run bench 600 python bench.py
echo "== all done"
