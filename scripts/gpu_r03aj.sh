#!/usr/bin/env bash
# r03aj: the four-tick SWAR plain go walk re-measured now that k_run ends with its option waves
# (refills in k_regen): A/B, GPU suite on it
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
V="base=gym-treasure-game_amd/libtg_amd.so,swar2=gym-treasure-game_amd/libtg_amd_swar2.so"
VARIANTS="$V" ROUNDS=4 STEPS=96 run ab_swar2 900 python scripts/ab.py
TG_LIB_PATH=$PWD/gym-treasure-game_amd/libtg_amd_swar2.so run pytest_swar2 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
echo "== all done"
