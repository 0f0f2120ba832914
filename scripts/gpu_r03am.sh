#!/usr/bin/env bash
# r03am: 24 steps per k_regen launch against 16 (A/B)
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
V="rs16=gym-treasure-game_amd/libtg_amd.so,rs24=gym-treasure-game_amd/libtg_amd_rs24.so"
VARIANTS="$V" ROUNDS=4 STEPS=96 run ab_rs24 900 python scripts/ab.py
echo "== all done"
