#!/usr/bin/env bash
# r03af: steps per k_regen launch: 8 / 16 (product) / 32, A/B
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
V="rs16=gym-treasure-game_amd/libtg_amd.so,rs8=gym-treasure-game_amd/libtg_amd_rs8.so,rs32=gym-treasure-game_amd/libtg_amd_rs32.so"
VARIANTS="$V" ROUNDS=3 STEPS=96 run ab_rs 900 python scripts/ab.py
echo "== all done"
