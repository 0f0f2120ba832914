#!/usr/bin/env bash
# r03z: k_run occupancy: launch bounds for 6 / 7 / 8 waves per SIMD (80 / 72 / 64 VGPRs, spills
# 4 / 39 / 90) against HEAD's 5 (84 VGPRs): more resident waves for the refill queue while
# the option loops run
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
V="p1=gym-treasure-game_amd/libtg_amd_p1.so,lb6=gym-treasure-game_amd/libtg_amd_lb6.so"
V="$V,lb7=gym-treasure-game_amd/libtg_amd_lb7.so,lb8=gym-treasure-game_amd/libtg_amd_lb8.so"
VARIANTS="$V" ROUNDS=3 STEPS=50 run ab_lb 900 python scripts/ab.py
echo "== all done"
