#!/usr/bin/env bash
# r03ak: k_run at 6 / 8 waves per SIMD (launch bounds) now that it holds no refills (masked:
# ~16k option waves in ~3 resident rounds at 5 waves/SIMD): A/B
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
V="base=gym-treasure-game_amd/libtg_amd.so,klb6=gym-treasure-game_amd/libtg_amd_klb6.so,klb8=gym-treasure-game_amd/libtg_amd_klb8.so"
VARIANTS="$V" ROUNDS=3 STEPS=96 run ab_klb 900 python scripts/ab.py
echo "== all done"
