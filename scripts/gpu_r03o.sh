#!/usr/bin/env bash
# r03o: DIAGNOSTIC lower bound: k_run without its refill queue (results not exact) vs the product; one refill region per grab
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
cp gym-treasure-game_amd/libtg_amd.so gym-treasure-game_amd/libtg_amd_p0.so
VARIANTS="p0=gym-treasure-game_amd/libtg_amd_p0.so,noq=gym-treasure-game_amd/libtg_amd_noq.so,grab1=gym-treasure-game_amd/libtg_amd_grab1.so" ROUNDS=2 STEPS=50 run ab_noq 600 python scripts/ab.py
echo "== all done"
