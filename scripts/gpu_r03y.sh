#!/usr/bin/env bash
# r03y: the plain go walk takes a whole code dword at once when all four ticks are plain
# (SWAR sums): GPU suite on that build, A/B against HEAD (p1)
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
TG_LIB_PATH=$PWD/gym-treasure-game_amd/libtg_amd_swar.so run pytest_gpu 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
VARIANTS="p1=gym-treasure-game_amd/libtg_amd_p1.so,swar=gym-treasure-game_amd/libtg_amd_swar.so" ROUNDS=4 STEPS=50 run ab_swar 600 python scripts/ab.py
echo "== all done"
