#!/usr/bin/env bash
# r03ad: k_regen without the software pipeline (52 VGPRs: 8 waves/SIMD instead of 6), and k_run
# workgroups with no listed chunk returning right after the prologue: GPU suite on each, A/B
# against HEAD (pipe)
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
TG_LIB_PATH=$PWD/gym-treasure-game_amd/libtg_amd_nopipe.so run pytest_nopipe 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
TG_LIB_PATH=$PWD/gym-treasure-game_amd/libtg_amd_idleexit.so run pytest_idleexit 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
V="pipe=gym-treasure-game_amd/libtg_amd.so,nopipe=gym-treasure-game_amd/libtg_amd_nopipe.so,idleexit=gym-treasure-game_amd/libtg_amd_idleexit.so"
VARIANTS="$V" ROUNDS=3 STEPS=64 run ab_nopipe 900 python scripts/ab.py
echo "== all done"
