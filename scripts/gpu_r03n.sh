#!/usr/bin/env bash
# r03n: length-class worklists again, on the ring (the option loops now end k_run): parity, A/B
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
export TG_LIB_PATH=$GRAFT_REPO_ROOT/gym-treasure-game_amd/libtg_amd_cls.so
run pytest_cls 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu
unset TG_LIB_PATH
cp gym-treasure-game_amd/libtg_amd.so gym-treasure-game_amd/libtg_amd_p0.so
VARIANTS="p0=gym-treasure-game_amd/libtg_amd_p0.so,cls=gym-treasure-game_amd/libtg_amd_cls.so" ROUNDS=3 STEPS=50 run ab_cls 600 python scripts/ab.py
echo "== all done"
