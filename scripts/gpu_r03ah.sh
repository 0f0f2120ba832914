#!/usr/bin/env bash
# r03ah: k_regen takes list regions dynamically from per-XCD counters (16 at a time) instead
# of a fixed share per wave: GPU suite, A/B against the fixed shares (stat), bench
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
V="stat=gym-treasure-game_amd/libtg_amd_stat.so,dyn=gym-treasure-game_amd/libtg_amd.so"
VARIANTS="$V" ROUNDS=4 STEPS=96 run ab_dyn 900 python scripts/ab.py
run bench 600 python bench.py
echo "== all done"
