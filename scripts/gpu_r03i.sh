#!/usr/bin/env bash
# r03i: ring of 4 + 4 generations (chained LDS twists): GPU tests, A/B vs the 2-generation build, bench
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
VARIANTS="gen2=gym-treasure-game_amd/libtg_amd_x4.so,ring=gym-treasure-game_amd/libtg_amd_ring.so" ROUNDS=3 STEPS=50 run ab_ring 600 python scripts/ab.py
run bench 600 python bench.py --steps 30 --warmup 5
echo "== all done"
