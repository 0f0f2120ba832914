#!/usr/bin/env bash
# r03u: episode start step (no S.ep store for reward-None envs): GPU suite, A/B against the
# pruned build without it (p0), bench
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
VARIANTS="p0=gym-treasure-game_amd/libtg_amd_p0.so,epstart=gym-treasure-game_amd/libtg_amd.so" ROUNDS=3 STEPS=50 run ab_epstart 600 python scripts/ab.py
run bench 600 python bench.py
echo "== all done"
