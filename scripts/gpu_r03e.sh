#!/usr/bin/env bash
# r03e: idle blocks interleaved with the option blocks (A/B), GPU tests of the product
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
L=gym-treasure-game_amd
VARIANTS="nb=$L/libtg_amd_nb.so,il4=$L/libtg_amd.so,il4nb=$L/libtg_amd_il4nb.so,il2nb=$L/libtg_amd_il2nb.so,il8nb=$L/libtg_amd_il8nb.so,queue=$L/libtg_amd_stampsQ.so" POLICIES=uniform,masked STEPS=40 ROUNDS=2 run ab_r03e 900 python scripts/ab.py
run pytest_gpu 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu
echo "== all done"
