#!/usr/bin/env bash
# r03m: per-wave stamps of the ring build at steady state; queue issue priority A/B
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
TAG=R NOBUILD=1 POLICY=uniform STEPS=3000 run stampsR_uniform 300 python scripts/diag_stamps.py
TAG=R NOBUILD=1 POLICY=masked STEPS=1500 run stampsR_masked 300 python scripts/diag_stamps.py
cp gym-treasure-game_amd/libtg_amd.so gym-treasure-game_amd/libtg_amd_p0.so
VARIANTS="p0=gym-treasure-game_amd/libtg_amd_p0.so,qprio2=gym-treasure-game_amd/libtg_amd_qprio2.so" ROUNDS=3 STEPS=50 run ab_qprio 600 python scripts/ab.py
echo "== all done"
