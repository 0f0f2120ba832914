#!/usr/bin/env bash
# r03d: decompose buckets / ladder walk / window size (A/B on one box)
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
VARIANTS="buckets=$L/libtg_amd.so,lad=$L/libtg_amd_lad.so,nb=$L/libtg_amd_nb.so,nblad=$L/libtg_amd_nblad.so,nbladw6=$L/libtg_amd_nbladw6.so,w6=$L/libtg_amd_w6.so,queue=$L/libtg_amd_stampsQ.so" POLICIES=uniform,masked STEPS=40 ROUNDS=2 run ab_r03d 900 python scripts/ab.py
echo "== all done"
