#!/usr/bin/env bash
# r03c: buckets: GPU tests, A/B (r02 / queue / buckets), bench, stamps
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-800
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu
VARIANTS="r02=gym-treasure-game_amd/libtg_amd_r02.so,queue=gym-treasure-game_amd/libtg_amd_stampsQ.so,buckets=gym-treasure-game_amd/libtg_amd.so,w6=gym-treasure-game_amd/libtg_amd_w6.so" POLICIES=uniform,masked STEPS=40 ROUNDS=2 run ab_r03c 500 python scripts/ab.py
VARIANTS="r02=gym-treasure-game_amd/libtg_amd_r02.so,buckets=gym-treasure-game_amd/libtg_amd.so" POLICIES=uniform BURN=300 STEPS=40 ROUNDS=2 run ab_r03c_b300 300 python scripts/ab.py
run bench 600 python bench.py --steps 30 --warmup 5 --cpu-seconds 0
TAG=B NOBUILD=1 POLICY=masked STEPS=60 run stampsB_masked 200 python scripts/diag_stamps.py
TAG=B NOBUILD=1 POLICY=uniform STEPS=300 run stampsB_uniform 200 python scripts/diag_stamps.py
echo "== all done"
