#!/usr/bin/env bash
# r03g: sampled step timing (every 8th step, three events) vs every step; per-kernel roofline
set -u
OUT=gpurun_out
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
Q="--steps 100 --warmup 5 --cpu-seconds 0 --secondary-steps 0 --episode-envs 0"
run t1a 300 python bench.py $Q --timing-every 1
run t8a 300 python bench.py $Q --timing-every 8
run t1b 300 python bench.py $Q --timing-every 1
run t8b 300 python bench.py $Q --timing-every 8
run t0 300 python bench.py $Q --timing-every 1000
run bench 600 python bench.py --steps 30 --warmup 5
echo "== all done"
