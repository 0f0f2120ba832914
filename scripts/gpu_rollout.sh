#!/usr/bin/env bash
# GPU session: the rollout parity test, then the bench per-step vs tg_rollout K = 1 / 10.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_rollout 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "rollout or checkpoint"
for k in 0 1 10; do
  step bench_roll$k 600 python bench.py --steps 100 --warmup 10 --cpu-seconds 0 --rollout $k
done
echo "== all done"
