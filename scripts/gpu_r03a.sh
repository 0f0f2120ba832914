#!/usr/bin/env bash
# r03a: GPU tests (new + full), bench, per-wave stamps (baseline build vs the batched walk), and
# the FETCH/WRITE calibration kernels.
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
run pytest_new 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c4.py "tests/test_gpu_parity.py::test_dropin_shares_the_global_random_stream" "tests/test_gpu_parity.py::test_dropin_with_seed_leaves_the_global_stream_alone" "tests/test_gpu_parity.py::test_reference_levels" "tests/test_gpu_rollout.py" -k "cascade or c4 or episodes or dropin or far_shard"
run pytest_gpu 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu
run bench 600 python bench.py --steps 30 --warmup 5 --cpu-seconds 0
NOBUILD=1 POLICY=masked STEPS=60 run stamps_masked 200 python scripts/diag_stamps.py
NOBUILD=1 POLICY=uniform STEPS=300 run stamps_uniform 200 python scripts/diag_stamps.py
TAG=W NOBUILD=1 POLICY=masked STEPS=60 run stampsW_masked 200 python scripts/diag_stamps.py
TAG=W NOBUILD=1 POLICY=uniform STEPS=300 run stampsW_uniform 200 python scripts/diag_stamps.py
run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib_fetch -o run --output-format csv -- ./scripts/calib/calib_fetch
run calib_write 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/calib_write -o run --output-format csv -- ./scripts/calib/calib_fetch
echo "== all done"
