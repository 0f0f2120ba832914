#!/usr/bin/env bash
# GPU session: parity tests of the product build, then step-time A/B of ring variants.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_stage.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_stage.log
if [ $rc -ne 0 ]; then exit $rc; fi
NOBUILD=1 VARIANTS="$VARIANTS" timeout -k 10 600 python scripts/diag_ablation.py > gpurun_out/abl_stage.txt 2>&1 || exit $?
grep -E '"|kernel_ms' gpurun_out/abl_stage.txt
