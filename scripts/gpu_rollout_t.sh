#!/usr/bin/env bash
# GPU session: the async rollout's parity tests, then its A/B timing against the per-step path.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ro_t.log 2>&1; rc=$?
tail -15 gpurun_out/ro_t.log
[ $rc -eq 0 ] || exit $rc
[ "${AB:-1}" = 1 ] || exit 0
timeout -k 10 300 python -u scripts/ro_ab.py ${RO_ARGS:-} > gpurun_out/ro_ab.log 2>&1; rc=$?
tail -60 gpurun_out/ro_ab.log
exit $rc
