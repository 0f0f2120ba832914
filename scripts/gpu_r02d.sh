#!/usr/bin/env bash
# GPU session r02d: the A/B of the air-tick neighbourhood variants (prebuilt in-tree), then
# the full profile session (tests, bench, trace, PMC) and the actions-in-loop bench line.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NOBUILD=1 VARIANTS="prod:compact:,nocache:compact:-DTG_AIR_CACHE=0,nonbhd:compact:-DTG_AIR_NBHD=0" \
  timeout -k 10 400 python scripts/diag_ablation.py > gpurun_out/ab_air.txt 2>&1 || exit $?
cat gpurun_out/ab_air.txt
TAG=r02d bash scripts/gpu_profile.sh || exit $?
timeout -k 10 300 python bench.py --actions-in-loop --secondary-steps 0 --cpu-seconds 0 \
  > gpurun_out/bench_inloop.log 2>&1 || exit $?
tail -c 400 gpurun_out/bench_inloop.log
