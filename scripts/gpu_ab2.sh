#!/usr/bin/env bash
# GPU session: step-time A/B of prebuilt variant libraries (diagnostics; VARIANTS as in
# scripts/diag_ablation.py, e.g. "old:compact:@gym-treasure-game_amd/libtg_amd_old.so,...").
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NOBUILD=1 VARIANTS="$VARIANTS" ROUNDS=${ROUNDS:-2} timeout -k 10 600 python scripts/diag_ablation.py > gpurun_out/abl.txt 2>&1 || exit $?
cat gpurun_out/abl.txt | tail -40
