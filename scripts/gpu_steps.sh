#!/usr/bin/env bash
# The one GPU-box runner (replaces round 3's per-session gpu_r03*.sh copies).
#
#   gpurun -- 'TAG=r04b POL=uniform bash scripts/gpu_steps.sh scripts/steps/<recipe>.txt'
#
# A recipe holds one step per line: "<name> <time limit s> <command ...>" ('#' lines and blank
# lines are skipped).  Each step runs under its own `timeout -k 10`, in `bash -c`, so the
# command sees the caller's environment (TAG, POL, ...) and OUT=gpurun_out; its output goes to
# $OUT/<name>.log, and the first failing step ends the run (no GPU step after a fault, an abort
# or a time limit).  Recipes: scripts/steps/README.
set -u
export OUT=gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ $# -eq 1 ] || { echo "usage: $0 RECIPE"; exit 2; }
while IFS= read -r line || [ -n "$line" ]; do
  case "$line" in ''|'#'*) continue ;; esac
  name=${line%% *}; rest=${line#* }
  lim=${rest%% *}; cmd=${rest#* }
  name=$(eval echo "$name")
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
done < "$1"
echo "== all done"
