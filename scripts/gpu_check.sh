#!/usr/bin/env bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; an ordinary test failure (exit 1) does not stop the
# session, but a fault / abort / segfault / timeout (any other non-zero code) ends it.
set -u
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name, timeout, command...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 600 python bench.py --steps ${STEPS:-100} --warmup ${WARMUP:-10}
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0
echo "== all done"
