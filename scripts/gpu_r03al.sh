#!/usr/bin/env bash
# r03al: end-of-session check of the tree as committed (fresh build): GPU suite, smoke, bench
set -u
OUT=gpurun_out
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 600 python bench.py
echo "== all done"
