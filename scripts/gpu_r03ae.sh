#!/usr/bin/env bash
# r03ae: the committed product build (k_regen one half at a time): GPU suite, smoke, bench,
# rocprofv3 kernel trace of the bench workload (both policies)
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
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
for pol in uniform masked; do
  if [ $pol = uniform ]; then B=3000; else B=1500; fi
  A="--policy $pol --steps 32 --warmup 5 --burn-in $B --cpu-seconds 0 --secondary-steps 0 --episode-envs 0"
  run trace_$pol 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_r03ae$pol -o run --output-format csv -- python3 bench.py $A
  rm -f $OUT/trace_r03ae$pol/run_kernel_trace.csv
done
echo "== all done"
