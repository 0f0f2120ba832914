#!/usr/bin/env bash
# GPU session: bench.py lines for several argument sets (BENCH_ARGS="args1|args2|...").
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bench_ab
IFS='|' read -ra SETS <<< "${BENCH_ARGS:-}"
i=0
for a in "${SETS[@]}"; do
  timeout -k 10 300 python -u bench.py $a --secondary-steps 0 --cpu-seconds 0 > gpurun_out/bench_ab/b$i.log 2>&1 || exit $?
  python3 - "$i" "$a" <<'PY'
import json, sys
i, a = sys.argv[1], sys.argv[2]
line = [l for l in open("gpurun_out/bench_ab/b%s.log" % i) if l.startswith("{")][0]
d = json.loads(line)
print(a, "->", "%.4e" % d["value"], "ms/step %.4f" % d["ms_per_step"], "kernel_ms", d["roofline"].get("kernel_ms"))
PY
  i=$((i+1))
done
