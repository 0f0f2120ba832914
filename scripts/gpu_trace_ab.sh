#!/usr/bin/env bash
# GPU session (diagnostics): per-kernel times (rocprofv3 kernel trace) of prebuilt variant
# libraries (LIBS="name:path ..."), one A/B harness run each.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/trace_ab
for nl in $LIBS; do
  name=${nl%%:*}; path=${nl#*:}
  VARIANTS="$name:compact:@$path" NOBUILD=1 ROUNDS=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_ab/$name -o run --output-format csv -- python3 scripts/diag_ablation.py > gpurun_out/trace_ab/$name.log 2>&1 || exit $?
  python3 - "$name" <<'PY'
import csv, sys
n = sys.argv[1]
for r in csv.DictReader(open("gpurun_out/trace_ab/%s/run_kernel_stats.csv" % n)):
    if "k_run" in r["Name"] or "k_classify" in r["Name"]:
        print(n, r["Name"].split("(")[1][:40] if "(" in r["Name"] else r["Name"], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
