#!/usr/bin/env bash
# GPU session (diagnostics): SQ counters of the step kernels for prebuilt variant libraries
# (LIBS="name:path ..."), each its own rocprofv3 --pmc pass over a short A/B harness run.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_ab
for nl in $LIBS; do
  name=${nl%%:*}; path=${nl#*:}
  VARIANTS="$name:compact:@$path" NOBUILD=1 ROUNDS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/pmc_ab/$name -o run --output-format csv -- python3 scripts/diag_ablation.py > gpurun_out/pmc_ab/$name.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc_ab/*/run_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]; k = "k_run" if "k_run" in k else "k_classify" if "k_classify" in k else ""
        if "k_run" in k or "k_classify" in k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(f.split("/")[-2], k, {c: "%.3g" % (sum(v) / len(v)) for c, v in sorted(d.items())})
PY
