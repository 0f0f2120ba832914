#!/usr/bin/env bash
# GPU session (diagnostics): LDS / VALU / wait counters of the step kernels (A/B harness run).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_lds
P1="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  VARIANTS="prod:compact:@gym-treasure-game_amd/libtg_amd.so" NOBUILD=1 ROUNDS=1 WARMUP=${WARMUP:-300} timeout -s KILL 180 rocprofv3 --pmc $P -d gpurun_out/pmc_lds/p$i -o run --output-format csv -- python3 scripts/diag_ablation.py > gpurun_out/pmc_lds/p$i.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob("gpurun_out/pmc_lds/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]; k = "k_run" if "k_run" in k else "k_classify" if "k_classify" in k else ""
        if k:
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: "%.4g" % (sum(v[-60:]) / len(v[-60:])) for c, v in sorted(d.items())})
PY
