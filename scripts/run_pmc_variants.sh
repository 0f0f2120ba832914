set -u
# TA/TD/SQ counters for diagnostic variant builds (scripts/diag_ablation.py VARIANTS syntax)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export VARIANTS=${VARIANTS:-"r4:compact:,norng:compact:-DTG_DIAG_NORNG"}
BUILD_ONLY=1 timeout -k 10 600 python scripts/diag_ablation.py || exit $?
for v in $(echo "$VARIANTS" | tr ',' '\n' | cut -d: -f1); do
  for pass in "${PASSES:-TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE}"; do :; done
  ONLY=$v NOBUILD=1 ROUNDS=1 timeout -k 10 600 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE -d gpurun_out/pv_$v -o run --output-format csv -- python3 scripts/diag_ablation.py > gpurun_out/pv_$v.log 2>&1 || exit $?
  ONLY=$v NOBUILD=1 ROUNDS=1 timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_VALU -d gpurun_out/pq_$v -o run --output-format csv -- python3 scripts/diag_ablation.py > gpurun_out/pq_$v.log 2>&1 || exit $?
done
echo ok
