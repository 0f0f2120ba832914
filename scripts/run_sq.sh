set -u
# SQ issue/wait breakdown + TA/TCP busy for the step kernels (PMC passes, kernel trace only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--steps 30 --warmup 5 --cpu-seconds 0 ${EXTRA:-}"
T=${TAG:-sq}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/${T}_a -o run --output-format csv -- python3 bench.py $A > gpurun_out/${T}_a.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${T}_b -o run --output-format csv -- python3 bench.py $A > gpurun_out/${T}_b.log 2>&1 || echo "pass b failed"
timeout -k 10 600 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/${T}_c -o run --output-format csv -- python3 bench.py $A > gpurun_out/${T}_c.log 2>&1 || echo "pass c failed"
echo ok
