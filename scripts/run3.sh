set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/diag_ablation.py > gpurun_out/ablation.log 2>&1 || exit $?
cat gpurun_out/ablation.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/trace.log 2>&1 || exit $?
tail -1 gpurun_out/trace.log | cut -c1-600
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_sq1_c3 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0 > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq2_c3 -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0 > gpurun_out/pmc2.log 2>&1 || exit $?
echo pmc done
