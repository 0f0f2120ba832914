set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc_ic -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-seconds 0 > gpurun_out/pmc_ic.log 2>&1 || exit $?
echo ok
