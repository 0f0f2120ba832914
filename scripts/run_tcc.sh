set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--steps 30 --warmup 5 --cpu-seconds 0"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tcc_f -o run --output-format csv -- python3 bench.py $A > /dev/null 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tcc_w -o run --output-format csv -- python3 bench.py $A > /dev/null 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum -d gpurun_out/tcc_h -o run --output-format csv -- python3 bench.py $A > /dev/null 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_REQ_sum GRBM_GUI_ACTIVE -d gpurun_out/tcc_x -o run --output-format csv -- python3 bench.py $A > /dev/null 2>&1 || exit $?
echo ok
