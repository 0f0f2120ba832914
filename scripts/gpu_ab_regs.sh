set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_regs.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_regs.log
if [ $rc -gt 1 ]; then exit $rc; fi
NOBUILD=1 VARIANTS="prod:compact:,ring:compact:-DTG_RNG_REGS=0,prodd:direct:,ringd:direct:-DTG_RNG_REGS=0" timeout -k 10 600 python scripts/diag_ablation.py > gpurun_out/abl_regs.txt 2>&1 || exit $?
grep -E '"|kernel_ms' gpurun_out/abl_regs.txt
