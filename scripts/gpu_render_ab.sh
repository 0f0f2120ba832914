set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_render.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_render.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_render.log
if [ $rc -gt 1 ]; then exit $rc; fi
NOBUILD=1 timeout -k 10 400 python -u scripts/diag_render.py > gpurun_out/diag_render.log 2>&1 || exit $?
cat gpurun_out/diag_render.log
