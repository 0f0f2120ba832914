set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/diag_ablation.py > gpurun_out/ablation.log 2>&1 || exit $?
cat gpurun_out/ablation.log
timeout -k 10 300 python scripts/diag_stamps.py > gpurun_out/stamps.log 2>&1 || exit $?
head -8 gpurun_out/stamps.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c2 -o run --output-format csv -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/trace.log 2>&1 || exit $?
echo trace ok
