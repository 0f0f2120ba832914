set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=base:compact:@gym-treasure-game_amd/libtg_amd_base.so,prod:compact:@gym-treasure-game_amd/libtg_amd.so ROUNDS=3 bash scripts/gpu_ab2.sh
