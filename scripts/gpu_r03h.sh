#!/usr/bin/env bash
# r03h: code window by dword LDS-DMA (conflict-free LDS reads) vs dwordx4: parity, A/B, LDS counters
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
export TG_LIB_PATH=$GRAFT_REPO_ROOT/gym-treasure-game_amd/libtg_amd_dw.so
run pytest_dw 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_rollout.py -m gpu
unset TG_LIB_PATH
VARIANTS="x4=gym-treasure-game_amd/libtg_amd_x4.so,dw=gym-treasure-game_amd/libtg_amd_dw.so" ROUNDS=3 STEPS=50 run ab_dw 600 python scripts/ab.py
A="--steps 20 --warmup 5 --burn-in 300 --cpu-seconds 0 --secondary-steps 0 --episode-envs 0"
for v in x4 dw; do
  export TG_LIB_PATH=$GRAFT_REPO_ROOT/gym-treasure-game_amd/libtg_amd_$v.so
  for pol in uniform masked; do
    run lds_${v}_$pol 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD -d $OUT/lds_${v}_$pol -o run --output-format csv -- python3 bench.py --policy $pol $A
  done
done
echo "== all done"
