#!/usr/bin/env bash
# r03w: instruction-cache counters of the step kernels (k_run's code is ~80 KB, the SQC
# instruction cache 64 KB per CU pair): available counters, then one PMC pass on the bench's
# workload after its burn-in (uniform policy)
set -u
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stop ($name rc=$rc)"; exit $rc; fi
}
run list 120 rocprofv3 -L
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_0-9]*\|SQ_INSTS_[A-Z_0-9]*\|SQ_WAIT_INST[A-Z_0-9]*" $OUT/list.log | sort -u > $OUT/icache_counters.txt
cat $OUT/icache_counters.txt | tr '\n' ' '; echo
B=3000
A="--policy uniform --steps 20 --warmup 5 --burn-in $B --cpu-seconds 0 --secondary-steps 0 --episode-envs 0 --progress"
K="--kernel-include-regex k_classify|k_run --kernel-iteration-range [$((B - 20))-$((B + 40))]"
run pmc_icache 300 rocprofv3 $K --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $OUT/pmc_icache -o run --output-format csv -- python3 bench.py $A
run pmc_ifetch 300 rocprofv3 $K --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU -d $OUT/pmc_ifetch -o run --output-format csv -- python3 bench.py $A
echo "== all done"
