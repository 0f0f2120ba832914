#!/usr/bin/env bash
# bench.py's episode drain interval (--gather-every) A/B at N = 1, both policies.
set -eu
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
for g in 1 10; do
  for pol in uniform masked; do
    timeout -k 10 240 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --policy $pol \
      --gather-every $g > "$OUT/gather_${g}_${pol}.log" 2>&1
    python - "$OUT/gather_${g}_${pol}.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "episodes", d["episodes"],
      "gathered", d["episodes_gathered"], "kernel_ms %.4f" % d["roofline"]["kernel_ms"])
PY
  done
done
