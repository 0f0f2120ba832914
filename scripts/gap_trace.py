#!/usr/bin/env python3
"""Where the time between a timed region's kernels goes, from a rocprofv3
kernel trace + HIP runtime trace of one bench run:

    rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d DIR -- \\
        python3 bench.py --gpus 1 --steps 20 --warmup 5 --secondary-steps 0 --cpu-seconds 0
    python scripts/gap_trace.py DIR STEPS

The timed region is found as the bench lays it out: its STEPS k_classify / k_run pairs (plus the
k_regen and episode-drain launches among them and the final tg_regenerate), immediately before
the first k_null of the bench's region probe.  Per kernel boundary it reports:
  gap      = next kernel's trace start - this kernel's trace end (GPU idle between the two: the
             packet processor's barrier, cache actions and dispatch of the next kernel)
  host lag = next kernel's trace start - the end of its hipLaunchKernel call (> 0: the launch
             was queued before the GPU reached it, the host is not on the path; < 0 would mean
             the GPU waited for the host)
and per kernel the trace duration (dispatch to completion; the bench's in-kernel spans cover
first wave start to last wave end).  Diagnostic, not the product."""
import csv
import glob
import os
import sys
from collections import defaultdict

import numpy as np


def load(pattern):
    paths = glob.glob(pattern, recursive=True)
    if not paths:
        return []
    with open(paths[0]) as f:
        return list(csv.DictReader(f))


def short(name):
    for k in ("k_classify", "k_run", "k_regen", "k_drain_episodes", "k_null", "k_step", "k_flow",
              "k_actions", "k_errors", "k_flow_check"):
        if k + "<" in name or k + "(" in name or name.endswith(k) or (k + "I") in name or k in name:
            return k
    return name[:40]


def main(d, steps):
    kt = load(os.path.join(d, "**", "*kernel_trace.csv"))
    api = load(os.path.join(d, "**", "*hip_api_trace.csv"))
    call_end = {}
    for r in api:
        if "Launch" in r["Function"]:
            call_end[r["Correlation_Id"]] = int(r["End_Timestamp"])
    ks = sorted(({"name": short(r["Kernel_Name"]), "s": int(r["Start_Timestamp"]),
                  "e": int(r["End_Timestamp"]), "corr": r["Correlation_Id"]} for r in kt),
                key=lambda k: k["s"])
    first_null = next(i for i, k in enumerate(ks) if k["name"] == "k_null")
    # the region ends with the final tg_regenerate's k_regen (the timing records' flush and the
    # probe follow it)
    while ks[first_null - 1]["name"] not in ("k_regen", "k_run", "k_flow", "k_flow_check"):
        first_null -= 1
    i, seen = first_null - 1, 0
    while i >= 0 and seen < steps:
        if ks[i]["name"] == "k_classify":
            seen += 1
        i -= 1
    reg = ks[i + 1:first_null]
    print("%s: timed region of %d steps: %d kernels, %.1f us from the first start to the last end"
          % (d, steps, len(reg), (reg[-1]["e"] - reg[0]["s"]) / 1e3))
    dur = defaultdict(list)
    gaps = defaultdict(list)
    lag = []
    for a, b in zip(reg, reg[1:]):
        gaps[(a["name"], b["name"])].append((b["s"] - a["e"]) / 1e3)
        if b["corr"] in call_end:
            lag.append((b["s"] - call_end[b["corr"]]) / 1e3)
    for k in reg:
        dur[k["name"]].append((k["e"] - k["s"]) / 1e3)
    tot_gap = sum(sum(v) for v in gaps.values())
    print("  kernels (trace duration, us):")
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print("    %-18s %4d launches  mean %8.2f  total %9.1f" % (name, len(v), np.mean(v), sum(v)))
    print("  boundaries (GPU idle between consecutive kernels, us):")
    for key, v in sorted(gaps.items(), key=lambda kv: -sum(kv[1])):
        print("    %-18s -> %-18s %4d  mean %6.2f  min %6.2f  max %6.2f  total %8.1f"
              % (key[0], key[1], len(v), np.mean(v), min(v), max(v), sum(v)))
    print("  all gaps: %.1f us = %.2f us per step" % (tot_gap, tot_gap / steps))
    if lag:
        lag = np.array(lag)
        print("  host lag (GPU start - end of the launch call): min %.1f p10 %.1f median %.1f us;"
              " launches the GPU reached before the host issued them: %d of %d"
              % (lag.min(), np.percentile(lag, 10), np.median(lag), int((lag < 0).sum()), len(lag)))
    # the region's ends on the host: the bench records ev0, launches the steps, records ev1,
    # polls ev1 (hipEventQuery) and synchronises
    k0, kz = reg[0], reg[-1]
    recs = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in api
                  if r["Function"] in ("hipEventRecord", "hipEventQuery", "hipDeviceSynchronize",
                                       "hipStreamSynchronize") or r["Correlation_Id"] == k0["corr"])
    c0 = [r for r in api if r["Correlation_Id"] == k0["corr"]]
    if c0:
        l0s, l0e = int(c0[0]["Start_Timestamp"]), int(c0[0]["End_Timestamp"])
        ev0 = max((r for r in recs if r[2] == "hipEventRecord" and r[0] < l0s), default=None)
        ev1 = min((r for r in recs if r[2] == "hipEventRecord" and r[0] > l0s), default=None)
        sync = min((r for r in recs if r[2] in ("hipDeviceSynchronize", "hipStreamSynchronize")
                    and ev1 and r[0] > ev1[0]), default=None)
        if ev0:
            print("  host, region start: ev0 recorded -> first launch call %.1f us; the call %.1f us;"
                  " its return -> the kernel's GPU start %.1f us"
                  % ((l0s - ev0[1]) / 1e3, (l0e - l0s) / 1e3, (k0["s"] - l0e) / 1e3))
        if ev1 and sync:
            polls = [r for r in recs if r[2] == "hipEventQuery" and ev1[0] < r[0] < sync[0]]
            print("  host, region end: last kernel's end -> the synchronise's return %.1f us (%d event"
                  " polls; ev1 recorded %.1f us before the last kernel's end)"
                  % ((sync[1] - kz["e"]) / 1e3, len(polls), (kz["e"] - ev1[1]) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
