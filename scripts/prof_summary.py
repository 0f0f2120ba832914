#!/usr/bin/env python3
"""Summarise a gpu_profile.sh session into profiles/<tag>_summary.json (+ traffic_step_<policy>.json).

    python scripts/prof_summary.py --tag r01 [--out gpurun_out] [--envs 1048576]

Reads the rocprofv3 kernel-trace stats (same command as bench.py) and the separate PMC passes
(FETCH_SIZE, WRITE_SIZE, SQ_*).  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE /
WRITE_SIZE are in KiB.  FETCH_SIZE is calibrated per access pattern by scripts/calib/
calib_fetch.hip (profiles/r03/fetch_calibration.json): a coalesced stream (dword or 16-B lanes)
is reported at HALF its bytes; a scattered 8-B / 16-B load or 16-B LDS-DMA (one env per lane)
is reported as 64-66 B, one 64-B HBM read each; WRITE_SIZE is 1:1 for coalesced stores and 32 B
per scattered 8- or 16-B store (the write granule).  So each step kernel's HBM read bytes are
its coalesced reads (known from the step's counters: the bench line of the profiled run) plus
the rest of FETCH_SIZE at face value:
    hbm_read = coalesced + (FETCH_SIZE - coalesced / 2)
k_classify's reads are all coalesced (env-order loads); k_run's coalesced reads are the
worklist rows (44 B per valid env) and the twist sources (2,496 B + a 4-B list entry per
regenerated half of MT_HALF_GENS generations); its scattered reads are the code-window
LDS-DMA fills.  The k_errors factor
(the round-2 method, 2.0 for its coalesced 16-B reads) is kept beside it as a cross-check.
"""
import argparse
import csv
import json
import os
import re
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MT_HALF_GENS = 8  # tg_core.h: generations per half of an env's MT ring
REGEN_STEPS = 16  # tg_amd.hip: steps per k_regen launch


def short(name):
    m = re.search(r"(k_[a-z_]+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name.split("(")[0][:60]


def kernel_stats(path):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                                     "pct": float(r["Percentage"])}
    return out


def bench_line(path):
    """the JSON line bench.py printed in a profiled run's log (its steps / regeneration rate)"""
    if not os.path.exists(path):
        return None
    lines = [ln for ln in open(path) if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def last_of(k, last):
    """dispatches of kernel k in the timed region: the last `last` of a step kernel, the last
    last / REGEN_STEPS of k_regen (one launch per 16 steps; the profile runs 160 steps)"""
    if not last:
        return None
    return max(last // REGEN_STEPS, 1) if k.startswith("k_regen") else last


def counters(path, last=None):
    per = defaultdict(lambda: defaultdict(list))
    meta = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]),
                       "sgpr": int(r["SGPR_Count"]), "lds": int(r["LDS_Block_Size"])}
    # the timed steps are the last dispatches of each step kernel
    avg = {}
    for k, d in per.items():
        n = last_of(k, last)
        avg[k] = {c: sum(v[-n:] if n else v) / len(v[-n:] if n else v) for c, v in d.items()}
    return avg, meta


def timed_durations(path, last):
    """average duration (ns) of each kernel's timed dispatches in a kernel-trace CSV"""
    per = defaultdict(list)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        for r in csv.DictReader(f):
            per[short(r["Kernel_Name"])].append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for k, v in per.items():
        v.sort()
        n = last_of(k, last)
        sel = [d for _, d in (v[-n:] if n else v)]
        out[k] = {"timed_dispatches": len(sel), "avg_ns": sum(sel) / len(sel)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--policy", default="uniform")
    ap.add_argument("--mode", default="compact")
    ap.add_argument("--dest", default=os.path.join(ROOT, "profiles"),
                    help="where the summaries go (on a GPU box: under gpurun_out/, which is what "
                         "comes back)")
    ap.add_argument("--render", action="store_true",
                    help="the C5 passes (<tag>c5): k_render -> profiles/traffic_render.json")
    a = ap.parse_args()
    if a.render:
        return render_summary(a)
    res = {"tag": a.tag, "envs": a.envs, "policy": a.policy}
    ks = kernel_stats(os.path.join(a.out, "trace_" + a.tag, "run_kernel_stats.csv"))
    res["kernel_trace"] = ks
    pm = {}
    meta = {}
    prof_line = None
    for name in ("pmc_fetch_%s.log" % a.tag, "pmc_fetch_%s.log" % a.policy, "pmc_fetch.log"):
        prof_line = prof_line or bench_line(os.path.join(a.out, name))
    last = prof_line["steps"] if prof_line else None
    # the kernels' durations in the timed region of the trace run (same workload)
    td = timed_durations(os.path.join(a.out, "trace_" + a.tag, "run_kernel_trace.csv"), last)
    for k, v in td.items():
        if k in ks:
            ks[k]["timed_avg_ns"] = v["avg_ns"]
            ks[k]["timed_dispatches"] = v["timed_dispatches"]
    for p in ("fetch", "write", "sq1", "sq2", "regen_fetch", "regen_write", "regen_sq1", "regen_sq2"):
        path = os.path.join(a.out, "pmc_%s_%s" % (p, a.tag), "run_counter_collection.csv")
        if os.path.exists(path):
            avg, m = counters(path, last)
            meta.update(m)
            for k, d in avg.items():
                pm.setdefault(k, {}).update(d)
    res["pmc_avg_per_dispatch"] = pm
    res["dispatch_meta"] = meta
    # the step's kernels: k_classify + k_run (compact) or k_step (direct)
    names = (("k_classify", "k_run", "k_regen") if a.mode == "compact" else ("k_step",))
    # k_regen drains REGEN_STEPS steps' refill lists per launch: its per-step share
    spl = 16.0  # tg_amd.hip REGEN_STEPS: steps per k_regen launch at steady state
    step_k = [k for k in pm if k.split("<")[0] in names]
    if step_k and all("FETCH_SIZE" in pm[k] for k in step_k):
        known = 16.0 * a.envs  # k_errors: one 16-B uint4 per env, 16 B per lane
        raw_err = pm.get("k_errors", {}).get("FETCH_SIZE", 0.0) * 1024.0
        cal = known / raw_err if raw_err > 0 else None
        valid = (prof_line or {}).get("valid_step_frac", 0.0) * a.envs
        regens = (prof_line or {}).get("regens_per_step", 0.0)
        per = {}
        for k in step_k:
            fr = pm[k]["FETCH_SIZE"] * 1024.0
            wr = pm[k].get("WRITE_SIZE", 0.0) * 1024.0
            base = k.split("<")[0]
            if base == "k_classify":
                coal = 44.0 * a.envs
            elif base == "k_run":  # the worklist rows (no regeneration since r03aa: k_regen)
                coal = 44.0 * valid
            elif base == "k_regen":  # per launch: spl steps' halves, one source read each
                coal = (2500.0 + 8.0) / MT_HALF_GENS * regens * spl
            else:  # k_step: env-order state loads + the refills' sources
                coal = 44.0 * a.envs + 2496.0 / MT_HALF_GENS * regens
            scat = max(fr - coal / 2.0, 0.0)
            rd = coal + scat
            kn = ks.get(k, {}).get("timed_avg_ns") or ks.get(k, {}).get("avg_ns")
            cyc = pm[k].get("SQ_WAVE_CYCLES")
            ent = {"fetch_bytes_raw": fr, "coalesced_read_bytes": coal,
                   "scattered_read_bytes": scat, "read_bytes": rd, "write_bytes": wr,
                   "hbm_bytes": rd + wr, "fetch_bytes_kerrors_factor": fr * (cal or 1.0),
                   "avg_ns": kn}
            if base == "k_regen" and regens:
                # per MT generation regenerated (a full launch: REGEN_STEPS steps' lists)
                gens = regens * spl
                alg = (((prof_line or {}).get("roofline", {}).get("step", {}).get("kernels", {})
                        .get("regen", {})).get("alg_bytes_per_generation"))
                ent.update({"generations_per_launch": gens, "write_bytes_per_generation": wr / gens,
                            "read_bytes_per_generation": rd / gens,
                            "hbm_bytes_per_generation": (rd + wr) / gens,
                            "alg_bytes_per_generation": alg,
                            "ns_per_generation": kn / gens if kn else None})
            if kn:
                ent["hbm_gbs"] = (rd + wr) / kn
                v = pm[k].get("SQ_INSTS_VALU")
                # VALU issue utilisation: wave64 VALU instructions x 2 cycles (SIMD-32) over the
                # SIMD-cycles of the kernel's duration at the 2.4 GHz nominal clock
                ent["valu_util"] = v * 2.0 / (1024 * kn * 2.4) if v else None
            if cyc:
                ent["wait_frac"] = pm[k].get("SQ_WAIT_ANY", 0.0) / cyc
                ent["lds_bank_conflict_frac"] = (pm[k].get("SQ_LDS_BANK_CONFLICT", 0.0) /
                                                 max(pm[k].get("SQ_ACTIVE_INST_LDS", 1.0), 1.0))
            # what bounds the kernel, from the counters: HBM when its traffic runs at >= 60 %
            # of the 8 TB/s peak, VALU when issue is >= 60 % busy, else latency
            g, vu, wf = ent.get("hbm_gbs"), ent.get("valu_util"), ent.get("wait_frac")
            if g is not None and g >= 0.6 * 8000:
                ent["limiter"] = "hbm (%.0f GB/s)" % g
            elif vu is not None and vu >= 0.6:
                ent["limiter"] = "valu (issue %.0f %%)" % (100 * vu)
            elif g is not None:
                ent["limiter"] = ("latency: HBM %.0f GB/s (%.0f %% of peak), VALU issue %s, waves "
                                  "waiting %s of their cycles" %
                                  (g, g / 80.0, "%.0f %%" % (100 * vu) if vu is not None else "?",
                                   "%.0f %%" % (100 * wf) if wf is not None else "?"))
            per[k] = ent
        tot = sum(v["hbm_bytes"] / (spl if k.startswith("k_regen") else 1.0) for k, v in per.items())
        res["hbm"] = {"kernels": per, "hbm_bytes_per_launch": tot,
                      "calibration": "per access pattern (profiles/r03/fetch_calibration.json): "
                                     "coalesced reads reported at 1/2, scattered 8/16-B loads "
                                     "and LDS-DMA at one 64-B read each, writes 1:1",
                      "fetch_calibration_kerrors": cal,
                      "kerrors_note": ("k_errors reads %d B, FETCH_SIZE reported %.0f B" %
                                       (known, raw_err)) if raw_err else "k_errors not profiled"}
        ns = sum(ks[k]["avg_ns"] / (spl if k.startswith("k_regen") else 1.0)
                 for k in ks if k.split("<")[0] in names)
        res["step_kernels_avg_ns"] = ns
        # VALU issue utilisation of the step kernels: wave64 VALU instructions x 2 cycles
        # (SIMD-32) over the SIMD-cycles of their duration at the 2.4 GHz nominal clock
        valu = sum(pm[k].get("SQ_INSTS_VALU", 0.0) for k in step_k)
        valu_util = valu * 2.0 / (1024 * ns * 2.4) if valu and ns else None
        res["valu_util"] = valu_util
        tj = {"envs": a.envs, "policy": a.policy, "mode": a.mode,
              "kernels": {k: {f: v[f] for f in ("hbm_bytes", "read_bytes", "write_bytes",
                                                 "coalesced_read_bytes", "scattered_read_bytes",
                                                 "avg_ns", "hbm_gbs", "valu_util", "wait_frac",
                                                 "lds_bank_conflict_frac", "limiter")
                              if f in v} for k, v in per.items()},
              "hbm_bytes_per_launch": tot, "step_kernels_avg_ns": ns, "valu_util": valu_util,
              "regens_per_step": prof_line.get("regens_per_step") if prof_line else None,
              "burn_in": prof_line.get("burn_in") if prof_line else None,
              "source": "profiles/%s_summary.json (rocprofv3 --pmc passes of bench.py %s)"
                        % (a.tag, "steps=%s" % last)}
        os.makedirs(a.dest, exist_ok=True)
        with open(os.path.join(a.dest, "traffic_step_%s.json" % a.policy), "w") as f:
            json.dump(tj, f, indent=1)
    os.makedirs(a.dest, exist_ok=True)
    with open(os.path.join(a.dest, "%s_summary.json" % a.tag), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in res if k in ("hbm", "step_kernels_avg_ns")}, indent=1))


def render_summary(a):
    """k_render's HBM bytes per launch from the C5 passes (bench.py --workload c5)."""
    tag = a.tag + "c5"
    envs = a.envs if a.envs != 1 << 20 else 65536
    ks = kernel_stats(os.path.join(a.out, "trace_" + tag, "run_kernel_stats.csv"))
    pm = {}
    for p in ("fetch", "write"):
        path = os.path.join(a.out, "pmc_%s_%s" % (p, tag), "run_counter_collection.csv")
        avg, _ = counters(path)
        for k, d in avg.items():
            pm.setdefault(k, {}).update(d)
    known = 16.0 * envs  # k_errors (vec.errors() at the end of the bench): 16 B per env
    raw_err = pm["k_errors"]["FETCH_SIZE"] * 1024.0
    cal = known / raw_err if raw_err > 0 else 1.0
    fr = pm["k_render"]["FETCH_SIZE"] * 1024.0
    wr = pm["k_render"]["WRITE_SIZE"] * 1024.0
    res = {"tag": tag, "envs": envs, "kernel_trace": ks, "pmc_avg_per_dispatch": pm,
           "k_render": {"fetch_bytes_raw": fr, "fetch_bytes": fr * cal, "write_bytes": wr,
                        "frame_bytes_algorithmic": 1257984 * envs,
                        "avg_ns": ks["k_render"]["avg_ns"]},
           "fetch_calibration": cal}
    os.makedirs(a.dest, exist_ok=True)
    with open(os.path.join(a.dest, "%s_summary.json" % tag), "w") as f:
        json.dump(res, f, indent=1)
    tj = {"envs": envs, "kernel": "k_render", "hbm_bytes_per_launch": fr * cal + wr,
          "avg_ns": ks["k_render"]["avg_ns"], "source": "profiles/%s_summary.json" % tag}
    with open(os.path.join(a.dest, "traffic_render.json"), "w") as f:
        json.dump(tj, f, indent=1)
    print(json.dumps(res["k_render"], indent=1))


if __name__ == "__main__":
    main()
