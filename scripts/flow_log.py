#!/usr/bin/env python3
"""Reads a TG_FLOW_DBG build's k_flow event log (TG_FLOW_LOG=<prefix>: <prefix>.<launch>.bin) and
reports the first protocol anomaly in clock order: a chunk classified twice for one step, an
env run twice for one step, a chunk's outstanding count out of step.  Diagnostic, not the product.

Records (8 x u32): type, a, b, c, d, wave, clock lo, clock hi
  1 classify start (c, t, path, x)    2 classify end (c, t, cnt, x)
  3 run lane (item, env, old outst, lane | mcnt << 8 | x << 16)
  4 push (item, slot, src, x)         5 ticket served: run starts (h, item, x)
  7 run end (item, chunks readied, entries, x)   8 ticket taken (h, x)
  9 wave exits (x)                    10 wave starts its loop (x)
(type 3 only in TG_FLOW_LANES builds).  --time: where the waves' time goes (clock: 100 MHz)."""
import sys
from collections import defaultdict

import numpy as np


def item_s(it):
    return "t%d k%d j%d" % (it >> 28, (it >> 24) & 15, it & 0xFFFFFF)


def main(path):
    raw = np.fromfile(path, dtype=np.uint32)
    hdr, ev = raw[:8], raw[8:].reshape(-1, 8)
    cnt, C, P, K = (int(v) for v in hdr[:4])
    print("%s: %d events, C %d P %d K %d" % (path, cnt, C, P, K))
    clk = ev[:, 6].astype(np.int64) | (ev[:, 7].astype(np.int64) << 32)
    order = np.argsort(clk, kind="stable")
    ev, clk = ev[order], clk[order] - clk.min()
    cls = defaultdict(list)   # (c, t) -> [(clock, path, wave)]
    runs = defaultdict(list)  # (env, t) -> [(clock, item, old, wave)]
    outst = {}                # c -> (t, expected remaining)
    first = []
    for r, tm in zip(ev, clk):
        ty, a, b, c, d, w = (int(v) for v in r[:6])
        if ty == 1:
            cls[(a, b)].append((tm, c, w))
            if len(cls[(a, b)]) == 2:
                first.append((tm, "dup classify c %d t %d path %d wave %d (first: %s)" % (a, b, c, w, cls[(a, b)][0])))
        elif ty == 2:
            outst[a] = [b, c]
        elif ty == 3:
            t = a >> 28
            runs[(b, t)].append((tm, a, c, w))
            if len(runs[(b, t)]) == 2:
                first.append((tm, "dup run env %d t %d item %s wave %d" % (b, t, item_s(a), w)))
            ch = b >> 6
            if ch not in outst or outst[ch][0] != t:
                first.append((tm, "run of env %d (chunk %d) at t %d while the chunk's classified step is %s"
                              % (b, ch, t, outst.get(ch, [None])[0])))
            else:
                outst[ch][1] -= 1
                if outst[ch][1] != c - 1:
                    first.append((tm, "chunk %d t %d: device outst %d -> %d, log expects %d" % (ch, t, c, c - 1, outst[ch][1])))
    first.sort()
    for tm, msg in first[:12]:
        print("  @%d %s" % (tm, msg))
    if not first:
        print("  no anomaly")
        return
    # the first anomaly's chunk: every event touching it, in order
    import re
    m = re.search(r"chunk (\d+)|c (\d+)|env (\d+)", first[0][1])
    ch = int(m.group(1) or m.group(2) or (int(m.group(3)) >> 6))
    print("timeline of chunk %d:" % ch)
    for r, tm in zip(ev, clk):
        ty, a, b, c, d, w = (int(v) for v in r[:6])
        if ty in (1, 2) and a == ch:
            print("  @%d %s c %d t %d %s %d wave %d" % (tm, "cls+" if ty == 1 else "cls=", a, b,
                                                      "path" if ty == 1 else "cnt", c, w))
        elif ty == 3 and (b >> 6) == ch:
            print("  @%d run %s env %d old %d lane %d mcnt %d wave %d" % (tm, item_s(a), b, c, d & 255, (d >> 8) & 255, w))


def timing(path):
    raw = np.fromfile(path, dtype=np.uint32)
    hdr, ev = raw[:8], raw[8:].reshape(-1, 8)
    print("%s: %d events, C %d P %d K %d" % (path, hdr[0], hdr[1], hdr[2], hdr[3]))
    clk = ev[:, 6].astype(np.int64) | (ev[:, 7].astype(np.int64) << 32)
    order = np.lexsort((clk, ev[:, 5]))  # by wave, then clock
    ev, clk = ev[order], clk[order]
    t0 = clk.min()
    tot = defaultdict(int)
    durs = defaultdict(list)
    open_ = {}
    span_end = 0
    step_last = defaultdict(int)
    for r, tm in zip(ev, clk):
        ty, a, b, w = int(r[0]), int(r[1]), int(r[2]), int(r[5])
        tm -= t0
        if ty == 10:
            open_[w] = ("gap", tm)
        elif ty in (1, 8, 5, 9):
            kind, st = open_.get(w, ("gap", tm))
            tot[kind] += tm - st
            durs[kind].append(tm - st)
            nxt = {1: "classify", 8: "gap", 5: "run", 9: None}[ty]
            if ty == 5:  # the ticket wait ended
                tot["ticket"] += 0
            if ty == 8:
                open_[w] = ("ticket", tm)
            elif nxt:
                open_[w] = (nxt, tm)
            if ty == 9:
                span_end = max(span_end, tm)
            if ty == 1:
                step_last[b] = max(step_last[b], tm)
        elif ty in (2, 7):
            kind, st = open_.get(w, ("gap", tm))
            tot[kind] += tm - st
            durs[kind].append(tm - st)
            open_[w] = ("gap", tm)
    waves = len(set(ev[:, 5].tolist()))
    allt = sum(tot.values())
    print("waves %d, span %.1f us, wave-time %.1f us per wave" % (waves, span_end / 100, allt / waves / 100))
    for k in sorted(tot):
        d = np.array(durs[k]) / 100
        if not len(d):
            continue
        print("  %-9s %5.1f %%  n %7d  median %7.2f us  p90 %7.2f us  max %8.2f us" % (
            k, 100 * tot[k] / allt, len(d), np.median(d), np.percentile(d, 90), d.max()))
    # classification phases (TG_FLOW_WAVELOG builds: 11 loads returned, 12 rows issued, 13
    # stores complete; 1 start, 2 end)
    ph = defaultdict(list)
    last = {}
    for r, tm in zip(ev, clk):
        ty, w = int(r[0]), int(r[5])
        if ty in (1, 11, 12, 13, 2):
            if ty != 1 and w in last:
                ph[(last[w][0], ty)].append(tm - last[w][1])
            last[w] = (ty, tm)
    for (a, b), d in sorted(ph.items()):
        if len(d) > 1000:
            d = np.array(d) / 100
            print("  classify phase %2d -> %2d: n %7d  median %6.2f us  p90 %6.2f us" % (a, b, len(d), np.median(d), np.percentile(d, 90)))
    print("  last classification of step t at (us):", " ".join("%d:%.0f" % (t, step_last[t] / 100) for t in sorted(step_last)))


if __name__ == "__main__":
    args = sys.argv[1:]
    if args and args[0] == "--time":
        for p in args[1:]:
            timing(p)
    else:
        for p in args:
            main(p)
