#!/usr/bin/env python3
"""Reads a TG_FLOW_DBG build's k_flow event log (TG_FLOW_LOG=<prefix>: <prefix>.<launch>.bin) and
reports the first protocol anomaly in clock order: a chunk classified twice for one step, an
env run twice for one step, a chunk's outstanding count out of step.  Diagnostic, not the product.

Records (8 x u32): type, a, b, c, d, wave, clock lo, clock hi
  1 classify start (c, t, path, x)    2 classify end (c, t, cnt, x)
  3 run lane (item, env, old outst, lane | mcnt << 8 | x << 16)
  4 push (item, slot, src, x)         5 ticket (h, item, x)"""
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


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
