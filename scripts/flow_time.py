#!/usr/bin/env python3
"""Where k_flow's waves spend a launch (round 6's run-ahead form), from a TG_FLOW_WAVELOG build's
event log (TG_FLOW_LOG=<prefix>: <prefix>.<launch>.bin, tg_flow_diag.h).  Per wave, the time
between consecutive lane-0 events is charged to the segment it ends:
  10 start -> 16 deal chunk / 8 ticket taken        (loop overhead)
  16 deal chunk -> 14 run-ahead done                 deal: loads + run-ahead from step 0
  8 ticket taken -> 5 item served                    waiting for an item
  5 item served -> 7 run done                        option loops (k_run's work)
  7 run done -> 14 run-ahead done                    run-ahead after a run
  14 run-ahead done -> 15 published                  listing, state stores, fills, step counts
  15 published -> 16 / 8                             loop overhead
  8 -> 9 exit                                        the final wait
Diagnostic, not the product."""
import sys
from collections import defaultdict

import numpy as np

NAMES = {(10, 16): "start", (10, 8): "start", (16, 14): "deal", (8, 5): "wait", (5, 7): "run",
         (7, 14): "ahead", (14, 15): "publish", (15, 16): "loop", (15, 8): "loop", (8, 9): "final wait",
         (16, 8): "loop"}


def main(path):
    raw = np.fromfile(path, dtype=np.uint32)
    hdr, ev = raw[:8], raw[8:].reshape(-1, 8)
    cnt, C, P, K = (int(v) for v in hdr[:4])
    clk = ev[:, 6].astype(np.int64) | (ev[:, 7].astype(np.int64) << 32)
    t0 = clk.min()
    byw = defaultdict(list)
    for r, tm in zip(ev, clk):
        byw[int(r[5])].append((tm - t0, int(r[0]), int(r[1]), int(r[2])))
    seg = defaultdict(float)
    nseg = defaultdict(int)
    ends = []
    for w, evs in byw.items():
        evs.sort()
        for (ta, ya, _, _), (tb, yb, _, _) in zip(evs, evs[1:]):
            name = NAMES.get((ya, yb), "%d->%d" % (ya, yb))
            seg[name] += tb - ta
            nseg[name] += 1
        ends.append(evs[-1][0])
    tot = sum(seg.values())
    span = max(ends)
    print("%s: %d events, %d waves, C %d P %d K %d, launch span %.1f us (%.1f us per step)"
          % (path, cnt, len(byw), C, P, K, span / 100.0, span / 100.0 / max(K, 1)))
    for name in sorted(seg, key=lambda k: -seg[k]):
        print("  %-12s %5.1f %% of wave time, %7d segments, mean %7.2f us"
              % (name, 100.0 * seg[name] / tot, nseg[name], seg[name] / nseg[name] / 100.0))
    ends = np.sort(np.array(ends)) / 100.0
    print("  waves ended by: 10%% %.1f 50%% %.1f 90%% %.1f 100%% %.1f us"
          % tuple(np.percentile(ends, [10, 50, 90, 100])))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
