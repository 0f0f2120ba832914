#!/usr/bin/env python3
"""A timed region's fixed costs on this platform, with
empty kernels (tg_probe_dispatch), timed exactly as bench.py times its region: barrier-free
torch.cuda.synchronize() on both sides, HIP events on the stream around it, the end event polled.

  (a) region of ONE empty kernel: the idle GPU's first dispatch + completion + the host's sync
  (b) regions of N = 2, 20, 40, 200 dependent empty kernels: the per-boundary gap is the slope
      (N empty kernels take N - 1 dependent boundaries), the constant the intercept
  (c) the same with the kernels at 4,096 workgroups (the step kernels' grid at 1M envs)

Prints one JSON line.  Diagnostic, not the product."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gym_treasure_game_amd import _lib  # noqa: E402


def region(L, st, n, blocks, reps):
    walls, evs = [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        _lib.check(L.tg_probe_dispatch(n, blocks, st), "probe")
        e1.record()
        while not e1.query():
            pass
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
        evs.append(e0.elapsed_time(e1))
    return statistics.median(walls), statistics.median(evs)


def main():
    L = _lib.load()
    torch.zeros(1, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = {}
    for blocks in (1, 4096):
        region(L, st, 50, blocks, 3)  # warm
        rows = {}
        for n in (1, 2, 20, 40, 200):
            w, e = region(L, st, n, blocks, 30)
            rows[n] = {"wall_ms": w, "events_ms": e}
        slope_w = (rows[200]["wall_ms"] - rows[20]["wall_ms"]) / 180
        slope_e = (rows[200]["events_ms"] - rows[20]["events_ms"]) / 180
        out["blocks_%d" % blocks] = {
            "regions": rows,
            "per_kernel_ms_wall": slope_w, "per_kernel_ms_events": slope_e,
            "region_constant_ms_wall": rows[20]["wall_ms"] - 20 * slope_w,
            "wall_minus_events_ms": {n: r["wall_ms"] - r["events_ms"] for n, r in rows.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
