#!/usr/bin/env python3
"""The N = 1 drop-in's call latency alone (bench.dropin_latency), for a profiler to wrap:

    rocprofv3 --kernel-trace --stats -d DIR -- python3 scripts/dropin_run.py [STEPS]

Also prints the floor of one launch + one synchronisation on this box: a one-element torch
add_ and hipStreamSynchronize, timed the same way.  Diagnostic, not the product."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import gym_treasure_game_amd as tg  # noqa: E402


def launch_sync_floor(n=2000):
    x = torch.zeros(1, device="cuda")
    for _ in range(50):
        x.add_(1)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        x.add_(1)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def wrapper_step_us(serve, n=300):
    """ObservationWrapper(TreasureGame) step: the env step + a rendered frame to the host"""
    w = tg.ObservationWrapper(tg.TreasureGame(seed=3), sprites=tg.synthetic_sprites(seed=1))
    w.env._vec.set_serve(serve)  # (the wrapper turns serving off; on: the A/B)
    w.reset()
    for i in range(20):
        w.step(i % 9)
    t0 = time.perf_counter()
    for i in range(n):
        if w.step(i % 9)[2]:
            w.reset()
    dt = (time.perf_counter() - t0) / n * 1e6
    w.env.close()
    return dt


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    out = bench.dropin_latency(tg, steps=steps)
    out["launch_sync_floor_us"] = launch_sync_floor()
    out["wrapper_step_us_serve_off"] = wrapper_step_us(False)
    out["wrapper_step_us_serve_on"] = wrapper_step_us(True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
