#!/usr/bin/env python3
"""DIAGNOSTIC (not the bench): would stepping the batch as G independent sub-batches on G HIP
streams overlap one sub-batch's latency-bound k_run tail with another's bandwidth-bound
k_classify / k_regen, and so raise env-steps/s?  The envs share nothing, so a batch
of N is G handles of N / G envs (global offsets g N / G: the same trajectories).

    N=1048576 GS=1,2,4 STEPS=100 BURN=3000 STAGGER=1 python scripts/overlap_probe.py

Per G: the handles are created, burned in (untimed, uniform policy), their timed actions
generated before timing; then each of STEPS rounds enqueues one tg_step per handle, each on its
own stream (round-robin, no host synchronisation), and a final tg_regenerate per handle; the
wall clock between device synchronisations gives the whole batch's steps/s.  STAGGER=1 delays
stream g by g / G of a step (torch.cuda._sleep) before the timed loop, so the streams start out
of phase."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402

A0 = 0x5EED0001


def p(t):
    return ctypes.c_void_p(t.data_ptr())


def run(n, G, steps, burn, stagger, dev):
    L = tg._lib.load()
    m = n // G
    vecs, streams = [], []
    for g in range(G):
        v = tg.TreasureGameVec(m, seed=0, global_offset=g * m, autoreset=False, device=dev)
        v.autoreset = True
        v.reset()
        vecs.append(v)
        streams.append(torch.cuda.Stream(dev))
    flags = tg._lib.TG_STEP_AUTORESET

    def step(g, a):
        v = vecs[g]
        tg._lib.check(L.tg_step(v.handle, p(a), p(v._obs), p(v._rew), p(v._valid), p(v._done),
                                None, flags, v._stream()), "tg_step")

    for t in range(burn):
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                step(g, vecs[g].policy_actions(t, A0, "uniform"))
    acts = []
    for g in range(G):
        with torch.cuda.stream(streams[g]):
            acts.append([vecs[g].policy_actions(burn + j, A0, "uniform").clone() for j in range(steps)])
            vecs[g].regenerate()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if stagger and G > 1:
        for g in range(1, G):
            with torch.cuda.stream(streams[g]):
                torch.cuda._sleep(int(2.1e3 * 130 * g / G))  # ~g/G of a 130-us step at ~2.1 GHz
    for j in range(steps):
        for g in range(G):
            with torch.cuda.stream(streams[g]):
                step(g, acts[g][j])
    for g in range(G):
        with torch.cuda.stream(streams[g]):
            vecs[g].regenerate()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    errs = sum(v.errors() for v in vecs)
    for v in vecs:
        v.close()
    return {"G": G, "stagger": bool(stagger), "ms_per_step": dt / steps * 1e3,
            "env_steps_per_s": n * steps / dt, "errors": errs}


def main():
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("N", 1 << 20))
    steps = int(os.environ.get("STEPS", 100))
    burn = int(os.environ.get("BURN", 3000))
    for G in [int(x) for x in os.environ.get("GS", "1,2,4").split(",")]:
        for stg in ([0, 1] if G > 1 else [0]):
            print(json.dumps(run(n, G, steps, burn, stg, dev)), flush=True)


if __name__ == "__main__":
    main()
