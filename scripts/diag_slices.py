#!/usr/bin/env python3
"""Diagnostics: the C3 workload (1,048,576 envs, uniform options, auto-reset) as K
independent handles of N/K envs (global offsets g*N/K), each stepping on its own HIP stream,
so one slice's long k_run tail overlaps the other slices' work.  ms per whole-batch step for
K in SLICES; every env takes the same trajectory for any K (keyed by the global index)."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402

N = int(os.environ.get("ENVS", 1 << 20))
STEPS = int(os.environ.get("STEPS", 100))
WARM = int(os.environ.get("WARMUP", 10))


def run(k):
    dev = torch.device("cuda", 0)
    per = N // k
    vecs, streams = [], []
    for s in range(k):
        v = tg.TreasureGameVec(per, seed=0, global_offset=s * per, device=dev)
        v.autoreset = True
        v.reset()
        vecs.append(v)
        streams.append(torch.cuda.Stream(dev))
    L = vecs[0]._L
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    rows = [torch.empty((4096, 2), dtype=torch.int64, device=dev) for _ in range(k)]
    cnts = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(k)]
    torch.cuda.synchronize()

    def step(t):
        for s, v in enumerate(vecs):
            st = ctypes.c_void_p(streams[s].cuda_stream)
            h = v.handle
            L.tg_policy_actions(h, 0x5EED0001, t, 0, p(v._act), st)
            L.tg_step(h, p(v._act), p(v._obs), p(v._rew), p(v._valid), p(v._done), None, 1, st)
            L.tg_episodes(h, p(rows[s]), p(cnts[s]), 4096, st)

    for t in range(WARM):
        step(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(WARM, WARM + STEPS):
        step(t)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    stats = [v.stats() for v in vecs]
    for v in vecs:
        assert v.errors() == 0
        v.close()
    return {"ms_per_step": dt / STEPS * 1e3, "env_steps_per_s": N * STEPS / dt,
            "steps_counted": sum(s["steps"] for s in stats)}


def main():
    out = {}
    for k in [int(x) for x in os.environ.get("SLICES", "1,2,4,8").split(",")]:
        out[k] = run(k)
        print(k, out[k], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
