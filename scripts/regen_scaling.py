#!/usr/bin/env python3
"""DIAGNOSTIC (not the bench): k_regen's launch time against the refill lists it drains.
After a burn-in (the bench's workload: 1M envs, uniform policy, auto-reset), each trial steps
S steps with the lists left pending (S < 16: no automatic drain), then times the one
tg_regenerate launch that drains them (in-kernel span stamps, tg_set_timing), and reports
ms per launch and per 1,000 generations.  A launch's fixed cost is the intercept."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402

A0 = 0x5EED0001


def main():
    n = int(os.environ.get("N", 1 << 20))
    pol = os.environ.get("POLICY", "uniform")
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True)
    vec.reset()
    rec = torch.empty((1 << 16, 2), dtype=torch.int64, device=vec.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=vec.device)
    t = 0
    for _ in range(int(os.environ.get("BURN", 3000))):
        vec.step(vec.policy_actions(t, A0, pol))
        t += 1
        if t % 10 == 0:
            vec.drain_episodes(rec, cnt)
    for s in [int(x) for x in os.environ.get("SLOTS", "1,2,4,8,15,1,2,4,8,15").split(",")]:
        vec.regenerate()  # nothing pending
        torch.cuda.synchronize()
        for _ in range(s):
            vec.step(vec.policy_actions(t, A0, pol))
            t += 1
        vec.drain_episodes(rec, cnt)
        torch.cuda.synchronize()
        vec.stats_reset()
        vec.set_timing(1)
        vec.regenerate()
        torch.cuda.synchronize()
        st = vec.stats()
        vec.set_timing(0)
        ms = st["regen_ms"] / max(st["regen_timed"], 1)
        gens = st["regens"]
        print(json.dumps({"slots": s, "launches": st["regen_timed"], "ms": ms, "generations": gens,
                          "ns_per_generation": ms * 1e6 / max(gens, 1)}), flush=True)


if __name__ == "__main__":
    main()
