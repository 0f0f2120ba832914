#!/usr/bin/env python3
"""Determinism check (diagnostic): two identical 1M-env runs must agree bit for bit on every
env; the oracle replays the envs that differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import gym_treasure_game_amd as tg  # noqa: E402
import oracle as O  # noqa: E402


def run(n, steps, mode):
    vec = tg.TreasureGameVec(n, seed=11, autoreset=True, mode=mode)
    vec.reset()
    obs = []
    for t in range(steps):
        o, r, v, d, info = vec.step(vec.policy_actions(t, 0xC3, "uniform"))
        obs.append(info["final_obs"].cpu().numpy().view(np.uint64).copy())
    st = vec.stats()
    vec.close()
    return np.stack(obs, 1), st


def main():
    n, steps = 1 << 20, 40
    mode = sys.argv[1] if len(sys.argv) > 1 else "compact"
    a, sa = run(n, steps, mode)
    b, sb = run(n, steps, mode)
    diff = np.argwhere((a != b).any(axis=(1, 2))).ravel()
    print("runs differ on %d envs" % len(diff), diff[:20].tolist(), sa["draws"], sb["draws"])
    O.build()
    for e in ([702001] + diff[:4].tolist()):
        r = O.run(11, int(e), 1, steps, 0xC3, 0, True)
        ro = r["final_obs"][0, 1:].view(np.uint64)
        for name, x in (("a", a[e]), ("b", b[e])):
            bad = np.argwhere(x != ro)
            print("env", e, name, "vs oracle: first bad", bad[0].tolist() if len(bad) else None,
                  "draws", int(r["draws"][0]))


if __name__ == "__main__":
    main()
