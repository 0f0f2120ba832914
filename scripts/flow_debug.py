#!/usr/bin/env python3
"""TG_MODE_FLOW bring-up diagnostics: small rollouts with TG_FLOW_DEBUG=1 (the library prints
the XCD census and every sub-problem's counters after each k_flow launch), each checked
against the per-step API.  Diagnostic, not the product."""
import os
import sys

import torch

os.environ["TG_FLOW_DEBUG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402

for n, k in [(int(a.split("x")[0]), int(a.split("x")[1])) for a in (sys.argv[1:] or ["1x3"])]:
    outs = []
    for mode in ("compact", "flow"):
        print("n %d k %d mode %s" % (n, k, mode), flush=True)
        v = tg.TreasureGameVec(n, seed=5, autoreset=True)
        v.reset()
        v.set_mode(mode)
        r = v.rollout(k, t0=0, action_seed=0xA5A5, policy="uniform")
        torch.cuda.synchronize()
        outs.append((r, v.errors()))
        v.close()
    (a, ea), (b, eb) = outs
    same = all(torch.equal(a[key], b[key]) for key in ("reward", "valid", "done", "actions")) and \
        torch.equal(a["obs"].view(torch.int64), b["obs"].view(torch.int64))
    print("n %d k %d errors %x %x equal %s" % (n, k, ea, eb, same), flush=True)
