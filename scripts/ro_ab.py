"""A/B of tg_rollout: the per-step kernels (compact) vs k_rollout (async) at the bench's size.
Usage: python scripts/ro_ab.py [n] [K] [burn_in] — prints ms per env-step for each variant."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402
from gym_treasure_game_amd import _lib  # noqa: E402

# VARIANTS="name:mode:path,..." (prebuilt libraries); default: this tree's library, both modes
VARIANTS = [v.split(":") for v in os.environ.get(
    "VARIANTS", "compact:compact:%s,async:async:%s" % (_lib.LIB_PATH, _lib.LIB_PATH)).split(",")]

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
K = int(sys.argv[2]) if len(sys.argv) > 2 else 100
burn = int(sys.argv[3]) if len(sys.argv) > 3 else 300
policy = os.environ.get("POLICY", "uniform")
a0 = 0x5EED0001
res = {}
for name, mode, path in VARIANTS:
    _lib._lib = None
    _lib.LIB_PATH = path if os.path.isabs(path) else os.path.join(ROOT, path)
    v = tg.TreasureGameVec(n, seed=0, autoreset=True, mode=mode)
    v.reset()
    v.rollout(burn, t0=0, action_seed=a0, policy=policy, obs=False, actions=False)
    v.episodes(cap=1 << 24)
    torch.cuda.synchronize()
    t = burn
    for rep in range(3):
        v.stats_reset()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        out = v.rollout(K, t0=t, action_seed=a0, policy=policy, obs=True, actions=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t1
        t += K
        st = v.stats()
        v.episodes(cap=1 << 24)
        del out
        res["%s/%d" % (name, rep)] = {"ms_step": dt / K * 1e3, "steps": st["steps"],
                                      "ticks": st["ticks"], "regens": st["regens"],
                                      "wave_ticks": st["wave_ticks"],
                                      "env_steps_per_s": n * K / dt}
    print(name, "errors", v.errors(), flush=True)
    v.close()
print(json.dumps(res, indent=1))
