#!/usr/bin/env python3
"""A/B timing of step libraries on one GPU (diagnostics; not the bench).

    VARIANTS="base=gym-treasure-game_amd/libtg_amd_r02.so,new=gym-treasure-game_amd/libtg_amd.so" \\
    POLICIES=uniform,masked BURN=3000 STEPS=50 ROUNDS=3 python scripts/ab.py

Each variant is a prebuilt libtg_amd.so (an earlier commit's build, or the product's sources
with -D flags); per policy and round, every variant runs the bench's workload (1,048,576 envs,
seed 0, auto-reset, the bench's action stream) from construction through BURN untimed steps,
then STEPS steps timed with HIP events (tg_step's kernels) and the wall clock.  Variants are
interleaved and the best round (by wall clock) is reported, so that box-to-box spread cancels."""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["TG_AB_LIB"] = "1"
import gym_treasure_game_amd as tg  # noqa: E402
from gym_treasure_game_amd import _lib  # noqa: E402

ACTION_SEED = 0x5EED0001


def time_one(path, policy, n, burn, steps, mode="compact", K=0):
    """K > 0: tg_rollout K steps per call (burn-in and timed steps) in step mode `mode`"""
    _lib._lib = None
    _lib.LIB_PATH = path
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True)
    vec.reset()
    vec.set_mode(mode)
    if K:
        return time_rollout(vec, policy, burn, steps, K)
    rec = torch.empty((1 << 16, 2), dtype=torch.int64, device=vec.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=vec.device)
    for t in range(burn):
        vec.step(vec.policy_actions(t, ACTION_SEED, policy))
        if t % 10 == 9:
            vec.drain_episodes(rec, cnt)
    acts = None
    if policy == "uniform":  # inputs resident before timing, as the bench
        acts = [vec.policy_actions(burn + j, ACTION_SEED, policy).clone() for j in range(steps)]
    regen = hasattr(vec._L, "tg_regenerate")  # deferred MT regeneration (round 3 r03aa+)
    if regen:
        vec.regenerate()
    torch.cuda.synchronize()
    vec.stats_reset()
    vec.set_timing(int(os.environ.get("TIMING", "0")))  # 0: the wall clock only (no events / stamps)
    # DIRECT=1: the bench's call (bench.py step): tg_step through ctypes with the pointers made
    # before timing and no final_obs rows, so that the host's per-call cost (a Python
    # TreasureGameVec.step: ~0.12 ms) does not bound the uniform line
    direct = os.environ.get("DIRECT") == "1" and acts is not None
    if direct:
        p = lambda x: ctypes.c_void_p(x.data_ptr())
        ptrs = [p(a) for a in acts]
        rest = (p(vec._obs), p(vec._rew), p(vec._valid), p(vec._done), None,
                _lib.TG_STEP_AUTORESET, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    t0 = time.perf_counter()
    out = None
    for j in range(steps):
        if direct:
            _lib.check(vec._L.tg_step(vec.handle, ptrs[j], *rest), "tg_step")
        else:
            out = vec.step(acts[j] if acts is not None else vec.policy_actions(burn + j, ACTION_SEED, policy))
        if j % 10 == 9:
            vec.drain_episodes(rec, cnt)
    if regen:
        vec.regenerate()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = vec.stats()
    # the last step's rows and the run's counts: equal for every variant (same results)
    obs = (vec._obs if out is None else out[0]).contiguous().view(torch.int64)
    digest = "%x/%d/%d" % (int((obs * torch.arange(1, obs.numel() + 1, device=obs.device,
                                                       dtype=torch.int64).view_as(obs)).sum()) & (2**64 - 1),
                          st["ticks"], st["draws"])
    vec.close()
    return {"digest": digest, "ms_step": dt / steps * 1e3,
            "kernel_ms": st["kernel_ms"] / max(st.get("timed_launches") or 1, 1),
            "lane_eff": st["ticks"] / max(64 * st["wave_ticks"], 1)}


def time_rollout(vec, policy, burn, steps, K):
    rec = torch.empty((1 << 16, 2), dtype=torch.int64, device=vec.device)
    cnt = torch.zeros(1, dtype=torch.int32, device=vec.device)
    t = 0
    while t < burn:
        k = min(K, burn - t)
        vec.rollout(k, t0=t, action_seed=ACTION_SEED, policy=policy, obs=False, actions=False)
        vec.drain_episodes(rec, cnt)
        t += k
    vec.regenerate()
    torch.cuda.synchronize()
    vec.stats_reset()
    vec.set_timing(int(os.environ.get("TIMING", "0")))
    t0 = time.perf_counter()
    out = None
    for j in range(0, steps, K):
        out = vec.rollout(min(K, steps - j), t0=t + j, action_seed=ACTION_SEED, policy=policy,
                          actions=False)
        vec.drain_episodes(rec, cnt)
    vec.regenerate()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = vec.stats()
    obs = out["obs"][-1].contiguous().view(torch.int64)
    digest = "%x/%d/%d" % (int((obs * torch.arange(1, obs.numel() + 1, device=obs.device,
                                                       dtype=torch.int64).view_as(obs)).sum()) & (2**64 - 1),
                          st["ticks"], st["draws"])
    err = vec.errors()
    vec.close()
    return {"digest": digest, "ms_step": dt / steps * 1e3, "errors": err,
            "kernel_ms": st["kernel_ms"] / max(st.get("timed_launches") or 1, 1),
            "lane_eff": st["ticks"] / max(64 * st["wave_ticks"], 1)}


def main():
    # VARIANTS: name=lib[:mode[:K]], e.g. flow=gym-treasure-game_amd/libtg_amd.so:flow:16
    variants = [v.split("=", 1) for v in os.environ["VARIANTS"].split(",")]
    policies = os.environ.get("POLICIES", "uniform,masked").split(",")
    n = int(os.environ.get("N", 1 << 20))
    steps = int(os.environ.get("STEPS", 50))
    rounds = int(os.environ.get("ROUNDS", 3))
    out = {}
    for pol in policies:
        burn = int(os.environ.get("BURN", 3000 if pol == "uniform" else 1500))
        for r in range(rounds):
            for name, spec in variants:
                path, mode, K = (spec.split(":") + ["compact", "0"])[:3]
                res = time_one(os.path.join(ROOT, path), pol, n, burn, steps, mode, int(K))
                key = "%s/%s" % (pol, name)
                print(key, "round", r, json.dumps(res), flush=True)
                best = out.get(key)
                if best is None or res["ms_step"] < best["ms_step"]:
                    out[key] = res
    for pol in policies:
        ds = {name: out["%s/%s" % (pol, name)]["digest"] for name, _ in variants}
        if len(set(ds.values())) > 1:
            print("DIGEST MISMATCH", pol, json.dumps(ds), flush=True)
    print(json.dumps({"best": out, "n": n, "steps": steps}), flush=True)


if __name__ == "__main__":
    main()
