#!/usr/bin/env python3
"""A/B timing of step variants on one GPU (diagnostics; not the bench).

Builds (if needed) and times, per variant, ms per batched step at 1,048,576 envs with the
bench's workload: the product library in both step modes, and a DIAGNOSTIC build
(-DTG_DIAG_NORNG: MT words from a register hash, no MT memory traffic; results are NOT
reference-exact) to price the RNG's memory traffic.  Interleaved, best of 3 rounds.
"""
import ctypes
import json
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402
from gym_treasure_game_amd import _lib  # noqa: E402

VARIANTS = os.environ.get(
    "VARIANTS", "prod:compact:,prod:direct:,norng:compact:-DTG_DIAG_NORNG,norng:direct:-DTG_DIAG_NORNG")


def build_variant(name, flags):
    """Variant libraries: the product sources with extra -D flags (diagnostic builds only)."""
    if not flags:
        return _lib.LIB_PATH
    if flags.startswith("@"):  # a prebuilt library, e.g. an earlier commit's (A/B)
        return os.path.join(ROOT, flags[1:])
    out = os.path.join(ROOT, "gym-treasure-game_amd", "libtg_amd_%s.so" % name)
    if os.environ.get("NOBUILD") and os.path.exists(out):
        return out
    from gym_treasure_game_amd import build as B
    subprocess.check_call([B.HIPCC] + B.FLAGS + flags.split() + ["-o", out] + B.SRCS)
    return out


def time_variant(lib_path, mode, n, steps, warmup):
    _lib._lib = None
    _lib.LIB_PATH = lib_path
    vec = tg.TreasureGameVec(n, seed=0, mode=mode)
    vec.reset()
    for t in range(warmup):
        vec.step(vec.policy_actions(t))
    torch.cuda.synchronize()
    vec.stats_reset()
    vec.set_timing(True)
    t0 = time.perf_counter()
    for t in range(warmup, warmup + steps):
        vec.step(vec.policy_actions(t))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = vec.stats()
    vec.close()
    return {"ms_step": dt / steps * 1e3, "kernel_ms": st["kernel_ms"] / steps,
            "ticks": st["ticks"] / steps}


def main():
    n = int(os.environ.get("N", 1 << 20))
    steps, warmup = 60, int(os.environ.get("WARMUP", 300))
    prod = _lib.LIB_PATH
    variants = []
    only = os.environ.get("ONLY")
    for v in VARIANTS.split(","):
        name, mode, flags = v.split(":", 2)
        if only and name != only:
            continue
        variants.append((name, build_variant(name, flags), mode))
    if os.environ.get("BUILD_ONLY"):
        return
    best = {}
    for _ in range(int(os.environ.get("ROUNDS", 3))):
        for name, path, mode in variants:
            r = time_variant(path, mode, n, steps, warmup)
            k = "%s/%s" % (name, mode)
            if k not in best or r["kernel_ms"] < best[k]["kernel_ms"]:
                best[k] = r
    _lib._lib = None
    _lib.LIB_PATH = prod
    print(json.dumps(best, indent=1))


if __name__ == "__main__":
    main()
