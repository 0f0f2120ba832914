#!/usr/bin/env python3
"""A/B timing of k_render variants (diagnostics; not the bench).

Builds (if needed) the product sources with extra -D flags per variant and times tg_render of
N envs (default 65,536 = config C5) into a resident frame buffer: HIP-event ms per launch and
the frame-write rate.  Interleaved, best of 3 rounds.
    VARIANTS="g16:,g1:-DTG_RENDER_G=1,plain:-DTG_RENDER_NT=0" python scripts/diag_render.py
"""
import ctypes
import json
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402
from gym_treasure_game_amd import _lib  # noqa: E402
from gym_treasure_game_amd import build as B  # noqa: E402

VARIANTS = os.environ.get("VARIANTS", "g16:,g4:-DTG_RENDER_G=4,g1:-DTG_RENDER_G=1,"
                                      "plain:-DTG_RENDER_NT=0,g32:-DTG_RENDER_G=32")
N = int(os.environ.get("ENVS", 65536))
REPS = int(os.environ.get("REPS", 10))


def build_variant(name, flags):
    if not flags:
        return _lib.LIB_PATH
    out = os.path.join(ROOT, "gym-treasure-game_amd", "libtg_amd_r%s.so" % name)
    if not (os.environ.get("NOBUILD") and os.path.exists(out)):
        subprocess.check_call([B.HIPCC] + B.FLAGS + flags.split() + ["-o", out] + B.SRCS)
    return out


def time_variant(lib_path, frames):
    _lib._lib = None
    _lib.LIB_PATH = lib_path
    vec = tg.TreasureGameVec(N, seed=0, autoreset=True)
    vec.render_init(tg.synthetic_sprites(seed=1))
    vec.reset()
    for t in range(5):
        vec.step(vec.policy_actions(t))
    vec.render(out=frames)
    torch.cuda.synchronize()
    evs = []
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        vec.render(out=frames)
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)[len(evs) // 2]
    chk = int(frames.view(N, -1)[:, ::4099].to(torch.int64).sum().item())
    assert vec.errors() == 0
    vec.close()
    return ms, chk


def main():
    vs = [v.split(":", 1) for v in VARIANTS.split(",") if v]
    libs = {name: build_variant(name, flags) for name, flags in vs}
    if os.environ.get("BUILD_ONLY"):
        return
    frames = torch.empty((N, 624, 672, 3), dtype=torch.uint8, device="cuda")
    res = {name: [] for name, _ in vs}
    chks = {}
    for _ in range(3):
        for name, _ in vs:
            ms, chk = time_variant(libs[name], frames)
            res[name].append(ms)
            chks[name] = chk
    out = {}
    # write-rate references on the same buffer: torch fill (a streaming-store kernel) and
    # hipMemsetAsync (zero_)
    for name, fn in (("torch_fill", lambda: frames.fill_(7)), ("memset", lambda: frames.zero_())):
        fn()
        torch.cuda.synchronize()
        evs = []
        for _ in range(REPS):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            evs.append((a, b))
        torch.cuda.synchronize()
        ms = min(a.elapsed_time(b) for a, b in evs)
        out[name] = {"ms": ms, "TB/s": frames.numel() / ms / 1e9}
    for name, _ in vs:
        ms = min(res[name])
        out[name] = {"ms": ms, "TB/s": N * 1257984 / ms / 1e9, "checksum": chks[name]}
    print(json.dumps(out, indent=1))
    prod = {n: c for n, c in chks.items() if not n.startswith("diag")}
    assert len(set(prod.values())) <= 1, "variants disagree"


if __name__ == "__main__":
    main()
