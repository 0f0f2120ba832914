#!/usr/bin/env python3
"""Per-wave k_run timing from a DIAGNOSTIC build (-DTG_DIAG_STAMPS): for each active wave,
cycles spent loading its envs (+ RNG window), running the option loop and in the epilogue,
with the loop's iteration count (max ticks over its lanes).  Not the product library."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import gym_treasure_game_amd as tg  # noqa: E402
from gym_treasure_game_amd import _lib  # noqa: E402

FLAGS = os.environ.get("FLAGS", "").split()
SO = os.path.join(ROOT, "gym-treasure-game_amd",
                  "libtg_amd_stamps%s.so" % os.environ.get("TAG", ""))


def main():
    from gym_treasure_game_amd import build as B
    if not (os.environ.get("NOBUILD") and os.path.exists(SO)):
        B.compile_lib(SO, extra=["-DTG_DIAG_STAMPS"] + FLAGS)
    _lib._lib = None
    _lib.LIB_PATH = SO
    L = _lib.load()
    L.tg_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    n = int(os.environ.get("N", 1 << 20))
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True)
    vec.reset()
    pol = os.environ.get("POLICY", "uniform")
    for t in range(int(os.environ.get("STEPS", 30))):
        vec.step(vec.policy_actions(t, policy=pol))
    torch.cuda.synchronize()
    # k_run's waves (tg_amd.hip run_grid_for): the env workgroups and 3 of padding (round 3:
    # no REFILL_BLOCKS, the refills are k_regen's)
    nw = min(((n + 255) // 256 + 3) * 4, 1 << 17)
    buf = np.zeros((nw, 11), np.uint64)
    vec.stats_reset()
    vec.step(vec.policy_actions(999, policy=pol))
    torch.cuda.synchronize()
    _lib.check(L.tg_diag_stamps(buf.ctypes.data_as(ctypes.c_void_p), nw), "stamps")
    allw = buf[:, 3] > 0
    idle = allw & ((buf[:, 3] >> 56) == 15)
    if idle.any():
        ist = buf[idle, 4].astype(np.int64)
        ien = buf[idle, 5].astype(np.int64)
        t00 = buf[allw, 4].astype(np.int64).min()
        ih = buf[idle, 10].astype(np.int64)
        print("idle waves %d (refill queue only): halves %d (%.1f per wave, max %d); started by "
              "10%% %.1f 50%% %.1f 90%% %.1f us; ended by 10%% %.1f 50%% %.1f 90%% %.1f 100%% %.1f us"
              % (idle.sum(), ih.sum(), ih.mean(), ih.max(),
                 *np.percentile((ist - t00) / 100.0, [10, 50, 90]),
                 *np.percentile((ien - t00) / 100.0, [10, 50, 90, 100])))
        with_job = idle & (buf[:, 10] > 0)
        if with_job.any():
            jen = (buf[with_job, 5].astype(np.int64) - t00) / 100.0
            print("idle waves that regenerated >= 1 half: %d, ended by 50%% %.1f 90%% %.1f 100%% %.1f us"
                  % (with_job.sum(), *np.percentile(jen, [50, 90, 100])))
    act = allw & ~idle
    oh = buf[act, 10].astype(np.int64)
    print("option waves' queue halves: %d (%.2f per wave)" % (oh.sum(), oh.mean()))
    b = buf[act].astype(np.float64)
    mx = (buf[act, 3] & 0xFFFFFFFF).astype(np.float64)
    sm = ((buf[act, 3] >> 32) & 0xFFFFFF).astype(np.float64)
    kk = (buf[act, 3] >> 56).astype(np.int64)
    print("active waves", act.sum(), "of", nw)
    for name, v in (("load", b[:, 0]), ("loop", b[:, 1]), ("epilogue", b[:, 2]),
                    ("loop/iter", b[:, 1] / np.maximum(mx, 1)), ("max ticks", mx),
                    ("lane eff", sm / 64 / np.maximum(mx, 1))):
        print("%-10s mean %10.1f p50 %10.1f p90 %10.1f max %10.1f" % (
            name, v.mean(), np.median(v), np.percentile(v, 90), v.max()))
    long = mx >= 80
    if long.any():
        v = b[long, 1] / mx[long]
        print("long waves (>=80 iters): %d, loop/iter mean %.1f p50 %.1f; load mean %.1f epi mean %.1f"
              % (long.sum(), v.mean(), np.median(v), b[long, 0].mean(), b[long, 2].mean()))
    # timeline (s_memrealtime, 100 MHz, chip-wide)
    st = buf[act, 4].astype(np.int64)
    en = buf[act, 5].astype(np.int64)
    t0 = st.min()
    st_us, en_us = (st - t0) / 100.0, (en - t0) / 100.0
    span = en_us.max()
    print("span %.1f us; waves started by: 10%% %.1f 50%% %.1f 90%% %.1f 100%% %.1f us"
          % (span, *np.percentile(st_us, [10, 50, 90, 100])))
    print("waves ended by: 10%% %.1f 50%% %.1f 90%% %.1f 99%% %.1f 100%% %.1f us"
          % tuple(np.percentile(en_us, [10, 50, 90, 99, 100])))
    for t in np.linspace(0, span, 11):
        print("  t=%6.1f us active waves %5d" % (t, ((st_us <= t) & (en_us > t)).sum()))
    names = ["go_left", "go_right", "up_ladder", "down_ladder", "interact", "down_left",
             "down_right", "jump_left", "jump_right", "reset_only"]
    for k in range(10):
        sel = kk == k
        if sel.any():
            print("  %-11s waves %5d end max %6.1f us p90 %6.1f  iters max %4d mean %5.1f  cyc/iter %6.0f"
                  "  | loop %7.0f = walk %7.0f + refill %7.0f + full ticks %7.0f, rounds %5.1f"
                  % (names[k], sel.sum(), en_us[sel].max(), np.percentile(en_us[sel], 90),
                     mx[sel].max(), mx[sel].mean(), (b[sel, 1] / np.maximum(mx[sel], 1)).mean(),
                     b[sel, 1].mean(), b[sel, 6].mean(), b[sel, 7].mean(), b[sel, 8].mean(),
                     b[sel, 9].mean()))
    top = np.argsort(-en_us)[:10]
    for j in top:
        print("  last: start %.1f end %.1f us iters %d loop cyc/iter %.0f" % (
            st_us[j], en_us[j], mx[j], b[j, 1] / max(mx[j], 1)))
    w = np.flatnonzero(act)
    for lo, hi in ((0, 100), (len(w) // 2, len(w) // 2 + 5), (len(w) - 5, len(w))):
        for k in range(lo, min(hi, len(w)), max(1, (hi - lo) // 5)):
            print("  wave %6d load %8d loop %9d epi %8d iters %4d" % (
                w[k], buf[w[k], 0], buf[w[k], 1], buf[w[k], 2], buf[w[k], 3] & 0xFFFFFFFF))
    vec.close()


if __name__ == "__main__":
    main()
