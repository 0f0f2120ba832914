"""The product's per-env core (csrc/tg_core.h: double-buffered MT generations, cell-level predicates,
register-stack trigger cascade) compiled for the host, against the golden vectors and the
oracle.  This is the same code every kernel lane runs; the GPU tests then check the kernels
themselves (LDS staging, SoA packing, ballots) on the device."""
import ctypes
import os

import numpy as np
import pytest

from conftest import golden

KEYS = ["obs", "reward", "valid", "done", "final_obs", "hash", "draws", "ticks"]


CORRIDOR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels", "corridor")


def level_texts(level_dir):
    if level_dir is None:
        return None, None, None
    return tuple(open(os.path.join(level_dir, f), "rb").read()
                 for f in ("domain.txt", "domain-objects.txt", "domain-interactions.txt"))


def hc_run(lib, seed_base, g0, n, steps, a0, policy, autoreset, level_dir=None):
    t1 = steps + 1
    o = {"obs": np.zeros((n, t1, 9)), "final_obs": np.zeros((n, t1, 9)),
         "reward": np.zeros((n, t1), np.int32), "valid": np.zeros((n, t1), np.uint8),
         "done": np.zeros((n, t1), np.uint8), "hash": np.zeros(n, np.uint64),
         "draws": np.zeros(n, np.int64), "ticks": np.zeros(n, np.int64)}
    p = {k: o[k].ctypes.data_as(ctypes.c_void_p) for k in o}
    rc = lib.hc_run(*level_texts(level_dir), seed_base, g0, n, steps, a0, policy, int(autoreset),
                    p["obs"], p["reward"], p["valid"], p["done"], p["final_obs"], p["hash"],
                    p["draws"], p["ticks"])
    assert rc == 0
    return o


def assert_same(a, b, keys=("obs", "final_obs", "reward", "valid", "done", "hash", "draws")):
    for k in keys:
        x, y = a[k], b[k]
        if x.dtype == np.float64:
            x, y = x.view(np.uint64), y.view(np.uint64)
        np.testing.assert_array_equal(x, y, err_msg=k)


@pytest.mark.parametrize("name,policy,autoreset", [("traj_uniform.npz", 0, False),
                                                   ("traj_masked.npz", 1, False),
                                                   ("traj_autoreset.npz", 1, True)])
def test_core_vs_golden_trajectories(hostcheck, name, policy, autoreset):
    d = golden(name)
    n, t1 = d["valid"].shape
    o = hc_run(hostcheck, int(d["seed_base"]), 0, n, t1 - 1, int(d["action_seed"]), policy,
               autoreset)
    g = {k: d[k] for k in ("obs", "final_obs", "reward", "valid", "done")}
    assert_same(o, g, keys=list(g))
    np.testing.assert_array_equal(o["draws"], d["draws"][:, -1])


@pytest.mark.parametrize("name,policy", [("hash_uniform.npz", 0), ("hash_masked.npz", 1)])
def test_core_vs_golden_hashes(hostcheck, name, policy):
    d = golden(name)
    o = hc_run(hostcheck, 0, 0, len(d["hash"]), int(d["steps"]), int(d["action_seed"]), policy,
               False)
    np.testing.assert_array_equal(o["hash"], d["hash"])
    np.testing.assert_array_equal(o["draws"], d["draws"])
    np.testing.assert_array_equal(o["ticks"], d["ticks"])


def test_core_predicates_vs_golden_and_oracle(hostcheck, oracle):
    d = golden("predicates.npz")
    x0, x1, y0, y1 = (int(v) for v in d["box"])
    e = oracle.OracleEnv(0)
    for db in range(8):  # all door states vs the oracle, the two pinned ones vs the reference
        out = np.zeros((y1 - y0, x1 - x0), np.uint8)
        hostcheck.hc_predicate_table(x0, x1, y0, y1, db, out.ctypes.data_as(ctypes.c_void_p))
        np.testing.assert_array_equal(out, e.predicate_table(x0, x1, y0, y1, db), err_msg=str(db))
        if db in (0, 7):
            np.testing.assert_array_equal(out, d["table"][0 if db == 0 else 1])


@pytest.mark.parametrize("seed_base,g0,n,steps,policy,autoreset", [
    (10**9, 0, 2048, 400, 0, False),          # other seeds, uniform
    (2**32 - 100, 0, 256, 300, 0, False),     # seeds crossing 2**32 (2-word init_by_array keys)
    (0, 2**40, 256, 300, 1, True),            # huge global index, masked + auto-reset
    (7, 5000, 512, 2500, 1, True),            # long masked runs: many episodes and resets
])
def test_core_vs_oracle(hostcheck, oracle, seed_base, g0, n, steps, policy, autoreset):
    a0 = 0xA5A5 + policy
    o = hc_run(hostcheck, seed_base, g0, n, steps, a0, policy, autoreset)
    r = oracle.run(seed_base, g0, n, steps, a0, policy, autoreset)
    assert_same(o, r)
    np.testing.assert_array_equal(o["ticks"], r["ticks"])
    if autoreset and steps > 1000:
        assert r["done"].sum() > 0


@pytest.mark.parametrize("seed", [0, 1, 12345, (1 << 32) + 5])
@pytest.mark.parametrize("pattern", ["small", "boundaries", "long"])
@pytest.mark.parametrize("defer", [1, 3, 0])
def test_rng_generations_vs_cpython(hostcheck, seed, pattern, defer):
    """tg::Rng's two pre-twisted generations == CPython's random() stream (Python's own random
    module IS the reference's generator).  The stale half is refilled before every launch,
    every third launch, or never (defer 0: every crossing regenerates in-launch); "long"
    launches cross two and three generation boundaries inside one launch."""
    import random
    rs = np.random.default_rng(seed & 0xFFFF)
    if pattern == "small":
        launches = rs.integers(0, 9, 600)
    elif pattern == "boundaries":
        launches = np.array([312, 312, 1, 311, 312, 2, 310, 312, 312, 624 - 2, 3])
    else:
        launches = np.array([5, 313, 700, 1, 950, 0, 312, 1000, 7])
    launches = launches.astype(np.int32)
    total = int(launches.sum())
    out = np.zeros(total)
    assert hostcheck.hc_rng_stream(seed, launches.ctypes.data_as(ctypes.c_void_p), len(launches),
                                   defer, out.ctypes.data_as(ctypes.c_void_p)) == 0
    r = random.Random(seed)
    want = np.array([r.random() for _ in range(total)])
    assert np.array_equal(out, want)


@pytest.mark.parametrize("policy,autoreset", [(0, False), (1, True)])
def test_core_vs_oracle_corridor(hostcheck, oracle, policy, autoreset):
    """Custom level whose go options take ~650 draws in one step (two MT generation crossings
    inside one launch; tests/golden/levels/corridor/README.md)."""
    n, steps, a0 = 64, 30, 0xC0FFEE
    o = hc_run(hostcheck, 3, 0, n, steps, a0, policy, autoreset, level_dir=CORRIDOR)
    r = oracle.run(3, 0, n, steps, a0, policy, autoreset, level_dir=CORRIDOR)
    assert_same(o, r)
    np.testing.assert_array_equal(o["ticks"], r["ticks"])
    assert r["draws"].max() > 624 * 4  # many multi-generation steps really happened


LEVELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels")


@pytest.mark.parametrize("level", ["corridor", "gen1", "gen2", "gen3", "exit", "cascade"])
@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_core_vs_reference_levels(hostcheck, level, policy):
    """F6: the product core's level loader + physics vs the reference on other levels."""
    d = golden("traj_level_%s_%s.npz" % (level, policy))
    n, t1 = d["valid"].shape
    o = hc_run(hostcheck, int(d["seed_base"]), 0, n, t1 - 1, int(d["action_seed"]),
               int(d["masked"]), bool(d["autoreset"]), level_dir=os.path.join(LEVELS, level))
    g = {k: d[k] for k in ("obs", "final_obs", "reward", "valid", "done")}
    assert_same(o, g, keys=list(g))
    np.testing.assert_array_equal(o["draws"], d["draws"][:, -1])


@pytest.mark.parametrize("level", [None, "corridor", "gen1", "gen2", "gen3", "exit", "cascade"])
@pytest.mark.parametrize("policy", [0, 1])
def test_core_gotable_matches_direct(hostcheck, level, policy):
    """The go options' GoTable (tg_core.h go_lookup, the device's path) against the direct
    scan it replaces, over whole auto-reset trajectories (keys and gold picked up and dropped
    into the bag, every door state the levels reach)."""
    ld = None if level is None else os.path.join(LEVELS, level)
    try:
        hostcheck.hc_set_gotab(0)
        direct = hc_run(hostcheck, 11, 0, 256, 60, 0xBEEF, policy, True, level_dir=ld)
    finally:
        hostcheck.hc_set_gotab(1)
    table = hc_run(hostcheck, 11, 0, 256, 60, 0xBEEF, policy, True, level_dir=ld)
    assert_same(direct, table)
    np.testing.assert_array_equal(direct["ticks"], table["ticks"])


@pytest.mark.parametrize("level", [None, "corridor", "gen1", "gen2", "gen3", "exit", "cascade"])
@pytest.mark.parametrize("policy", [0, 1])
def test_core_level_masks_match_cell_probes(hostcheck, level, policy):
    """The level bitmasks (tg_core.h Map::mk: the ladder options' fused full tick and span
    limits, the go options' span limits as bit scans; the device's path) against the cell
    probes they replace, over whole auto-reset trajectories on seven levels, and both against
    the oracle (the other host tests run with the masks on)."""
    ld = None if level is None else os.path.join(LEVELS, level)
    try:
        hostcheck.hc_set_masks(0)
        probes = hc_run(hostcheck, 13, 0, 512, 80, 0xFACE, policy, True, level_dir=ld)
    finally:
        hostcheck.hc_set_masks(1)
    masks = hc_run(hostcheck, 13, 0, 512, 80, 0xFACE, policy, True, level_dir=ld)
    assert_same(probes, masks)
    np.testing.assert_array_equal(probes["ticks"], masks["ticks"])


def test_draw_code_from_the_top_27_bits(hostcheck):
    """code_of_top27 (k_regen's code pass: one tempered word, integer compares) equals
    draw_code(random()) at both ends of every interval of 2^26 draws it decides; draw_code's
    outcomes are monotone in r, so it equals it on the whole interval.  The intervals next to
    the thresholds 0.25, 0.75 and 0.8 go to the exact f64 path."""
    slow = ctypes.c_int64(0)
    hostcheck.hc_check_code_top27.restype = ctypes.c_int64
    bad = hostcheck.hc_check_code_top27(ctypes.byref(slow))
    assert bad == 0
    assert slow.value == 9


@pytest.mark.parametrize("seed", [0, 7, 2**40 + 3])
def test_odd_generation_words_equal_the_twist(hostcheck, seed):
    """The ring stores its even generations only (tg_core.h MT_STORE): an odd generation's
    word pairs, twisted from the stored generation before it — branch-free (mt_pair, the option
    loops' doubles), with a branch (mt_pair_branchy, tg::Rng) and out of line (mt_pair_ool) —
    equal CPython's generations (init_by_array, then plain twists) at every even position of
    all 16 generations, including word 623 (new words 0 and 396)"""
    hostcheck.hc_check_mt_pair.restype = ctypes.c_int64
    hostcheck.hc_check_mt_pair.argtypes = [ctypes.c_uint64]
    assert hostcheck.hc_check_mt_pair(seed) == 0


def test_lean_draw_code_equals_top27(hostcheck):
    """top27_code / top27_slow (the wave twist's code pass, tg_twist.h: the class from a's top
    two bits plus one compare) equal code_of_top27 on every a they decide, and the slow set
    (a within one of a multiple of 2^25 or of floor(0.8 * 2^27)) covers every CODE_SLOW a"""
    slow = ctypes.c_int64(0)
    hostcheck.hc_check_code_lean.restype = ctypes.c_int64
    bad = hostcheck.hc_check_code_lean(ctypes.byref(slow))
    assert bad == 0
    assert slow.value == 15  # 0, 1; 2^25 k - 1 .. 2^25 k + 1 (k = 1..3); 2^27 - 1; F8 - 1 .. F8 + 1
