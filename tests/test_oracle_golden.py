"""Pin the CPU oracle to the reference: every golden family from tests/golden/make_golden.py.

The fixtures were produced by running the unmodified reference; the oracle
(oracle/tg_oracle.c) must reproduce them bit for bit before it is trusted as the checker.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden

TRAJ = [("traj_uniform.npz", 0, False), ("traj_masked.npz", 1, False),
        ("traj_autoreset.npz", 1, True)]


def test_rng_kat(oracle):
    """CPython MT19937 / random() / uniform / gauss for 11 seeds incl. 2**32 and 2**64-1."""
    kat = json.load(open(os.path.join(GOLDEN, "rng_kat.json")))
    assert len(kat["kats"]) >= 10
    for k in kat["kats"]:
        s = int(k["seed"])
        assert oracle.rng_words(s, len(k["words"])).tolist() == k["words"], s
        assert oracle.rng_random(s, 700).view(np.uint64).tolist() == k["random_bits"], s
        assert oracle.rng_uniform5(s).view(np.uint64).tolist() == k["uniform_bits"], s
        assert oracle.rng_gauss(s, 16).view(np.uint64).tolist() == k["gauss_bits"], s


@pytest.mark.parametrize("name,policy,autoreset", TRAJ)
def test_trajectories(oracle, name, policy, autoreset):
    d = golden(name)
    n, t1 = d["valid"].shape
    out = oracle.run(int(d["seed_base"]), 0, n, t1 - 1, int(d["action_seed"]), policy, autoreset)
    np.testing.assert_array_equal(out["obs"].view(np.uint64), d["obs"].view(np.uint64))
    np.testing.assert_array_equal(out["final_obs"].view(np.uint64), d["final_obs"].view(np.uint64))
    np.testing.assert_array_equal(out["reward"], d["reward"])
    np.testing.assert_array_equal(out["valid"], d["valid"])
    np.testing.assert_array_equal(out["done"], d["done"])
    np.testing.assert_array_equal(out["draws"], d["draws"][:, -1])


@pytest.mark.parametrize("name,policy", [("hash_uniform.npz", 0), ("hash_masked.npz", 1)])
def test_rolling_hashes(oracle, name, policy):
    d = golden(name)
    n = len(d["hash"])
    out = oracle.run(0, 0, n, int(d["steps"]), int(d["action_seed"]), policy, False, full=False)
    np.testing.assert_array_equal(out["hash"], d["hash"])
    np.testing.assert_array_equal(out["draws"], d["draws"])
    np.testing.assert_array_equal(out["ticks"], d["ticks"])


def test_resets(oracle):
    d = golden("resets.npz")
    out = oracle.run(0, 0, len(d["obs"]), 0, 0, 0, False)
    np.testing.assert_array_equal(out["obs"][:, 0].view(np.uint64), d["obs"].view(np.uint64))


def test_predicate_tables(oracle):
    """The oracle's pixel-loop predicates == the reference's at every pixel of the box."""
    d = golden("predicates.npz")
    x0, x1, y0, y1 = (int(v) for v in d["box"])
    e = oracle.OracleEnv(0)
    for k, db in enumerate(d["door_bits"]):
        np.testing.assert_array_equal(e.predicate_table(x0, x1, y0, y1, int(db)), d["table"][k])


def test_golden_coverage():
    """The fixtures exercise the rare branches the survey lists."""
    m = golden("traj_masked.npz")
    a = golden("traj_autoreset.npz")
    u = golden("traj_uniform.npz")
    assert m["done"].sum() > 0 and a["done"].sum() > 0           # gold + return to row 0
    assert (m["internal"][:, :, 5] == 0).any()                    # bolt unlocked (key dropped)
    assert (m["internal"][:, 1:, 2] > 0).any()                    # jump ticker left over
    assert m["internal"][:, :, 1].min() < 0                       # negative playery
    assert (m["internal"][:, :, 3] != m["internal"][:, :1, 3]).any()  # doors toggled
    assert (u["valid"][:, 1:] == 0).mean() > 0.5                  # None rewards dominate
    assert set(np.unique(m["action"][:, 1:])) == set(range(9))    # every option ran


LEVELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels")
LEVEL_TRAJ = [(lv, pol) for lv in ("corridor", "gen1", "gen2", "gen3", "exit", "cascade")
              for pol in ("uniform", "masked")]


def assert_level_traj(out, d):
    for k in ("obs", "final_obs"):
        np.testing.assert_array_equal(out[k].view(np.uint64), d[k].view(np.uint64), err_msg=k)
    for k in ("reward", "valid", "done"):
        np.testing.assert_array_equal(out[k], d[k], err_msg=k)


@pytest.mark.parametrize("level,policy", LEVEL_TRAJ)
def test_level_trajectories(oracle, level, policy):
    """F6: the reference constructor pointed at other level files (tests/golden/levels/*:
    the 42-cell corridor, three generated layouts, a hand-made level that finishes episodes)
    vs the oracle's level loader + physics."""
    d = golden("traj_level_%s_%s.npz" % (level, policy))
    n, t1 = d["valid"].shape
    out = oracle.run(int(d["seed_base"]), 0, n, t1 - 1, int(d["action_seed"]), int(d["masked"]),
                     bool(d["autoreset"]), level_dir=os.path.join(LEVELS, level))
    assert_level_traj(out, d)
    np.testing.assert_array_equal(out["draws"], d["draws"][:, -1])


def test_level_fixture_coverage():
    """The level fixtures exercise multi-generation steps and auto-reset episodes."""
    assert golden("traj_level_corridor_masked.npz")["draws"][:, -1].max() > 624 * 100
    ex = golden("traj_level_exit_masked.npz")
    assert ex["autoreset"] and ex["done"].sum() > 100
