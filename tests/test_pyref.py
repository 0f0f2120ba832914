"""The pure-Python restatement timed as the reference-Python CPU leg of bench.py
(oracle/pyref.py) against the reference's own trajectories (tests/golden/traj_*.npz)."""
import os

import numpy as np
import pytest

from conftest import golden

LEVELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels")


@pytest.mark.parametrize("name,envs,steps,level", [
    ("traj_uniform.npz", 4, 400, None), ("traj_masked.npz", 3, 300, None),
    ("traj_autoreset.npz", 2, 1200, None), ("traj_level_exit_masked.npz", 3, 300, "exit"),
    ("traj_level_gen1_uniform.npz", 3, 300, "gen1")])
def test_pyref_vs_reference(name, envs, steps, level):
    import pyref
    d = golden(name)
    lv = pyref.read_level(os.path.join(LEVELS, level)) if level else None
    for g in range(envs):
        obs, fin, rew, don = pyref.run_env(g, steps, int(d["action_seed"]), bool(d["masked"]),
                                           bool(d["autoreset"]), lv, int(d["seed_base"]))
        np.testing.assert_array_equal(np.array(obs).view(np.uint64),
                                      d["obs"][g, :steps + 1].view(np.uint64))
        np.testing.assert_array_equal(np.array(fin).view(np.uint64),
                                      d["final_obs"][g, :steps + 1].view(np.uint64))
        np.testing.assert_array_equal([r is not None for r in rew[1:]], d["valid"][g, 1:steps + 1])
        np.testing.assert_array_equal([r or 0 for r in rew[1:]], d["reward"][g, 1:steps + 1])
        np.testing.assert_array_equal(don[1:], d["done"][g, 1:steps + 1])


def test_pyref_throughput_runs():
    import pyref
    r = pyref.throughput(0.4, "uniform", 0x5EED0001)
    assert r["value"] > 0 and r["value_1proc"] > 0 and r["procs"] >= 1
