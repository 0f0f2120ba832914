"""TG_MODE_OVERLAP: tg_rollout with each step's classification split in two — the envs not
listed in the previous step (k_classify part 1, in the previous step's k_run launch: k_run_cls)
and the previous step's listed envs (part 2, one lane per worklist entry, after it) — against
K x (tg_policy_actions + tg_step), bit for bit (outputs, states, MT streams, episodes,
counters).  DESIGN.md §9.3."""
import pytest

from test_gpu_rollout import check_pair, run_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 70001])
def test_overlap_ragged_batches(tg, n):
    """partial waves / workgroups; rollouts over 3 calls (each call's first step is whole)"""
    k = 21
    check_pair(run_pair(tg, n, k, "uniform", chunks=(7, 1, 13), mode="overlap"), n, k)


@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_overlap_after_steps_and_before(tg, policy):
    """envs enter with stale MT halves left by tg_step; per-step calls after the rollouts; the
    k_regen of every 16th step inside a rollout"""
    n, k = 50000, 45
    check_pair(run_pair(tg, n, k, policy, pre_steps=9, chunks=(40, 5), post_steps=6,
                        mode="overlap"), n, k)


@pytest.mark.parametrize("level", ["corridor", "gen2", "exit", "cascade"])
def test_overlap_levels(tg, level):
    n, k = 4096, 25
    check_pair(run_pair(tg, n, k, "uniform", level=level, mode="overlap"), n, k,
               errors=(1 << 24) if level == "corridor" else 0)


@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_overlap_1m_envs(tg, policy):
    n, k = 1 << 20, 24
    check_pair(run_pair(tg, n, k, policy, mode="overlap"), n, k)


def test_overlap_no_obs_no_autoreset(tg):
    """obs=None (the shared scratch rows) and auto-reset off"""
    import numpy as np
    import torch
    n, k, a0 = 20000, 20, 77
    res = []
    for mode in ("compact", "overlap"):
        v = tg.TreasureGameVec(n, seed=9, autoreset=False)
        v.reset()
        v.set_mode(mode)
        r = v.rollout(k, t0=0, action_seed=a0, policy="uniform", obs=False)
        res.append((r, v.read_state(mt=True), v.observe().clone()))
        v.close()
    (ra, sa, oa), (rb, sb, ob) = res
    for key in ("reward", "valid", "done", "actions"):
        assert torch.equal(ra[key], rb[key]), key
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    assert torch.equal(oa.view(torch.int64), ob.view(torch.int64))
