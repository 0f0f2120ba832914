"""tg_rollout (K steps per call, the synthetic policy evaluated inside k_classify: no action
launch, no host round trip) against K x (tg_policy_actions + tg_step), bit for bit: every
output row, the final env states and MT streams, and the completed episodes.  Ragged batch
sizes up to the bench's 1M envs, levels whose options cross MT generations inside one step,
rollouts split over several calls, and batches that enter the rollout with stale MT halves
left by tg_step.  (Round 2's one-launch TG_MODE_ASYNC rollout, slower, was removed in round 3:
DESIGN.md §9.1.)"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LEVELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels")


def episodes_sorted(vec):
    e = vec.episodes(cap=vec.num_envs * 64).cpu().numpy()
    return e[np.lexsort((e[:, 2], e[:, 1], e[:, 0]))] if len(e) else e


def run_pair(tg, n, k, policy, pre_steps=0, level=None, seed=5, a0=0xA5A5, chunks=(None,),
             groups=1, stagger=False, post_steps=0, mode="compact"):
    """the same batch through K x (tg_policy_actions + tg_step) and through tg_rollout (in
    `chunks` calls, in step mode `mode`); returns both sides' outputs, final states and sorted
    episodes"""
    ld = None if level is None else os.path.join(LEVELS, level)
    sides = []
    for side in ("steps", "rollout"):
        v = tg.TreasureGameVec(n, seed=seed, autoreset=True, level_dir=ld)
        v.reset()
        for t in range(pre_steps):  # leaves stale MT halves for the rollout to start from
            v.step(v.policy_actions(t, a0, policy))
        outs = []
        if side == "steps":
            for t in range(pre_steps, pre_steps + k):
                act = v.policy_actions(t, a0, policy).clone()
                o, r, va, d, _ = v.step(act)
                outs.append({"obs": o.clone(), "reward": r.clone(), "valid": va.clone(),
                             "done": d.clone(), "actions": act})
            out = {key: torch.stack([x[key] for x in outs]) for key in outs[0]}
        else:
            v.set_mode(mode)
            if groups > 1:
                v.set_groups(groups, stagger)
            t0, parts = pre_steps, []
            sizes = [k] if chunks == (None,) else list(chunks)
            assert sum(sizes) == k
            for c in sizes:
                parts.append(v.rollout(c, t0=t0, action_seed=a0, policy=policy))
                t0 += c
            out = {key: torch.cat([p[key] for p in parts]) for key in parts[0]}
        # the per-step API afterwards (the grouped steppers' lists were drained)
        for t in range(pre_steps + k, pre_steps + k + post_steps):
            v.step(v.policy_actions(t, a0, policy))
        torch.cuda.synchronize()
        sides.append((out, v.read_state(mt=True), episodes_sorted(v), v.stats(), v.errors()))
        v.close()
    return sides


def check_pair(sides, n, k, errors=0):
    (oa, sa, ea, sta, era), (ob, sb, eb, stb, erb) = sides
    assert era == errors and erb == errors
    for key in ("reward", "valid", "done", "actions"):
        assert torch.equal(oa[key], ob[key]), key
    assert torch.equal(oa["obs"].view(torch.int64), ob["obs"].view(torch.int64)), "obs"
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    assert np.array_equal(ea, eb)
    assert stb["steps"] >= n * k
    for key in ("valid_steps", "ticks", "draws", "episodes"):
        assert sta[key] == stb[key], key


@pytest.mark.parametrize("n", [1, 63, 64, 1000, 70001])
def test_rollout_ragged_batches(tg, n):
    """batches that leave a partial wave / workgroup; rollouts in 3 calls"""
    k = 21
    check_pair(run_pair(tg, n, k, "uniform", chunks=(7, 1, 13)), n, k)


def test_rollout_after_steps(tg):
    """envs enter the rollout with MT_STALE halves left by tg_step"""
    n, k = 50000, 30
    check_pair(run_pair(tg, n, k, "masked", pre_steps=9), n, k)


@pytest.mark.parametrize("level", ["corridor", "gen2", "exit", "cascade"])
def test_rollout_levels(tg, level):
    """corridor: go options of ~650 draws (two MT generation crossings inside one step).  Some
    of its envs get stuck against an end wall in an option that never ends (the reference
    would loop forever; the kernels stop at TICK_CAP and flag E_TICKCAP): both sides must
    flag exactly that, with identical outputs"""
    n, k = 4096, 25
    check_pair(run_pair(tg, n, k, "uniform", level=level), n, k,
               errors=(1 << 24) if level == "corridor" else 0)


def test_rollout_no_obs_and_no_autoreset(tg):
    """obs=None (the scratch row) and auto-reset off, against the per-step API"""
    n, k, a0 = 20000, 20, 77
    res = []
    for side in ("steps", "rollout"):
        v = tg.TreasureGameVec(n, seed=9, autoreset=False)
        v.reset()
        if side == "steps":
            outs = []
            for t in range(k):
                act = v.policy_actions(t, a0, "uniform").clone()
                _, rw, va, d, _ = v.step(act)
                outs.append({"reward": rw.clone(), "valid": va.clone(), "done": d.clone(),
                             "actions": act})
            r = {key: torch.stack([x[key] for x in outs]) for key in outs[0]}
        else:
            r = v.rollout(k, t0=0, action_seed=a0, policy="uniform", obs=False)
        res.append((r, v.read_state(mt=True), v.observe().clone()))
        v.close()
    (ra, sa, oa), (rb, sb, ob) = res
    for key in ("reward", "valid", "done", "actions"):
        assert torch.equal(ra[key], rb[key]), key
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    assert torch.equal(oa.view(torch.int64), ob.view(torch.int64))


@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_rollout_1m_envs(tg, policy):
    """the bench's size: 1M envs"""
    n, k = 1 << 20, 24
    check_pair(run_pair(tg, n, k, policy), n, k)


@pytest.mark.parametrize("n,groups,stagger,policy", [(20000, 3, True, "masked"),
                                                     (70001, 2, False, "uniform"),
                                                     (1 << 20, 2, True, "uniform"),
                                                     (1 << 20, 4, True, "masked")])
def test_grouped_rollout(tg, n, groups, stagger, policy):
    """tg_set_groups: the batch stepped as contiguous groups on their own streams (forked from and
    joined to the caller's) equals the per-step API: every output row, states, MT streams,
    episodes and counters; rollouts over several calls, envs entering with stale MT halves,
    and per-step calls after the grouped rollouts"""
    k = 30
    check_pair(run_pair(tg, n, k, policy, pre_steps=5, chunks=(10, 3, 17), groups=groups,
                        stagger=stagger, post_steps=6), n, k)


@pytest.mark.parametrize("level", ["corridor", "cascade"])
def test_grouped_rollout_levels(tg, level):
    """groups on levels whose go options cross MT generations inside one step (corridor) and
    whose INTERACT ticks draw 10 times (cascade)"""
    n, k = 12288, 25
    check_pair(run_pair(tg, n, k, "uniform", level=level, groups=3, stagger=True), n, k,
               errors=(1 << 24) if level == "corridor" else 0)
