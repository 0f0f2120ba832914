"""TG_MODE_FLOW (tg_flow.h k_flow): tg_rollout's K steps in one launch per 16 steps, each 64-env
chunk classified for step t + 1 as soon as its envs are done with step t, against K x
(tg_policy_actions + tg_step), bit for bit: every output row, the final env states and MT
streams, the completed episodes and the launch counters.  Ragged batches (fewer chunks than
sub-problems, partial chunks), rollouts over several calls and across the 16-step launch bound,
envs entering with stale MT halves, levels whose options cross MT generations inside one step
(corridor: the per-lane regeneration on whichever CU the env's item runs) and whose INTERACT
ticks draw 10 times (cascade), both policies at 1M envs, and the per-step API after flow
rollouts.  Reference: TG/:91-96 (the step each chunk takes), OP/:20-36."""
import numpy as np
import pytest
import torch

from test_gpu_rollout import check_pair, run_pair

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 70001])
def test_flow_ragged_batches(tg, n):
    """fewer chunks than XCD sub-problems (n <= 448), a partial last chunk; 3 calls"""
    k = 21
    check_pair(run_pair(tg, n, k, "uniform", chunks=(7, 1, 13), mode="flow"), n, k)


@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_flow_after_steps_and_long_rollouts(tg, policy):
    """stale MT halves from tg_step; 40 steps in one call (launches of 16 + 16 + 8) and a
    17-step call; the per-step API afterwards"""
    n, k = 50000, 57
    check_pair(run_pair(tg, n, k, policy, pre_steps=9, chunks=(40, 17), mode="flow",
                        post_steps=5), n, k)


@pytest.mark.parametrize("level", ["corridor", "gen2", "exit", "cascade"])
def test_flow_levels(tg, level):
    n, k = 4096, 25
    check_pair(run_pair(tg, n, k, "uniform", level=level, mode="flow"), n, k,
               errors=(1 << 24) if level == "corridor" else 0)


@pytest.mark.parametrize("level", ["corridor", "cascade"])
def test_flow_levels_masked(tg, level):
    n, k = 8192, 32
    check_pair(run_pair(tg, n, k, "masked", level=level, mode="flow"), n, k,
               errors=(1 << 24) if level == "corridor" else 0)


@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_flow_1m_envs(tg, policy):
    """the bench's size"""
    n, k = 1 << 20, 24
    check_pair(run_pair(tg, n, k, policy, mode="flow"), n, k)


def test_flow_no_obs_and_no_autoreset(tg):
    """obs=None (the scratch rows) and auto-reset off, against the per-step API"""
    n, k, a0 = 20000, 20, 77
    res = []
    for side in ("steps", "flow"):
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
            v.set_mode("flow")
            r = v.rollout(k, t0=0, action_seed=a0, policy="uniform", obs=False)
        res.append((r, v.read_state(mt=True), v.observe().clone(), v.errors()))
        v.close()
    (ra, sa, oa, ea), (rb, sb, ob, eb) = res
    assert ea == eb == 0
    for key in ("reward", "valid", "done", "actions"):
        assert torch.equal(ra[key], rb[key]), key
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    assert torch.equal(oa.view(torch.int64), ob.view(torch.int64))


def test_flow_equals_oracle(tg, oracle):
    """4,096 envs x 48 masked auto-reset steps in flow rollouts against the oracle's replay"""
    n, steps, a0 = 4096, 48, 0x3C3C
    v = tg.TreasureGameVec(n, seed=4, autoreset=True)
    v.set_mode("flow")
    obs0 = v.reset().cpu().numpy()
    r = v.rollout(steps, t0=0, action_seed=a0, policy="masked")
    ref = oracle.run(4, 0, n, steps, a0, 1, True)
    assert np.array_equal(obs0.view(np.uint64), ref["obs"][:, 0].view(np.uint64))
    got = r["obs"].cpu().numpy().transpose(1, 0, 2)
    assert np.array_equal(got.view(np.uint64), ref["obs"][:, 1:].view(np.uint64))
    for key in ("reward", "valid", "done"):
        assert np.array_equal(r[key].cpu().numpy().T, ref[key][:, 1:]), key
    assert v.errors() == 0
    v.close()


def test_flow_unstepped_subproblem_is_flagged(tg, monkeypatch):
    """chunks x, x + P, ... are stepped only by waves on XCD x; a launch that leaves
    a sub-problem without waves must not pass silently.  The test hook TG_FLOW_SKIP_PART (read
    at tg_create) makes sub-problem 3's waves leave at once; k_flow_check sets TG_ERR_FLOW and
    rollout() raises"""
    monkeypatch.setenv("TG_FLOW_SKIP_PART", "3")
    v = tg.TreasureGameVec(4096, seed=2, autoreset=True, mode="flow")
    monkeypatch.delenv("TG_FLOW_SKIP_PART")
    v.reset()
    with pytest.raises(tg.TgError, match="TG_ERR_FLOW"):
        v.rollout(4, t0=0, action_seed=5, policy="uniform")
    v.rollout(4, t0=4, action_seed=5, policy="uniform", check_flow=False)
    assert v.errors() & tg.TG_ERR_FLOW
    v.close()
    # a handle created without the hook steps every sub-problem
    w = tg.TreasureGameVec(4096, seed=2, autoreset=True, mode="flow")
    w.reset()
    w.rollout(4, t0=0, action_seed=5, policy="uniform")
    assert w.errors() == 0
    w.close()


def test_flow_rejects_groups(tg):
    """TG_MODE_FLOW steps the whole batch in one k_flow launch; env groups are a
    compact-mode rollout form, so the two are refused together instead of one being ignored"""
    v = tg.TreasureGameVec(8192, seed=1)
    v.set_groups(2)
    with pytest.raises(tg.TgError, match="groups"):
        v.set_mode("flow")
    v.set_groups(1)
    v.set_mode("flow")
    with pytest.raises(tg.TgError, match="groups"):
        v.set_groups(2)
    v.close()
