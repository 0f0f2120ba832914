"""GPU parity: the gfx950 kernels, called through the C ABI (libtg_amd.so), against the
reference's golden vectors and the CPU oracle.  Bit-exact everywhere: obs compared as f64 bit
patterns, reward / None / done exactly, draw and tick counts exactly."""
import os

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def sm64(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def rec_hash(h, obs, rew, valid, done):
    """vectorised tests/golden/make_golden.py:rec_hash over envs"""
    bits = np.ascontiguousarray(obs).view(np.uint64)
    for k in range(9):
        h = sm64(h ^ bits[:, k])
    w = (rew.astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)) | \
        (valid.astype(np.uint64) << np.uint64(32)) | (done.astype(np.uint64) << np.uint64(40))
    return sm64(h ^ w)


MODES = ["compact", "direct"]


def run_gpu(tg, seed_base, g0, n, steps, a0, policy, autoreset, rows=None, hash_only=False,
            drain_every=0, mode="compact", level_dir=None):
    """Drive a TreasureGameVec like tgo_run drives the oracle; returns env-major arrays.
    drain_every > 0 collects the auto-reset episode records every that many steps."""
    pol = "masked" if policy else "uniform"
    vec = tg.TreasureGameVec(n, seed=seed_base, global_offset=g0, autoreset=autoreset, mode=mode,
                             level_dir=level_dir)
    idx = None if rows is None else torch.as_tensor(rows, device=vec.device)
    pick = (lambda t: t) if idx is None else (lambda t: t.index_select(0, idx))
    obs0 = pick(vec.reset()).cpu().numpy()
    m = obs0.shape[0]
    h = (np.arange(g0, g0 + n, dtype=np.uint64) if rows is None
         else (np.uint64(g0) + np.asarray(rows, dtype=np.uint64)))
    h = rec_hash(h, obs0, np.zeros(m, np.int32), np.zeros(m, np.uint8), np.zeros(m, np.uint8))
    out = None
    if not hash_only:
        out = {"obs": np.zeros((m, steps + 1, 9)), "final_obs": np.zeros((m, steps + 1, 9)),
               "reward": np.zeros((m, steps + 1), np.int32),
               "valid": np.zeros((m, steps + 1), np.uint8),
               "done": np.zeros((m, steps + 1), np.uint8)}
        out["obs"][:, 0] = obs0
        out["final_obs"][:, 0] = obs0
    eps = []
    for t in range(steps):
        a = vec.policy_actions(t, a0, pol)
        o, r, v, d, info = vec.step(a)
        if drain_every and (t + 1) % drain_every == 0:
            eps.append(vec.episodes(cap=n).cpu().numpy())
        fo = info["final_obs"] if autoreset else o
        o, r, v, d, fo = (pick(x).cpu().numpy() for x in (o, r, v, d, fo))
        h = rec_hash(h, fo, r, v, d)
        if out is not None:
            out["obs"][:, t + 1] = o
            out["final_obs"][:, t + 1] = fo
            out["reward"][:, t + 1] = r
            out["valid"][:, t + 1] = v
            out["done"][:, t + 1] = d
    res = out or {}
    res["hash"] = h
    if drain_every:
        eps.append(vec.episodes().cpu().numpy())
        res["episodes"] = np.concatenate(eps)
    res["stats"] = vec.stats()
    res["errors"] = vec.errors()
    res["vec"] = vec
    return res


def assert_bits(a, b, what):
    if a.dtype == np.float64:
        a, b = a.view(np.uint64), b.view(np.uint64)
    bad = np.argwhere(a != b)
    assert len(bad) == 0, "%s differs first at %s (%d cells)" % (what, bad[0].tolist(), len(bad))


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name,policy,autoreset", [("traj_uniform.npz", 0, False),
                                                   ("traj_masked.npz", 1, False),
                                                   ("traj_autoreset.npz", 1, True)])
def test_golden_trajectories(tg, name, policy, autoreset, mode):
    d = golden(name)
    n, t1 = d["valid"].shape
    o = run_gpu(tg, int(d["seed_base"]), 0, n, t1 - 1, int(d["action_seed"]), policy, autoreset,
                mode=mode)
    for k in ("obs", "final_obs", "reward", "valid", "done"):
        assert_bits(o[k], d[k], k)
    st = o["stats"]
    assert st["draws"] == int((d["draws"][:, -1] - 8).sum())  # auto-resets draw in k_step
    assert o["errors"] == 0


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("name,policy", [("hash_uniform.npz", 0), ("hash_masked.npz", 1)])
def test_golden_hashes(tg, name, policy, mode):
    """4,096 envs x 1,000 uniform steps (config C2) and 1,024 x 600 masked, vs the reference."""
    d = golden(name)
    o = run_gpu(tg, 0, 0, len(d["hash"]), int(d["steps"]), int(d["action_seed"]), policy, False,
                hash_only=True, mode=mode)
    np.testing.assert_array_equal(o["hash"], d["hash"])
    st = o["stats"]
    assert st["draws"] == int((d["draws"] - 8).sum())
    assert st["ticks"] == int(d["ticks"].sum())
    assert st["valid_steps"] == int(d["valid_steps"].sum())
    assert st["steps"] == len(d["hash"]) * int(d["steps"])
    # every wavefront's trip count is its longest lane's ticks: 64 x it bounds the lanes' ticks
    assert st["ticks"] <= 64 * st["wave_ticks"] <= 64 * st["ticks"]


@pytest.mark.parametrize("mode", MODES)
def test_full_size_sampled_vs_oracle(tg, oracle, mode):
    """1,048,576 envs (config C3) with auto-reset: 8 blocks of 256 envs spread over the batch
    replayed exactly by the oracle (every env is independent and seeded by its global index)."""
    n, steps, a0 = 1 << 20, 40, 0xC3
    rng = np.random.default_rng(5)
    starts = np.sort(rng.choice(np.arange(0, n - 256, 256), 8, replace=False))
    starts[0], starts[-1] = 0, n - 256
    rows = np.concatenate([np.arange(s, s + 256) for s in starts])
    o = run_gpu(tg, 11, 0, n, steps, a0, 0, True, rows=rows, mode=mode)
    for bi, s in enumerate(starts):
        r = oracle.run(11, int(s), 256, steps, a0, 0, True)
        sl = slice(bi * 256, (bi + 1) * 256)
        for k in ("obs", "final_obs", "reward", "valid", "done"):
            assert_bits(o[k][sl], r[k], "%s block %d" % (k, s))
    assert o["stats"]["steps"] == n * steps
    assert o["errors"] == 0


@pytest.mark.parametrize("mode", MODES)
def test_masked_autoreset_long_vs_oracle(tg, oracle, mode):
    """Many episodes: masked policy, auto-reset, 3,000 steps; episode records == oracle's."""
    n, steps, a0 = 512, 3000, 0x77
    o = run_gpu(tg, 0, 10**6, n, steps, a0, 1, True, hash_only=True, drain_every=250, mode=mode)
    r = oracle.run(0, 10**6, n, steps, a0, 1, True)
    np.testing.assert_array_equal(o["hash"], r["hash"])
    # the episodes the kernel compacted with its ballots == the oracle's (env, return, length)
    eps = o["episodes"]
    exp = []
    for i in range(n):
        ret, ln = 0, 0
        for t in range(1, steps + 1):
            ret += int(r["reward"][i, t])
            ln += 1
            if r["done"][i, t]:
                exp.append((10**6 + i, ret, ln))
                ret, ln = 0, 0
    assert len(exp) > 100
    assert sorted(map(tuple, eps.tolist())) == sorted(exp)
    assert o["stats"]["episodes"] == len(exp)
    assert o["stats"]["episodes_dropped"] == 0


def test_sharding_is_invisible(tg):
    """One 4,096-env batch == two 2,048-env batches at global offsets 0 and 2,048."""
    full = run_gpu(tg, 5, 0, 4096, 200, 9, 1, True, hash_only=True)["hash"]
    a = run_gpu(tg, 5, 0, 2048, 200, 9, 1, True, hash_only=True)["hash"]
    b = run_gpu(tg, 5, 2048, 2048, 200, 9, 1, True, hash_only=True)["hash"]
    np.testing.assert_array_equal(np.concatenate([a, b]), full)


def test_available_mask_matches_oracle(tg, oracle):
    n, a0 = 256, 0x31
    vec = tg.TreasureGameVec(n, seed=3, autoreset=False)
    vec.reset()
    envs = [oracle.OracleEnv(3 + g) for g in range(n)]
    for t in range(60):
        m = vec.available_mask().cpu().numpy().astype(np.uint16)
        exp = np.array([e.mask() for e in envs], np.uint16)
        np.testing.assert_array_equal(m & 0x1FF, exp)
        a = vec.policy_actions(t, a0, "masked").cpu().numpy()
        for g, e in enumerate(envs):
            assert a[g] == oracle.pick_action(a0, g, t, True, int(exp[g]))
            e.step(int(a[g]))
        vec.step(torch.as_tensor(a, device=vec.device))


def test_done_envs_reset_when_autoreset_turns_on(tg, oracle):
    """Envs left done with auto-reset off, then stepped with it on: an env whose option cannot
    run is reset within the step (reward None: k_run's reset-only list since round 4), one
    whose option runs finishes it and resets.  Rows, final rows and the state after equal
    OracleEnv under the same rule (a step that ends done is followed by reset())."""
    n, a0, t1 = 256, 0x5A, 700
    vec = tg.TreasureGameVec(n, seed=11, autoreset=True)  # (allocates the final-obs rows)
    vec.autoreset = False
    vec.reset()
    envs = [oracle.OracleEnv(11 + g) for g in range(n)]
    for t in range(t1 + 1):
        a = vec.policy_actions(t, a0, "masked")
        o, _, _, d, _ = vec.step(a)
        o, d, a = o.cpu().numpy(), d.cpu().numpy(), a.cpu().numpy()
        for g, e in enumerate(envs):
            eo, _, ed, _ = e.step(int(a[g]))
            assert bool(d[g]) == ed and np.array_equal(o[g].view(np.uint64), eo.view(np.uint64)), \
                ("auto-reset off", t, g)
    assert int(d.sum()) >= 3  # envs that enter the auto-reset steps done (5 with these seeds)
    vec.autoreset = True
    for t in range(t1 + 1, t1 + 25):
        a = vec.policy_actions(t, a0, "masked")
        o, r, v, d, info = vec.step(a)
        o, r, v, d, fo = (x.cpu().numpy() for x in (o, r, v, d, info["final_obs"]))
        a = a.cpu().numpy()
        for g, e in enumerate(envs):
            eo, er, ed, _ = e.step(int(a[g]))
            where = ("auto-reset on", t, g, int(a[g]), er, ed)
            assert np.array_equal(fo[g].view(np.uint64), eo.view(np.uint64)), where
            assert (bool(v[g]), bool(d[g])) == (er is not None, ed), where
            assert er is None or int(r[g]) == er, where
            if ed:
                eo = e.reset()
            assert np.array_equal(o[g].view(np.uint64), eo.view(np.uint64)), where
    assert vec.errors() == 0


def test_dropin_single_env(tg, oracle):
    """TreasureGame(seed=s) == random.seed(s); TreasureGame() of the reference, with the
    reference's Python types (TG/:91-96): list of floats, int or None, bool, {}."""
    for seed in (0, 1, 2**33 + 1):
        env = tg.TreasureGame(seed=seed)
        ref = oracle.OracleEnv(seed)
        s = env.reset()
        assert isinstance(s, list) and len(s) == 9 and all(type(v) is float for v in s)
        np.testing.assert_array_equal(np.array(s).view(np.uint64), ref.obs.view(np.uint64))
        for t in range(300):
            mask = env.available_mask
            assert mask.tolist() == [(ref.mask() >> k) & 1 for k in range(9)]
            a = oracle.pick_action(0xD1, seed, t, True, ref.mask())
            if t % 7 == 3:
                a = a - 9  # negative indices wrap like option_list[a]
            st, r, d, info = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert type(st) is list and info == {} and type(d) is bool
            assert r is None or type(r) is int
            np.testing.assert_array_equal(np.array(st).view(np.uint64), rs.view(np.uint64))
            assert (r, d) == (rr, rd)
        with pytest.raises(IndexError):
            env.step(9)
        with pytest.raises(IndexError):
            env.step(-10)
        with pytest.raises(TypeError):
            env.step(1.0)
        env.close()


def test_step_before_reset_is_the_constructed_state(tg):
    """tg_create == TreasureGame.__init__ (4 draws): reset() then equals a 2nd build."""
    vec = tg.TreasureGameVec(64, seed=0)
    o1 = vec.observe().clone()
    o2 = vec.reset().clone()
    d = golden("resets.npz")
    np.testing.assert_array_equal(o2.cpu().numpy().view(np.uint64), d["obs"][:64].view(np.uint64))
    assert not torch.equal(o1, o2)


@pytest.mark.parametrize("mode", MODES)
def test_bad_action_flags_error(tg, mode):
    vec = tg.TreasureGameVec(128, seed=0, mode=mode)
    vec.reset()
    a = torch.zeros(128, dtype=torch.int32, device=vec.device)
    a[17] = 42
    o, r, v, d, _ = vec.step(a)
    assert int(v[17]) == 0
    assert vec.errors() & tg._lib.TG_ERR_ACTION


def test_reset_mask(tg, oracle):
    vec = tg.TreasureGameVec(32, seed=0)
    vec.reset()
    for t in range(20):
        vec.step(vec.policy_actions(t, 1, "masked"))
    before = vec.observe().clone()
    mask = torch.zeros(32, dtype=torch.uint8, device=vec.device)
    mask[::3] = 1
    after = vec.reset(mask).clone()
    keep = mask.cpu().numpy() == 0
    np.testing.assert_array_equal(after.cpu().numpy()[keep], before.cpu().numpy()[keep])
    for g in np.flatnonzero(~keep):
        e = oracle.OracleEnv(g)
        for t in range(20):
            e.step(oracle.pick_action(1, g, t, True, e.mask()))
        np.testing.assert_array_equal(after[g].cpu().numpy().view(np.uint64),
                                      e.reset().view(np.uint64))


def test_modes_identical_full_outputs(tg):
    """compact and direct modes write identical rows for every env, incl. invalid steps."""
    n = 1 << 16
    outs = []
    for mode in MODES:
        vec = tg.TreasureGameVec(n, seed=2, autoreset=True, mode=mode)
        vec.reset()
        acc = []
        for t in range(30):
            o, r, v, d, info = vec.step(vec.policy_actions(t, 0x44, "uniform"))
            acc.append(torch.cat([o.view(torch.int64).flatten(), r.to(torch.int64), v.to(torch.int64),
                                  d.to(torch.int64), info["final_obs"].view(torch.int64).flatten()]).cpu())
        outs.append((torch.stack(acc), vec.stats()))
    assert torch.equal(outs[0][0], outs[1][0])
    for k in ("steps", "valid_steps", "ticks", "draws", "episodes"):
        assert outs[0][1][k] == outs[1][1][k], k


CORRIDOR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels", "corridor")


@pytest.mark.parametrize("level,n,steps", [(None, 1 << 16, 80), (None, 192, 80), (None, 1000, 64),
                                             ("corridor", 192, 40)])
def test_deferred_regeneration_is_invisible(tg, level, n, steps):
    """k_regen drains the listed stale MT halves every 16 compact steps; when it runs must not
    matter.  The same batch stepped with the automatic drains only, and with tg_regenerate
    after every step, gives identical rows, states, MT generations and counters.  Masked
    policy (an option every step, ~37 draws per env-step), and the corridor level (~650 draws
    per go step: lanes reach still-stale halves and regenerate them themselves)."""
    ld = None if level is None else CORRIDOR
    sides = []
    for eager in (False, True):
        vec = tg.TreasureGameVec(n, seed=6, autoreset=True, level_dir=ld)
        vec.reset()
        acc = []
        for t in range(steps):
            o, r, v, d, info = vec.step(vec.policy_actions(t, 0x77, "masked"))
            acc.append(torch.cat([o.view(torch.int64).flatten(), r.to(torch.int64), v.to(torch.int64),
                                  d.to(torch.int64), info["final_obs"].view(torch.int64).flatten()]).cpu())
            if eager:
                vec.regenerate()
        vec.regenerate()
        torch.cuda.synchronize()
        sides.append((torch.stack(acc), vec.read_state(mt=True), vec.stats(), vec.errors()))
        vec.close()
    (a, sa, ta, ea), (b, sb, tb, eb) = sides
    assert torch.equal(a, b)
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    for k in ("steps", "valid_steps", "ticks", "draws", "episodes"):
        assert ta[k] == tb[k], k
    # every half left stale is regenerated exactly once, by k_regen or by its lane: the counts
    # agree unless a drain skipped listed halves (a k_regen grid below 8 workgroups
    # left the regions of the missing XCD counters to the lanes) or regenerated one twice (round
    # 4 on the corridor, whose lanes reach still-stale halves and get listed again: 20,320 vs
    # 15,360 halves, until k_regen claimed each entry's half with an atomic AND).  The corridor's
    # lanes also flag errors (ea, equal on both sides)
    assert ta["regens"] == tb["regens"]
    assert tb["regen_launches"] >= steps and ta["regen_launches"] <= steps // 16 + 1
    assert ea == eb == (0 if level is None else ea)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("policy,autoreset", [(0, False), (1, True)])
def test_corridor_multi_generation_steps(tg, oracle, mode, policy, autoreset):
    """~650 draws per go step: the LDS ring crosses two MT generations inside one launch and
    must regenerate the second one itself (RngRing::fetch -> regen_half), and the wave refills
    the rest after the launch (wave_refill).  Bit-exact vs the oracle on the same level."""
    n, steps, a0 = 192, 40, 0xC0FFEE
    g = run_gpu(tg, 3, 0, n, steps, a0, policy, autoreset, mode=mode, level_dir=CORRIDOR)
    r = oracle.run(3, 0, n, steps, a0, policy, autoreset, level_dir=CORRIDOR)
    for k in ("obs", "final_obs", "reward", "valid", "done"):
        x, y = g[k], r[k]
        if x.dtype == np.float64:
            x, y = x.view(np.uint64), y.view(np.uint64)
        np.testing.assert_array_equal(x, y, err_msg=k)
    np.testing.assert_array_equal(g["hash"], r["hash"])
    assert g["stats"]["draws"] == int(r["draws"].sum()) - 8 * n  # minus construct + reset
    assert r["draws"].max() > 624 * 4
    assert g["errors"] == 0


@pytest.mark.parametrize("mode", MODES)
def test_every_env_hash_vs_oracle(tg, oracle, mode):
    """Every env of a 262,144-env batch (40 steps, auto-reset) against the oracle, twice in the
    default mode: the ring's hand-placed waits must hold for every lane under full load, not
    only for a sample (a race shows up as a handful of envs per million, different per run)."""
    n, steps, a0 = 1 << 18, 40, 0xC3
    r = oracle.run(11, 0, n, steps, a0, 0, True, full=False)
    for rep in range(2 if mode == "compact" else 1):
        g = run_gpu(tg, 11, 0, n, steps, a0, 0, True, hash_only=True, mode=mode)
        bad = np.flatnonzero(g["hash"] != r["hash"])
        assert len(bad) == 0, "run %d: %d envs differ, first %s" % (rep, len(bad), bad[:8].tolist())


@pytest.mark.parametrize("mode", MODES)
def test_checkpoint_restore_continues_bit_exact(tg, oracle, tmp_path, mode):
    """read_state(mt=True) -> write_state into another batch (other seed): both continue
    identically, and equal the oracle's uninterrupted run (masked policy, auto-reset)."""
    n, t0, t1, a0 = 2048, 30, 45, 0xC4EC
    a = tg.TreasureGameVec(n, seed=0, autoreset=True, mode=mode)
    a.reset()
    for t in range(t0):
        a.step(a.policy_actions(t, a0, "masked"))
    snap = a.read_state(mt=True)
    path = str(tmp_path / "ckpt.npz")
    a.save(path)
    b = tg.TreasureGameVec(n, seed=987654, autoreset=True, mode=mode)
    b.load(path)
    ref = oracle.run(0, 0, n, t0 + t1, a0, 1, True)
    for t in range(t0, t0 + t1):
        oa, ra, va, da, _ = a.step(a.policy_actions(t, a0, "masked"))
        ob, rb, vb, db, _ = b.step(b.policy_actions(t, a0, "masked"))
        got = ob.cpu().numpy()
        assert np.array_equal(oa.cpu().numpy().view(np.uint64), got.view(np.uint64))
        assert np.array_equal(got.view(np.uint64), ref["obs"][:, t + 1].view(np.uint64)), t
        assert torch.equal(ra, rb) and torch.equal(va, vb) and torch.equal(da, db)
        assert np.array_equal(rb.cpu().numpy(), ref["reward"][:, t + 1])
    sa, sb = a.read_state(mt=True), b.read_state(mt=True)
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    assert a.errors() == 0 and b.errors() == 0
    # the snapshot's RNG part is CPython's getstate(): Python's random accepts it as a state
    import random
    r = random.Random()
    r.setstate((3, tuple(int(w) for w in snap["mt"][5]) + (int(snap["mt_pos"][5]),), None))
    assert 0.0 <= r.random() < 1.0
    bad = dict(snap)
    bad["mt_pos"] = snap["mt_pos"].copy()
    bad["mt_pos"][3] |= 1
    with pytest.raises(tg.TgError):
        b.write_state(bad)
    a.close()
    b.close()


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_rollout_equals_step_loop_and_oracle(tg, oracle, mode, policy):
    """tg_rollout (the on-device policy inside the step kernels, K steps per call, continued
    across calls) == the per-step API loop == the oracle, bit for bit."""
    n, k1, k, a0 = 4096, 20, 37, 0xF00D
    pol = 1 if policy == "masked" else 0
    a = tg.TreasureGameVec(n, seed=0, autoreset=True, mode=mode)
    a.reset()
    r1 = a.rollout(k1, t0=0, action_seed=a0, policy=policy)
    r2 = a.rollout(k - k1, t0=k1, action_seed=a0, policy=policy)
    ref = oracle.run(0, 0, n, k, a0, pol, True)
    obs = torch.cat([r1["obs"], r2["obs"]]).cpu().numpy().transpose(1, 0, 2)
    assert np.array_equal(np.ascontiguousarray(obs).view(np.uint64), ref["obs"][:, 1:].view(np.uint64))
    for key in ("reward", "valid", "done"):
        got = torch.cat([r1[key], r2[key]]).cpu().numpy().T
        assert np.array_equal(got, ref[key][:, 1:]), key
    b = tg.TreasureGameVec(n, seed=0, autoreset=True, mode=mode)
    b.reset()
    for t in range(k):
        act = b.policy_actions(t, a0, policy)
        want = (r1 if t < k1 else r2)["actions"][t if t < k1 else t - k1]
        assert torch.equal(act, want), t
        b.step(act)
    sa, sb = a.read_state(mt=True), b.read_state(mt=True)
    for key in sa:
        assert np.array_equal(sa[key], sb[key]), key
    assert a.stats()["steps"] == n * k and a.errors() == 0
    r0 = a.rollout(0)
    assert r0["reward"].shape == (0, n)
    a.close()
    b.close()


LEVELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels")


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("level", ["corridor", "gen1", "gen2", "gen3", "exit", "cascade"])
@pytest.mark.parametrize("policy", ["uniform", "masked"])
def test_reference_levels(tg, level, policy, mode):
    """F6: the kernels on other levels vs the REFERENCE's trajectories on them (the reference
    constructor pointed at tests/golden/levels/<level>, tests/golden/make_golden.py)."""
    d = golden("traj_level_%s_%s.npz" % (level, policy))
    n, t1 = d["valid"].shape
    o = run_gpu(tg, int(d["seed_base"]), 0, n, t1 - 1, int(d["action_seed"]), int(d["masked"]),
                bool(d["autoreset"]), mode=mode, level_dir=os.path.join(LEVELS, level))
    for k in ("obs", "final_obs", "reward", "valid", "done"):
        assert_bits(o[k], d[k], k)
    assert o["stats"]["draws"] == int((d["draws"][:, -1] - 8).sum())
    assert o["errors"] == 0


@pytest.mark.parametrize("level", [None, "corridor", "gen1", "exit"])
def test_device_predicates(tg, oracle, level):
    """The six predicates as the DEVICE computes them (mul24 / div48 take their __umul24 path
    only in the device build) at every pixel of the F2 box, all 8 door states, vs the oracle's
    pixel loops; the default level's all-open / all-closed tables vs the reference (F2)."""
    d = golden("predicates.npz")
    x0, x1, y0, y1 = (int(v) for v in d["box"])
    ld = os.path.join(LEVELS, level) if level else None
    vec = tg.TreasureGameVec(1, seed=0, level_dir=ld)
    e = oracle.OracleEnv(0, level_dir=ld)
    for db in range(8):
        got = vec.predicate_table(x0, x1, y0, y1, db).cpu().numpy()
        np.testing.assert_array_equal(got, e.predicate_table(x0, x1, y0, y1, db), err_msg=str(db))
        if level is None and db in (0, 7):
            np.testing.assert_array_equal(got, d["table"][0 if db == 0 else 1])
    vec.close()


def test_all_golden_resets(tg):
    """F5: all 10,000 construct + reset states (seeds 0..9999) on the device, bit for bit
    (gauss's log/cos/sin: OCML here, glibc in the reference)."""
    d = golden("resets.npz")
    n = len(d["obs"])
    vec = tg.TreasureGameVec(n, seed=0)
    obs = vec.reset().cpu().numpy()
    assert_bits(obs, d["obs"], "reset obs")
    np.testing.assert_array_equal(vec.read_state()["pos"], d["pos"])
    assert vec.errors() == 0
    vec.close()


def test_episode_queue_full_without_drain(tg, oracle):
    """An undrained queue never overflows: records beyond its capacity are dropped and
    counted, the count stays at the capacity, the kept records are real episodes."""
    n, steps, a0, cap = 256, 1500, 0x77, 16
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True)
    vec.set_episode_capacity(cap)
    vec.reset()
    for t in range(steps):
        vec.step(vec.policy_actions(t, a0, "masked"))
    st = vec.stats()
    assert st["episodes"] > cap
    assert st["episodes_dropped"] == st["episodes"] - cap
    eps = vec.episodes().cpu().numpy()
    assert len(eps) == cap
    assert len(vec.episodes()) == 0
    r = oracle.run(0, 0, n, steps, a0, 1, True)
    exp = set()
    for i in range(n):
        ret = ln = 0
        for t in range(1, steps + 1):
            ret += int(r["reward"][i, t])
            ln += 1
            if r["done"][i, t]:
                exp.add((i, ret, ln))
                ret = ln = 0
    assert set(map(tuple, eps.tolist())) <= exp
    with pytest.raises(ValueError):
        vec.drain_episodes(torch.empty((4, 2), dtype=torch.int32, device=vec.device),
                           torch.zeros(1, dtype=torch.int32, device=vec.device))
    with pytest.raises(ValueError):
        vec.drain_episodes(torch.empty((4, 2), dtype=torch.int64, device=vec.device),
                           torch.zeros(1, dtype=torch.int64, device=vec.device))
    with pytest.raises(tg.TgError):
        vec.set_episode_capacity(0)
    vec.close()


def test_checkpoint_full_size_round_trip(tg):
    """read_state(mt=True) at config C3 (1,048,576 envs): the MT generations are gathered on
    the device (no per-env copies); save -> load into another batch -> identical state and
    identical next steps."""
    import time
    n = 1 << 20
    a = tg.TreasureGameVec(n, seed=0, autoreset=True)
    a.reset()
    for t in range(3):
        a.step(a.policy_actions(t, 0x31, "masked"))
    t0 = time.time()
    snap = a.read_state(mt=True)
    dt = time.time() - t0
    assert dt < 30, dt
    b = tg.TreasureGameVec(n, seed=12345, autoreset=True)
    b.write_state(snap)
    sb = b.read_state(mt=True)
    for k in snap:
        assert np.array_equal(snap[k], sb[k]), k
    for t in range(3, 5):
        oa = a.step(a.policy_actions(t, 0x31, "masked"))[0].clone()
        ob = b.step(b.policy_actions(t, 0x31, "masked"))[0]
        assert torch.equal(oa.view(torch.int64), ob.view(torch.int64))
    a.close()
    b.close()


def test_seed_limits(tg):
    with pytest.raises(ValueError):
        tg.TreasureGameVec(4, seed=-1)
    with pytest.raises(ValueError):
        tg.TreasureGameVec(4, seed=2**64 - 2)
    env = tg.TreasureGame(seed=-7)  # random.seed(-7) == random.seed(7)
    ref = tg.TreasureGame(seed=7)
    assert env.reset() == ref.reset()
    env.close()
    ref.close()


def test_option_objects_drive_the_gpu_env(tg, oracle):
    """TreasureGame.option_list holds option objects (create_options, IM/:484-498): can_run()
    and run() (-> int | None, OP/:20-36) drive the device env like the reference's demo loop
    (IM/:515-518); the env's state then equals the oracle's."""
    env = tg.TreasureGame(seed=11)
    ref = oracle.OracleEnv(11)
    env.reset()
    assert [o.name for o in env.option_list] == tg.OPTION_NAMES
    for t in range(150):
        can = [o.can_run() for o in env.option_list]
        assert can == [bool(ref.mask() >> k & 1) for k in range(9)]
        a = oracle.pick_action(0xAB, 11, t, t % 3 != 0, ref.mask())
        r = env.option_list[a].run()
        _, rr, _, _ = ref.step(a)
        assert r == rr
        got = env._vec.observe().cpu().numpy()[0]
        np.testing.assert_array_equal(got.view(np.uint64), ref.obs.view(np.uint64))
    env.close()


def test_vector_env_gymnasium_surface(tg, oracle):
    """TreasureGameVectorEnv: (obs, reward, terminated, truncated, info) with same-step
    auto-reset and a TimeLimit, vs the oracle driven the same way (reset after done or after
    max_episode_steps steps of an episode)."""
    n, steps, a0, tmax = 48, 400, 0x3C, 60
    ve = tg.make_vec("treasure_game-v0", num_envs=n, seed=5, max_episode_steps=tmax)
    assert ve.single_action_space.n == 9 and ve.single_observation_space.shape == (9,)
    assert ve.observation_space.shape == (n, 9)
    obs, info = ve.reset()
    envs = [oracle.OracleEnv(5 + g) for g in range(n)]
    lens = [0] * n
    np.testing.assert_array_equal(obs.cpu().numpy().view(np.uint64),
                                  np.stack([e.obs for e in envs]).view(np.uint64))
    n_term = n_trunc = 0
    for t in range(steps):
        acts = [oracle.pick_action(a0, g, t, True, envs[g].mask()) for g in range(n)]
        obs, rew, term, trunc, info = ve.step(torch.tensor(acts, dtype=torch.int32,
                                                           device=ve.device))
        obs, rew, term, trunc = (x.cpu().numpy() for x in (obs, rew, term, trunc))
        fin, val = info["final_obs"].cpu().numpy(), info["valid"].cpu().numpy()
        for g, e in enumerate(envs):
            o, r, d, _ = e.step(acts[g])
            lens[g] += 1
            np.testing.assert_array_equal(fin[g].view(np.uint64), o.view(np.uint64))
            assert (rew[g], bool(val[g]), bool(term[g])) == (float(r or 0), r is not None, d)
            tr = (not d) and lens[g] >= tmax
            assert bool(trunc[g]) == tr
            if d or tr:
                o = e.reset()
                lens[g] = 0
            np.testing.assert_array_equal(obs[g].view(np.uint64), o.view(np.uint64))
        n_term += int(term.sum())
        n_trunc += int(trunc.sum())
    assert n_trunc > 0
    ve.close()


def test_vector_env_outputs_are_not_overwritten(tg):
    """A gymnasium loop keeps obs_t while it steps to obs_t+1: the vector env's outputs (obs,
    info['final_obs'], info['valid'], reward, flags) are the caller's own tensors, not the
    library's buffers that the next step rewrites."""
    ve = tg.make_vec("treasure_game-v0", num_envs=256, seed=3)
    obs0, _ = ve.reset()
    keep0 = obs0.clone()
    obs1, r1, te1, tr1, info1 = ve.step(ve.env.policy_actions(0, policy="masked").clone())
    keep1 = [x.clone() for x in (obs1, r1, info1["final_obs"], info1["valid"])]
    for t in range(1, 6):
        ve.step(ve.env.policy_actions(t, policy="masked").clone())
    assert torch.equal(obs0, keep0)
    for x, k in zip((obs1, r1, info1["final_obs"], info1["valid"]), keep1):
        assert torch.equal(x, k)
    assert not torch.equal(obs0, obs1)  # the step moved something
    ve.close()


@pytest.mark.parametrize("make", ["default", "make", "explicit"])
def test_dropin_shares_the_global_random_stream(tg, make):
    """TreasureGame() -- the default, as gym.make('treasure_game-v0') builds it -- draws from
    Python's global random like the reference's module-level calls (IM/:2, OB/:9): after
    random.seed(s), construction, reset, step and the user's own draws between steps
    interleave on ONE stream, draw for draw.  The user's draws include single 32-bit words
    (randrange, getrandbits(32): the index goes odd) and a lone gauss (gauss_next stays
    cached; the reference's next reset consumes it as its first gauss).  The reference side
    is oracle/pyref.py's Env over one Random(s) that the "user" draws from too."""
    import random
    import pyref  # test infrastructure (oracle/), on sys.path via conftest
    seed = 2024
    saved = random.getstate()
    try:
        random.seed(seed)
        env = {"default": lambda: tg.TreasureGame(),
               "make": lambda: tg.make("treasure_game-v0"),
               "explicit": lambda: tg.TreasureGame(share_global_random=True)}[make]()
        ref = pyref.Env(seed)
        assert env.reset() == ref.reset()
        u = random.Random(7)
        resets = 0
        for t in range(400):
            a = u.randrange(9)
            k = t % 10
            if k == 1:
                assert random.random() == ref.rng.random()
            elif k == 3:
                assert random.randrange(1000) == ref.rng.randrange(1000)
            elif k == 5:
                assert random.gauss(0, 1) == ref.rng.gauss(0, 1)
            elif k == 7:
                assert random.getrandbits(32) == ref.rng.getrandbits(32)
            st, r, d, _ = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert (st, r, d) == (list(rs), rr, rd), t
            if d or t % 40 == 6:  # some resets right after a lone gauss (gauss_next cached)
                assert env.reset() == ref.reset()
                resets += 1
            assert random.getstate() == ref.rng.getstate(), t
        assert resets >= 10
        mask = ref.available_mask()
        for k in range(9):
            assert env.option_list[k].can_run() == bool(mask[k])
        run = [k for k in range(9) if env.option_list[k].can_run()][0]
        assert env.option_list[run].run() == ref.step(run)[1]
        assert random.getstate() == ref.rng.getstate()
        assert env._vec.errors() == 0
        env.close()
    finally:
        random.setstate(saved)


def test_dropin_with_seed_leaves_the_global_stream_alone(tg, oracle):
    """TreasureGame(seed=s) is the private-stream env (random.seed(s); TreasureGame() in a
    fresh reference process) and never touches Python's global random."""
    import random
    random.seed(99)
    before = random.getstate()
    env = tg.TreasureGame(seed=5)
    ref = oracle.OracleEnv(5)
    assert np.array_equal(np.array(env.reset()).view(np.uint64), ref.obs.view(np.uint64))
    for t in range(50):
        a = t % 9
        st, r, d, _ = env.step(a)
        rs, rr, rd, _ = ref.step(a)
        assert np.array_equal(np.array(st).view(np.uint64), rs.view(np.uint64)) and (r, d) == (rr, rd)
    assert random.getstate() == before
    env.close()


def test_step1_rejects_batches_and_bad_outputs(tg):
    """tg_step1 is the 1-env drop-in's call: a batch handle or a null output is an error"""
    import ctypes
    from gym_treasure_game_amd import _lib
    v = tg.TreasureGameVec(2, seed=0)
    obs = np.zeros(9)
    r, va, d = ctypes.c_int32(), ctypes.c_uint8(), ctypes.c_uint8()
    with pytest.raises(tg.TgError):
        _lib.check(v._L.tg_step1(v.handle, 0, obs.ctypes.data, ctypes.byref(r), ctypes.byref(va),
                                 ctypes.byref(d), None), "tg_step1")
    v.close()
    one = tg.TreasureGameVec(1, seed=0)
    with pytest.raises(tg.TgError):
        _lib.check(one._L.tg_step1(one.handle, 0, None, ctypes.byref(r), ctypes.byref(va),
                                   ctypes.byref(d), None), "tg_step1")
    one.close()
