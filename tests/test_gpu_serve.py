"""The N = 1 drop-in's resident server (k_serve1, tg_set_serve): every call of TreasureGame
through it equals the launch-per-call path and the reference restatements, including the server's
leaving and relaunching (TG_SERVE_IDLE_US), the races around it (a 1 us idle limit: nearly every
call finds the server gone or leaving), sleeps longer than the limit between calls (the next
server reloads the Python stream's generations from the device cache), the user's own draws on
the shared stream (the ring rebuilt from the caller's state) and other calls on the handle in
between (which stop the server)."""
import random
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _shared_run(tg, seed, serve, sleeps, words=True):
    import pyref  # test infrastructure (oracle/), on sys.path via conftest
    saved = random.getstate()
    try:
        random.seed(seed)
        env = tg.TreasureGame()
        env._vec.set_serve(serve)
        if words:  # steps in place on the global Random's words (tg_step1_pywords)
            assert env._pywords is not None
        else:  # steps through a tg_pystate (tg_step1_py), getstate / setstate around each
            env._pywords = None
        ref = pyref.Env(seed)
        assert env.reset() == ref.reset()
        u = random.Random(seed + 1)
        out = []
        for t in range(160):
            a = u.randrange(9)
            if t % 9 == 4:
                assert random.random() == ref.rng.random()
            if t % 13 == 6:
                assert random.gauss(0, 1) == ref.rng.gauss(0, 1)
            if sleeps and t % 17 == 5:
                time.sleep(0.003)
            st, r, d, _ = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert (st, r, d) == (list(rs), rr, rd), (serve, t)
            out.append((st, r, d))
            if d or t % 50 == 11:
                assert env.reset() == ref.reset()
            if t % 31 == 30:  # another call on the handle: stops the server
                assert env.available_mask.tolist() == list(ref.available_mask())
            assert random.getstate() == ref.rng.getstate(), (serve, t)
        assert env._vec.errors() == 0
        env.close()
        return out
    finally:
        random.setstate(saved)


@pytest.mark.parametrize("idle_us", [None, "1"])
def test_serve_shared_stream_matches_launch_path(tg, monkeypatch, idle_us):
    if idle_us:
        monkeypatch.setenv("TG_SERVE_IDLE_US", idle_us)
    on = _shared_run(tg, 31, True, sleeps=True)
    off = _shared_run(tg, 31, False, sleeps=False)
    assert on == off
    assert _shared_run(tg, 31, True, sleeps=False, words=False) == on
    assert _shared_run(tg, 31, False, sleeps=False, words=False) == on


@pytest.mark.parametrize("idle_us", [None, "1"])
def test_serve_private_stream_matches_oracle(tg, oracle, monkeypatch, idle_us):
    if idle_us:
        monkeypatch.setenv("TG_SERVE_IDLE_US", idle_us)
    for serve in (True, False):
        env = tg.TreasureGame(seed=8)
        env._vec.set_serve(serve)
        ref = oracle.OracleEnv(8)
        assert np.array_equal(np.array(env.reset()).view(np.uint64), ref.obs.view(np.uint64))
        for t in range(200):
            a = oracle.pick_action(0xA5, 8, t, True, ref.mask())
            if serve and t % 23 == 7:
                time.sleep(0.002)
            st, r, d, _ = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert np.array_equal(np.array(st).view(np.uint64), rs.view(np.uint64)), (serve, t)
            assert (r, d) == (rr, rd), (serve, t)
            if d:
                s0 = env.reset()
                ref.reset()
                assert np.array_equal(np.array(s0).view(np.uint64), ref.obs.view(np.uint64))
        assert env._vec.errors() == 0
        env.close()


def test_serve_toggle_mid_episode(tg, oracle):
    """tg_set_serve stops a running server; the env continues on either path"""
    env = tg.TreasureGame(seed=3)
    ref = oracle.OracleEnv(3)
    env.reset()
    for t in range(120):
        if t % 10 == 0:
            env._vec.set_serve(t % 20 == 0)
        a = t % 9
        st, r, d, _ = env.step(a)
        rs, rr, rd, _ = ref.step(a)
        assert np.array_equal(np.array(st).view(np.uint64), rs.view(np.uint64)) and (r, d) == (rr, rd), t
    env.close()


def test_process_exits_with_the_server_resident(tmp_path):
    """A process that ends with a server still running (idle limit 1 s, no close(); the env is
    kept alive past interpreter teardown) exits cleanly and promptly: the library stops live
    servers at unload (tg_amd.hip SrvReaper)"""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys, builtins; sys.path.insert(0, %r); import gym_treasure_game_amd as tg\n"
            "env = tg.TreasureGame(seed=1); env.reset()\n"
            "for i in range(50): env.step(i %% 9)\n"
            "builtins._tg_keep = env\n"
            "print('stepped', flush=True)\n" % root)
    env = dict(os.environ, TG_SERVE_IDLE_US="1000000")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "stepped" in r.stdout
    assert time.time() - t0 < 100


def test_mask_first_then_steps(tg, oracle):
    """A server first launched by available_mask (tg_available_mask1) serves the steps after it:
    the call that starts a server must not matter (round 6: the row buffer was allocated only by
    the step calls, and a mask-first server wrote its first step's row through a null pointer)"""
    for serve in (True, False):
        env = tg.TreasureGame(seed=12)
        env._vec.set_serve(serve)
        ref = oracle.OracleEnv(12)
        env.reset()  # (tg_reset: no server yet, so the mask read below launches it)
        assert env.available_mask.tolist() == [(ref.mask() >> k) & 1 for k in range(9)]
        for t in range(40):
            a = oracle.pick_action(0x5A, 12, t, True, ref.mask())
            st, r, d, _ = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert np.array_equal(np.array(st).view(np.uint64), rs.view(np.uint64)) and (r, d) == (rr, rd)
            assert env.available_mask.tolist() == [(ref.mask() >> k) & 1 for k in range(9)]
        env.close()


@pytest.mark.parametrize("idle_us", [None, "1"])
def test_private_resets_through_the_server(tg, oracle, monkeypatch, idle_us):
    """TreasureGame(seed=s).reset() (tg_reset1, SRV_RESET: k_reset's work on the server) between
    steps, with the server and without, against the oracle's resets"""
    if idle_us:
        monkeypatch.setenv("TG_SERVE_IDLE_US", idle_us)
    for serve in (True, False):
        env = tg.TreasureGame(seed=21)
        env._vec.set_serve(serve)
        ref = oracle.OracleEnv(21)
        s0 = env.reset()
        assert np.array_equal(np.array(s0).view(np.uint64), ref.obs.view(np.uint64))
        for t in range(150):
            if t % 17 == 9:
                s0 = env.reset()
                ref.reset()
                assert np.array_equal(np.array(s0).view(np.uint64), ref.obs.view(np.uint64)), (serve, t)
            a = oracle.pick_action(0x3C, 21, t, True, ref.mask())
            st, r, d, _ = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert np.array_equal(np.array(st).view(np.uint64), rs.view(np.uint64)), (serve, t)
            assert (r, d) == (rr, rd), (serve, t)
        assert env._vec.errors() == 0
        env.close()


def test_one_env_calls_reject_bad_arguments(tg):
    """tg_step1_pywords / tg_available_mask1 / tg_reset1 are 1-env calls: a batch handle, a
    null output or an index outside [0, 624] is an error (TgError), not a launch"""
    import ctypes
    from gym_treasure_game_amd import _lib
    L = _lib.load()
    words = (ctypes.c_uint32 * 624)()
    idx = ctypes.c_int32(624)
    obs = np.zeros(9)
    r, va, d, m = ctypes.c_int32(), ctypes.c_uint8(), ctypes.c_uint8(), ctypes.c_uint16()
    v = tg.TreasureGameVec(2, seed=0)
    for call, name in ((lambda h: L.tg_available_mask1(h, ctypes.byref(m), None), "mask1"),
                       (lambda h: L.tg_reset1(h, obs.ctypes.data, None), "reset1"),
                       (lambda h: L.tg_step1_pywords(h, 0, words, ctypes.byref(idx), obs.ctypes.data,
                                                     ctypes.byref(r), ctypes.byref(va),
                                                     ctypes.byref(d), None), "pywords")):
        with pytest.raises(tg.TgError):
            _lib.check(call(v.handle), name)
    v.close()
    one = tg.TreasureGameVec(1, seed=0)
    with pytest.raises(tg.TgError):
        _lib.check(L.tg_available_mask1(one.handle, None, None), "mask1")
    with pytest.raises(tg.TgError):
        _lib.check(L.tg_step1_pywords(one.handle, 0, None, ctypes.byref(idx), obs.ctypes.data,
                                      ctypes.byref(r), ctypes.byref(va), ctypes.byref(d), None),
                   "pywords")
    for bad in (-1, 625):
        idx.value = bad
        with pytest.raises(tg.TgError):
            _lib.check(L.tg_step1_pywords(one.handle, 0, words, ctypes.byref(idx), obs.ctypes.data,
                                          ctypes.byref(r), ctypes.byref(va), ctypes.byref(d), None),
                       "pywords")
    # the handle still steps after the refusals (with and without the server)
    for serve in (True, False):
        _lib.check(L.tg_set_serve(one.handle, int(serve)), "serve")
        _lib.check(L.tg_step1(one.handle, 1, obs.ctypes.data, ctypes.byref(r), ctypes.byref(va),
                              ctypes.byref(d), None), "step1")
        _lib.check(L.tg_available_mask1(one.handle, ctypes.byref(m), None), "mask1")
        assert m.value < 512
    one.close()


@pytest.mark.parametrize("level", ["corridor", "gen1", "exit", "cascade"])
def test_serve_other_levels(tg, oracle, level):
    """The server on the reference's other levels (tests/golden/levels): a level too wide for
    the bitmasks (no Map::mk), GoTables of other sizes (staged in the server's LDS when they
    fit), with and without the server, against the oracle"""
    import os
    ld = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels", level)
    for serve in (True, False):
        env = tg.TreasureGame(seed=7, level_dir=ld)
        env._vec.set_serve(serve)
        ref = oracle.OracleEnv(7, level_dir=ld)
        s0 = env.reset()
        assert np.array_equal(np.array(s0).view(np.uint64), ref.obs.view(np.uint64))
        for t in range(80):
            assert env.available_mask.tolist() == [(ref.mask() >> k) & 1 for k in range(9)], (level, serve, t)
            a = oracle.pick_action(0x77, 7, t, True, ref.mask())
            st, r, d, _ = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert np.array_equal(np.array(st).view(np.uint64), rs.view(np.uint64)), (level, serve, t)
            assert (r, d) == (rr, rd), (level, serve, t)
            if d or t % 37 == 20:
                s0 = env.reset()
                ref.reset()
                assert np.array_equal(np.array(s0).view(np.uint64), ref.obs.view(np.uint64)), (level, serve, t)
        assert env._vec.errors() == 0
        env.close()


def test_serve_wide_level_gotable_over_64k(tg, oracle, tmp_path):
    """gen1 widened to 60 cells: its GoTable (60 x 11 x 32 x 4 B = 84 KB) exceeds 64 KB, so the
    server's dynamic LDS needs hipFuncSetAttribute (the staging path a default-size level never
    takes); no level bitmasks at that width.  Server and launch-per-call vs the oracle."""
    import os
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels", "gen1")
    rows = [r.rstrip("\n") for r in open(os.path.join(src, "domain.txt")) if r.strip()]
    extra = 60 - len(rows[0])
    wide = [r[:-1] + ("/" if y % 2 == 0 else " ") * extra + r[-1] for y, r in enumerate(rows)]
    ld = tmp_path / "gen1_wide"
    ld.mkdir()
    (ld / "domain.txt").write_text("\n".join(wide) + "\n")
    for f in ("domain-objects.txt", "domain-interactions.txt"):
        (ld / f).write_text(open(os.path.join(src, f)).read())
    for serve in (True, False):
        env = tg.TreasureGame(seed=5, level_dir=str(ld))
        env._vec.set_serve(serve)
        ref = oracle.OracleEnv(5, level_dir=str(ld))
        s0 = env.reset()
        assert np.array_equal(np.array(s0).view(np.uint64), ref.obs.view(np.uint64))
        for t in range(60):
            assert env.available_mask.tolist() == [(ref.mask() >> k) & 1 for k in range(9)], (serve, t)
            a = oracle.pick_action(0x99, 5, t, True, ref.mask())
            st, r, d, _ = env.step(a)
            rs, rr, rd, _ = ref.step(a)
            assert np.array_equal(np.array(st).view(np.uint64), rs.view(np.uint64)), (serve, t)
            assert (r, d) == (rr, rd), (serve, t)
            if d:
                env.reset()
                ref.reset()
        assert env._vec.errors() == 0
        env.close()
