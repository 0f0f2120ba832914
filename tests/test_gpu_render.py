"""GPU: render('rgb_array') (k_render through tg_render) against the oracle's pygame/SDL
restatement, byte for byte.  Parity with the reference renderer itself is UNPINNED (pygame is
absent from this image); the sprite sheets are synthetic (random colours, alpha 0
/ 255 / in between, so every blend case is exercised) because the reference's art does not
travel to the GPU box."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _frames_vs_oracle(oracle, got, envs, steps, a0, policy, autoreset, sprites, level_dir=None):
    want = oracle.run_render(0, envs, steps, a0, policy, autoreset, sprites, level_dir=level_dir)
    for i, g in enumerate(envs):
        if not np.array_equal(got[i], want[i]):
            bad = np.argwhere((got[i] != want[i]).any(-1))
            raise AssertionError("env %d step %d: %d pixels differ, first at (y, x) = %s"
                                 % (g, steps, len(bad), tuple(bad[0])))


def test_render_every_step_vs_oracle(tg, oracle):
    """48 envs, masked policy with auto-reset: every frame of 40 steps."""
    n, steps, a0 = 48, 40, 0x77
    sprites = tg.synthetic_sprites(seed=5)
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True)
    vec.render_init(sprites)
    assert vec.frame_shape == (624, 672, 3)
    vec.reset()
    envs = np.arange(n)
    for t in range(steps + 1):
        if t:
            vec.step(vec.policy_actions(t - 1, a0, "masked"))
        _frames_vs_oracle(oracle, vec.render().cpu().numpy(), envs, t, a0, 1, True, sprites)
    assert vec.errors() == 0
    vec.close()


def test_render_subrange_and_out(tg):
    n = 300  # not a multiple of the 16-env workgroup
    vec = tg.TreasureGameVec(n, seed=9, autoreset=True)
    vec.render_init(tg.synthetic_sprites(seed=1, size=16))
    for t in range(15):
        vec.step(vec.policy_actions(t, 3, "uniform"))
    full = vec.render().clone()
    part = vec.render(first=37, count=100)
    assert torch.equal(part, full[37:137])
    buf = torch.empty((5,) + vec.frame_shape, dtype=torch.uint8, device=vec.device)
    assert vec.render(first=n - 5, count=5, out=buf).data_ptr() == buf.data_ptr()
    assert torch.equal(buf, full[n - 5:])
    with pytest.raises(tg.TgError):
        vec.render(first=n - 4, count=5)
    vec.close()


def test_render_c5_sample_vs_oracle(tg, oracle):
    """Config C5: 65,536 envs rendered in one launch (82 GB of frames); 512 spread envs vs
    the oracle after 25 uniform auto-reset steps, and a rerender is identical."""
    n, steps, a0 = 65536, 25, 0xC5
    sprites = tg.synthetic_sprites(seed=55)
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True)
    vec.render_init(sprites)
    vec.reset()
    for t in range(steps):
        vec.step(vec.policy_actions(t, a0, "uniform"))
    frames = vec.render()
    envs = np.unique(np.concatenate([np.arange(64), np.linspace(0, n - 1, 448).astype(np.int64)]))
    for k in range(0, len(envs), 64):
        chunk = envs[k:k + 64]
        got = frames.index_select(0, torch.as_tensor(chunk, device=vec.device)).cpu().numpy()
        _frames_vs_oracle(oracle, got, chunk, steps, a0, 0, True, sprites)
    sums = frames.view(n, -1).view(torch.int64).sum(1)  # per-frame checksum (wrapping)
    again = vec.render(out=frames)
    assert torch.equal(again.view(n, -1).view(torch.int64).sum(1), sums)
    assert vec.errors() == 0
    del frames, again
    vec.close()
    torch.cuda.empty_cache()


def test_single_env_render_and_observation_wrapper(tg, oracle):
    sprites = tg.synthetic_sprites(seed=8)
    env = tg.make("treasure_game-v0", seed=3, sprites=sprites)
    e = oracle.OracleEnv(3)
    env.reset()
    for t in range(30):
        a = oracle.pick_action(1, 3, t, True, e.mask())
        env.step(a)
        e.step(a)
        f = env.render(mode="rgb_array")
        assert f.shape == (624, 672, 3) and f.dtype == np.uint8
        np.testing.assert_array_equal(f, e.render(sprites), err_msg="step %d" % t)
    with pytest.raises(NotImplementedError):
        env.render(mode="human")
    env.close()

    w = tg.ObservationWrapper(tg.make("treasure_game-v0", seed=4), sprites=sprites)
    e = oracle.OracleEnv(4)
    np.testing.assert_array_equal(w.reset(), e.render(sprites))
    for t in range(10):
        a = oracle.pick_action(1, 4, t, True, e.mask())
        screen, r, d, info = w.step(a)
        o, r2, d2, _ = e.step(a)
        np.testing.assert_array_equal(screen, e.render(sprites))
        assert (r, d) == (r2, d2)
        assert np.array_equal(np.array(info["world_state"]).view(np.uint64), o.view(np.uint64))
    w.close()


def test_vec_observation_wrapper(tg, oracle):
    n, a0 = 32, 0x99
    sprites = tg.synthetic_sprites(seed=12)
    w = tg.ObservationWrapper(tg.TreasureGameVec(n, seed=0, autoreset=True), sprites=sprites)
    frames = w.reset()
    assert frames.shape == (n, 624, 672, 3)
    _frames_vs_oracle(oracle, frames.cpu().numpy(), np.arange(n), 0, a0, 1, True, sprites)
    for t in range(6):
        frames, rew, valid, done, info = w.step(w.env.policy_actions(t, a0, "masked"))
        assert info["world_state"].shape == (n, 9)
    _frames_vs_oracle(oracle, frames.cpu().numpy(), np.arange(n), 6, a0, 1, True, sprites)
    w.close()


def test_render_other_level_vs_oracle(tg, oracle):
    """A 44 x 5-cell level (frames 240 x 2,112, 396 chunks per row) through the C ABI."""
    import os
    level = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "levels", "corridor")
    sprites = tg.synthetic_sprites(seed=21, size=40)
    n, a0 = 40, 0x3C
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True, level_dir=level)
    vec.render_init(sprites)
    assert vec.frame_shape == (240, 2112, 3)
    vec.reset()
    for t in range(8):
        vec.step(vec.policy_actions(t, a0, "masked"))
    _frames_vs_oracle(oracle, vec.render().cpu().numpy(), np.arange(n), 8, a0, 1, True, sprites,
                      level_dir=level)
    assert vec.errors() == 0
    vec.close()

