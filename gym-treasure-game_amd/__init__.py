"""MI355X-native batched Treasure Game (drop-in for gym_treasure_game's ``treasure_game-v0``).

    import gym_treasure_game_amd as tg
    env = tg.make("treasure_game-v0", seed=0)            # N = 1, reference types
    vec = tg.make("treasure_game-v0", num_envs=1 << 20)  # N envs on one GPU, torch tensors

The step path runs in libtg_amd.so (hand-written HIP for gfx950, C ABI in include/tg_amd.h);
there is no CPU fallback.  Registration with gym / gymnasium happens on import when either is
installed, mirroring gym_treasure_game/__init__.py:3-6.
"""
from ._lib import TG_ERR_FLOW, TgError  # noqa: F401
from .envs import (OPTION_NAMES, STATE_NAMES, GpuOption, ObservationWrapper,  # noqa: F401
                   TreasureGame, TreasureGameVec, TreasureGameVectorEnv, make_vec, read_level)
from .render import load_sprites, synthetic_sprites  # noqa: F401

__version__ = "0.1.0"
ENV_ID = "treasure_game-v0"


def make(id=ENV_ID, num_envs=None, **kwargs):
    """``gym.make`` stand-in: ``num_envs=None`` -> TreasureGame, else TreasureGameVec."""
    if id != ENV_ID:
        raise KeyError("unknown env id %r (only %r)" % (id, ENV_ID))
    if num_envs is None:
        return TreasureGame(**kwargs)
    return TreasureGameVec(num_envs, **kwargs)


def register():
    """Register ``treasure_game-v0`` with gym and/or gymnasium when they are importable."""
    done = []
    for mod in ("gym", "gymnasium"):
        try:
            reg = __import__(mod + ".envs.registration", fromlist=["register"])
        except Exception:  # noqa: BLE001 — not installed
            continue
        try:
            reg.register(id=ENV_ID, entry_point="gym_treasure_game_amd.envs:TreasureGame")
            done.append(mod)
        except Exception:  # noqa: BLE001 — already registered
            done.append(mod)
    return done


register()
