"""Sprite sheets for render('rgb_array') (TG/:98-105, DR/:57-134).

The renderer (libtg_amd.so ``tg_render_init`` / ``tg_render``) takes the reference's sprites
as one RGBA8 sheet in ``TG_SPR_*`` order.  The sprites are the reference's art, not shipped
here (the hero, handle and key are Braid assets used with permission, see the reference's
sprites/attribution.txt): ``load_sprites`` decodes them from an installed
gym_treasure_game (or any directory with the same layout) with PIL, the same RGBA decode
pygame's ``image.load().convert_alpha()`` gives for these PNGs.  ``synthetic_sprites`` makes a
sheet of the same shape with random colours and alphas (every blend case: 0, 255 and
in between) for tests and benchmarks on machines without the reference.
"""
import importlib.util
import os

import numpy as np

# TG_SPR_* order (include/tg_amd.h); paths relative to the reference's sprites/ directory
SPRITE_FILES = (
    ["background/background_%d.png" % i for i in range(5)]
    + ["wall/wall_%d.png" % i for i in range(5)]
    + ["floor/floor-%d.png" % i for i in range(5)]
    + ["ladder.png", "closeddoor.png", "open-door.png", "key.png", "gold.png", "bolt-open.png",
       "bolt-locked.png", "hero.png", "handle-base.png"])
SPRITE_COUNT = len(SPRITE_FILES)  # TG_SPR_COUNT


def default_sprite_dir():
    """$TG_SPRITE_DIR, else the sprites/ of an installed gym_treasure_game, else None."""
    d = os.environ.get("TG_SPRITE_DIR")
    if d:
        return d
    try:
        spec = importlib.util.find_spec("gym_treasure_game")  # does not import it (gym-free)
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return None
    d = os.path.join(list(spec.submodule_search_locations)[0], "envs", "_treasure_game_impl",
                     "sprites")
    return d if os.path.isdir(d) else None


def load_sprites(sprite_dir=None):
    """uint8 [24, h, w, 4] RGBA from the reference's sprite PNGs (all the same size)."""
    from PIL import Image

    sprite_dir = sprite_dir or default_sprite_dir()
    if not sprite_dir:
        raise FileNotFoundError("no sprite directory: pass sprite_dir, set TG_SPRITE_DIR, or "
                                "install gym_treasure_game (its sprites/ is used)")
    imgs = [np.asarray(Image.open(os.path.join(sprite_dir, f)).convert("RGBA"), np.uint8)
            for f in SPRITE_FILES]
    if len({im.shape for im in imgs}) != 1:
        raise ValueError("sprites differ in size: %s" % sorted({im.shape for im in imgs}))
    return np.ascontiguousarray(np.stack(imgs))


def synthetic_sprites(seed=0, size=32):
    """uint8 [24, size, size, 4]: random RGB, alpha 0 / 255 / uniform in thirds per pixel."""
    rng = np.random.default_rng(seed)
    sheet = rng.integers(0, 256, (SPRITE_COUNT, size, size, 4), dtype=np.uint8)
    kind = rng.integers(0, 3, (SPRITE_COUNT, size, size))
    sheet[..., 3] = np.where(kind == 0, 0, np.where(kind == 1, 255, sheet[..., 3]))
    return sheet
