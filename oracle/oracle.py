"""ctypes wrapper of oracle/libtg_oracle.so — TEST INFRASTRUCTURE ONLY.

The CPU parity oracle (see tg_oracle.c's header).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg import this module, and only as the checker / CPU baseline; the
product package never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libtg_oracle.so")
LEVEL_DIR = os.path.join(os.path.dirname(HERE), "gym-treasure-game_amd", "levels", "default")

_lib = None
_levels = {}


def build(force=False):
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        u64, i64, i32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int
        L.tgo_level_parse.restype = P
        L.tgo_level_parse.argtypes = [ctypes.c_char_p] * 3
        L.tgo_env_new.restype = P
        L.tgo_env_new.argtypes = [P, u64, P]
        L.tgo_env_free.argtypes = [P]
        L.tgo_step.restype = i32
        L.tgo_step.argtypes = [P, i32, P, P, P, P]
        L.tgo_reset.argtypes = [P, P]
        L.tgo_mask.restype = ctypes.c_uint
        L.tgo_mask.argtypes = [P]
        L.tgo_draws.restype = u64
        L.tgo_draws.argtypes = [P]
        L.tgo_ticks.restype = i64
        L.tgo_ticks.argtypes = [P]
        L.tgo_internal.argtypes = [P, P]
        L.tgo_predicates.restype = ctypes.c_uint
        L.tgo_predicates.argtypes = [P, i32, i32, ctypes.c_uint]
        L.tgo_predicate_table.argtypes = [P, i32, i32, i32, i32, ctypes.c_uint, P]
        L.tgo_run.restype = i32
        L.tgo_run.argtypes = [P, u64, i64, i64, i32, u64, i32, i32, P, P, P, P, P, P, P, P, i32]
        L.tgo_run_episodes.restype = i32
        L.tgo_run_episodes.argtypes = [P, u64, i64, i64, i32, u64, i32, i32, P, P, i32]
        L.tgo_rng_words.argtypes = [u64, i32, P]
        L.tgo_rng_random.argtypes = [u64, i32, P]
        L.tgo_rng_uniform5.argtypes = [u64, P]
        L.tgo_rng_gauss.argtypes = [u64, i32, P]
        L.tgo_sm64.restype = u64
        L.tgo_sm64.argtypes = [u64]
        L.tgo_action_hash.restype = u64
        L.tgo_action_hash.argtypes = [u64, u64, u64]
        L.tgo_pick_action.restype = i32
        L.tgo_pick_action.argtypes = [u64, u64, u64, i32, ctypes.c_uint]
        L.tgo_render.restype = i32
        L.tgo_render.argtypes = [P, P, i32, i32, P]
        L.tgo_run_render.restype = i32
        L.tgo_run_render.argtypes = [P, u64, P, i64, i32, u64, i32, i32, P, i32, i32, P, i32]
        L.tgo_choice_seq.argtypes = [u64, i32, i32, P]
        _lib = L
    return _lib


def level(level_dir=None):
    """Parsed level (the reference's three level texts); default = the shipped level."""
    d = os.path.abspath(level_dir or LEVEL_DIR)
    if d not in _levels:
        texts = []
        for f in ("domain.txt", "domain-objects.txt", "domain-interactions.txt"):
            with open(os.path.join(d, f), "rb") as fh:
                texts.append(fh.read())
        lv = lib().tgo_level_parse(*texts)
        if not lv:
            raise RuntimeError("oracle: level parse failed: %s" % d)
        _levels[d] = lv
    return _levels[d]


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """One reference-equivalent env: random.seed(seed); TreasureGame(); reset()."""

    def __init__(self, seed, level_dir=None):
        self._obs = np.zeros(9, np.float64)
        self._h = lib().tgo_env_new(level(level_dir), seed, _p(self._obs))
        self._shape = _level_frame_shape(level_dir)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().tgo_env_free(self._h)
            self._h = None

    @property
    def obs(self):
        return self._obs.copy()

    def step(self, a):
        o = np.zeros(9, np.float64)
        r = np.zeros(1, np.int32)
        v = np.zeros(1, np.uint8)
        d = np.zeros(1, np.uint8)
        rc = lib().tgo_step(self._h, int(a), _p(o), _p(r), _p(v), _p(d))
        if rc == -1:
            raise IndexError("list index out of range")
        self._obs = o
        return o, (int(r[0]) if v[0] else None), bool(d[0]), {}

    def reset(self):
        o = np.zeros(9, np.float64)
        lib().tgo_reset(self._h, _p(o))
        self._obs = o
        return o

    def mask(self):
        return int(lib().tgo_mask(self._h))

    def draws(self):
        return int(lib().tgo_draws(self._h))

    def ticks(self):
        return int(lib().tgo_ticks(self._h))

    def internal(self):
        out = np.zeros(12, np.int32)
        lib().tgo_internal(self._h, _p(out))
        return out

    def render(self, sprites):
        """render('rgb_array') of the current state (PARITY UNPINNED, see tg_oracle.c):
        uint8 [H*48, W*48, 3].  sprites: uint8 [24, sh, sw, 4] RGBA in TG_SPR_* order."""
        sprites = np.ascontiguousarray(sprites, np.uint8)
        h, w = self._shape
        out = np.zeros((h, w, 3), np.uint8)
        rc = lib().tgo_render(self._h, _p(sprites), sprites.shape[2], sprites.shape[1], _p(out))
        if rc < 0:
            raise RuntimeError("oracle render: unsupported geometry")
        return out

    def predicates(self, px, py, door_bits):
        return int(lib().tgo_predicates(self._h, int(px), int(py), int(door_bits)))

    def predicate_table(self, x0, x1, y0, y1, door_bits):
        out = np.zeros((y1 - y0, x1 - x0), np.uint8)
        lib().tgo_predicate_table(self._h, x0, x1, y0, y1, door_bits, _p(out))
        return out


def run(seed_base, g0, n, steps, action_seed, policy=0, autoreset=False, full=True,
        nthreads=0, level_dir=None):
    """Batched oracle run. Returns dict of numpy arrays (env-major, t=0 is the reset)."""
    T1 = steps + 1
    out = {}
    if full:
        out["obs"] = np.zeros((n, T1, 9), np.float64)
        out["final_obs"] = np.zeros((n, T1, 9), np.float64)
        out["reward"] = np.zeros((n, T1), np.int32)
        out["valid"] = np.zeros((n, T1), np.uint8)
        out["done"] = np.zeros((n, T1), np.uint8)
    out["hash"] = np.zeros(n, np.uint64)
    out["draws"] = np.zeros(n, np.int64)
    out["ticks"] = np.zeros(n, np.int64)
    rc = lib().tgo_run(level(level_dir), seed_base, g0, n, steps, action_seed, policy, int(autoreset),
                       _p(out.get("obs")), _p(out.get("reward")), _p(out.get("valid")),
                       _p(out.get("done")), _p(out.get("final_obs")), _p(out["hash"]),
                       _p(out["draws"]), _p(out["ticks"]), nthreads)
    if rc != 0:
        raise RuntimeError("oracle run failed")
    return out


def run_episodes(seed_base, g0, n, steps, action_seed, policy=0, t_from=0, nthreads=0,
                 level_dir=None):
    """Auto-reset run of envs [g0, g0 + n): (count, digest) of the episodes whose last step
    index is >= t_from (digest as gym_treasure_game_amd.dist.episode_digest)."""
    cnt = ctypes.c_int64(0)
    dig = ctypes.c_uint64(0)
    rc = lib().tgo_run_episodes(level(level_dir), seed_base, g0, n, steps, action_seed, policy,
                                t_from, ctypes.byref(cnt), ctypes.byref(dig), nthreads)
    if rc != 0:
        raise RuntimeError("oracle run failed")
    return int(cnt.value), int(dig.value)


def rng_words(seed, n):
    out = np.zeros(n, np.uint32)
    lib().tgo_rng_words(seed, n, _p(out))
    return out


def rng_random(seed, n):
    out = np.zeros(n, np.float64)
    lib().tgo_rng_random(seed, n, _p(out))
    return out


def rng_uniform5(seed):
    out = np.zeros(5, np.float64)
    lib().tgo_rng_uniform5(seed, _p(out))
    return out


def rng_gauss(seed, pairs):
    out = np.zeros(2 * pairs, np.float64)
    lib().tgo_rng_gauss(seed, pairs, _p(out))
    return out


def pick_action(a0, g, t, masked=False, mask=0):
    return int(lib().tgo_pick_action(a0, g, t, int(masked), mask))


def _level_frame_shape(level_dir=None):
    d = os.path.abspath(level_dir or LEVEL_DIR)
    with open(os.path.join(d, "domain.txt")) as fh:
        rows = [ln.strip() for ln in fh.read().split("\n")]
    while rows and not rows[-1]:
        rows.pop()
    return len(rows) * 48, len(rows[0]) * 48


def run_render(seed_base, envs, steps, action_seed, policy, autoreset, sprites, nthreads=0,
               level_dir=None):
    """Frames of the listed global envs after `steps` env-steps of the run() action stream:
    uint8 [len(envs), H*48, W*48, 3] (PARITY UNPINNED renderer restatement)."""
    envs = np.ascontiguousarray(envs, np.int64)
    sprites = np.ascontiguousarray(sprites, np.uint8)
    h, w = _level_frame_shape(level_dir)
    out = np.zeros((len(envs), h, w, 3), np.uint8)
    rc = lib().tgo_run_render(level(level_dir), seed_base, _p(envs), len(envs), steps, action_seed,
                              int(policy), int(autoreset), _p(sprites), sprites.shape[2],
                              sprites.shape[1], _p(out), nthreads)
    if rc < 0:
        raise RuntimeError("oracle run_render failed")
    return out


def choice_seq(seed, n, count):
    out = np.zeros(count, np.int32)
    lib().tgo_choice_seq(seed, n, count, _p(out))
    return out
