"""Env surfaces over the C ABI: ``TreasureGameVec`` (N envs on one GPU, torch tensors) and
``TreasureGame`` (the N=1 drop-in for the reference ``TreasureGame``, treasure_game.py:54-114).

Seeding contract: env ``g`` of a batch created with ``seed=s,
global_offset=o`` replays, bit for bit, a reference env in a fresh process after
``random.seed(s + o + g); env = TreasureGame(); env.reset()``.  Every env owns its own
CPython-compatible MT19937 stream; the reference's envs share one process-global stream
(IM/:2, OB/:9), which is the one deliberate difference.
"""
import ctypes
import operator
import os
import random
import struct

import numpy as np
import torch

from . import _lib
from ._lib import TgError, check

OPTION_NAMES = ["go_left_option", "go_right_option", "up_ladder_option", "down_ladder_option",
                "interact_option", "down_left_option", "down_right_option", "jump_left_option",
                "jump_right_option"]  # create_options order (IM/:484-498)
STATE_NAMES = ["playerx", "playery", "handle1.angle", "handle2.angle", "key.x", "key.y",
               "bolt.locked", "goldcoin.x", "goldcoin.y"]  # get_state_descriptors (IM/:380-400)
LEVEL_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "levels", "default")


# ---- spaces: gym's / gymnasium's when importable, else minimal stand-ins with the same fields
def _spaces():
    for mod in ("gym.spaces", "gymnasium.spaces"):
        try:
            m = __import__(mod, fromlist=["Discrete", "Box", "MultiDiscrete"])
            return m.Discrete, m.Box, m.MultiDiscrete
        except Exception:  # noqa: BLE001 — absent or broken install: use the stand-ins
            continue

    class Discrete:
        def __init__(self, n):
            self.n = int(n)
            self.shape = ()
            self.dtype = np.int64

        def sample(self):
            return random.randrange(self.n)

        def contains(self, x):
            try:
                return 0 <= int(x) < self.n
            except (TypeError, ValueError):
                return False

        def __repr__(self):
            return "Discrete(%d)" % self.n

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.shape = tuple(shape)
            self.dtype = np.dtype(dtype)
            self.low = np.full(self.shape, low, self.dtype)
            self.high = np.full(self.shape, high, self.dtype)

        def sample(self):
            return np.random.uniform(self.low, self.high).astype(self.dtype)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

        def __repr__(self):
            return "Box(%s, %s, %s, %s)" % (self.low.min(), self.high.max(), self.shape, self.dtype)

    class MultiDiscrete:
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec, np.int64)
            self.shape = self.nvec.shape
            self.dtype = np.int64

        def sample(self):
            return (np.random.random_sample(self.shape) * self.nvec).astype(np.int64)

        def contains(self, x):
            x = np.asarray(x)
            return x.shape == self.shape and bool(np.all((x >= 0) & (x < self.nvec)))

        def __repr__(self):
            return "MultiDiscrete(%s)" % (self.nvec,)

    return Discrete, Box, MultiDiscrete


Discrete, Box, MultiDiscrete = _spaces()


def read_level(path=LEVEL_DIR):
    """The three level files (reference formats, IM/:75-202) as bytes."""
    out = []
    for f in ("domain.txt", "domain-objects.txt", "domain-interactions.txt"):
        with open(os.path.join(path, f), "rb") as fh:
            out.append(fh.read())
    return tuple(out)


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class TreasureGameVec:
    """``num_envs`` Treasure Game envs resident in one GPU's HBM.

    ``step`` takes an int32 action tensor [N] (values in [-9, 8], Python list indexing as in
    TG/:92) and returns ``(obs f64 [N,9], reward i32 [N], valid u8 [N], done u8 [N], info)``;
    ``valid == 0`` is the reference's ``None`` reward (OP/:22-23).  Returned tensors are the
    env's own output buffers and are overwritten by the next call (``copy=True`` clones).
    With ``autoreset=True`` an env that returns done is reset in the same step (the reference
    never resets by itself; this is the equivalent of calling ``reset()`` right after), its
    pre-reset obs goes to ``info["final_obs"]`` and its episode (return, length) to
    ``episodes()``.
    """

    def __init__(self, num_envs, seed=0, device=None, global_offset=0, autoreset=False,
                 level_dir=None, copy=False, mode="compact"):
        if not torch.cuda.is_available():
            raise TgError("TreasureGameVec needs a ROCm GPU (gfx950); there is no CPU path")
        self._L = _lib.load()
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.seed = int(seed)
        self.global_offset = int(global_offset)
        if self.num_envs <= 0 or self.global_offset < 0:
            raise ValueError("num_envs must be > 0 and global_offset >= 0")
        # env g is random.seed(seed + global_offset + g); the device seeds init_by_array with
        # a key of at most two 32-bit words, so every env's seed must lie in [0, 2^64)
        # (CPython's abs() of a negative seed is not monotone in g: TreasureGame maps it)
        if self.seed < 0 or self.seed + self.global_offset + self.num_envs - 1 >= 2**64:
            raise ValueError("seed + global_offset + g must lie in [0, 2**64) for every env "
                             "(got seed=%d, global_offset=%d, num_envs=%d)"
                             % (self.seed, self.global_offset, self.num_envs))
        self.autoreset = bool(autoreset)
        self.copy = bool(copy)
        texts = read_level(level_dir) if level_dir else (None, None, None)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self._L.tg_create(ctypes.byref(h), self.num_envs, self.seed,
                                    self.global_offset, self.device.index, *texts), "tg_create")
        self._h = h
        n, dev = self.num_envs, self.device
        self._obs = torch.empty((n, 9), dtype=torch.float64, device=dev)
        self._final = torch.empty((n, 9), dtype=torch.float64, device=dev) if autoreset else None
        self._rew = torch.empty(n, dtype=torch.int32, device=dev)
        self._valid = torch.empty(n, dtype=torch.uint8, device=dev)
        self._done = torch.empty(n, dtype=torch.uint8, device=dev)
        self._act = torch.empty(n, dtype=torch.int32, device=dev)
        self._mask = torch.empty(n, dtype=torch.int16, device=dev)
        self.action_space = Discrete(_lib.NUM_ACTIONS)
        self.observation_space = Box(np.float32(0.0), np.float32(1.0), shape=(_lib.OBS_DIM,))
        self.option_names = list(OPTION_NAMES)
        self._mode = "compact"
        if mode != "compact":
            self.set_mode(mode)

    # -- plumbing ---------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _out(self, t):
        return t.clone() if self.copy else t

    @property
    def handle(self):
        if self._h is None:
            raise TgError("env is closed")
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None:
            torch.cuda.synchronize(self.device)
            self._L.tg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 — interpreter teardown
            pass

    # -- reference surface --------------------------------------------------------------------
    def reset(self, mask=None):
        """reset() (TG/:78-81) of every env, or of those with mask[i] != 0."""
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
            if m.numel() != self.num_envs:
                raise ValueError("mask must have num_envs entries")
        check(self._L.tg_reset(self.handle, _ptr(m), _ptr(self._obs), self._stream()), "tg_reset")
        return self._out(self._obs)

    def step(self, actions):
        """step(a) (TG/:91-96) for every env."""
        a = actions
        if not (isinstance(a, torch.Tensor) and a.dtype == torch.int32 and a.device == self.device
                and a.is_contiguous()):
            a = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        if a.numel() != self.num_envs:
            raise ValueError("actions must have num_envs entries")
        check(self._L.tg_step(self.handle, _ptr(a), _ptr(self._obs), _ptr(self._rew),
                              _ptr(self._valid), _ptr(self._done), _ptr(self._final),
                              _lib.TG_STEP_AUTORESET if self.autoreset else 0, self._stream()),
              "tg_step")
        info = {"final_obs": self._out(self._final)} if self.autoreset else {}
        return (self._out(self._obs), self._out(self._rew), self._out(self._valid),
                self._out(self._done), info)

    def rollout(self, steps, t0=0, action_seed=0x5EED0001, policy="uniform", obs=True,
                actions=True, check_flow=True):
        """``steps`` env-steps in one call with the on-device synthetic policy (tg_rollout):
        step t0 + s takes ``policy_actions(t0 + s, action_seed, policy)``, evaluated inside the
        step kernels.  Returns step-major device tensors: reward i32 [K, N], valid / done u8
        [K, N], and (optionally) obs f64 [K, N, 9], actions i32 [K, N].  With auto-reset the
        obs rows are the post-reset ones and finished episodes queue for ``episodes()``.

        In "flow" mode a k_flow launch that fails its protocol checks (a wait past its bound,
        a sub-problem left unstepped, an item out of range) sets TG_ERR_FLOW and its rows are
        not valid: with ``check_flow`` (the default) the call then synchronises on
        ``errors()`` and raises TgError."""
        pol = {"uniform": _lib.TG_POLICY_UNIFORM, "masked": _lib.TG_POLICY_MASKED}[policy]
        k, n, dev = int(steps), self.num_envs, self.device
        out = {"reward": torch.empty((k, n), dtype=torch.int32, device=dev),
               "valid": torch.empty((k, n), dtype=torch.uint8, device=dev),
               "done": torch.empty((k, n), dtype=torch.uint8, device=dev)}
        if obs:
            out["obs"] = torch.empty((k, n, 9), dtype=torch.float64, device=dev)
        if actions:
            out["actions"] = torch.empty((k, n), dtype=torch.int32, device=dev)
        check(self._L.tg_rollout(self.handle, k, action_seed, int(t0), pol,
                                 _lib.TG_STEP_AUTORESET if self.autoreset else 0,
                                 _ptr(out.get("actions")), _ptr(out.get("obs")),
                                 _ptr(out["reward"]), _ptr(out["valid"]), _ptr(out["done"]),
                                 self._stream()), "tg_rollout")
        if check_flow and self._mode == "flow" and self.errors() & _lib.TG_ERR_FLOW:
            raise TgError("tg_rollout: a k_flow launch set TG_ERR_FLOW (its rows are not valid)")
        return out

    def set_groups(self, groups=1, stagger=False):
        """rollout() steps the batch as ``groups`` contiguous groups, each on a stream of its
        own (tg_set_groups: overlaps one group's option loops with another's bandwidth-bound
        passes; results identical).  1: off."""
        check(self._L.tg_set_groups(self.handle, int(groups), 1 if stagger else 0),
              "tg_set_groups")

    def available_mask(self):
        """available_mask (TG/:83-89) as bits: int16 [N], bit k == option k can run."""
        check(self._L.tg_available_mask(self.handle, _ptr(self._mask), self._stream()),
              "tg_available_mask")
        return self._out(self._mask)

    def observe(self):
        """get_state (IM/:368-378) of every env."""
        check(self._L.tg_observe(self.handle, _ptr(self._obs), self._stream()), "tg_observe")
        return self._out(self._obs)

    # -- batch extras -------------------------------------------------------------------------
    def policy_actions(self, t, action_seed=0x5EED0001, policy="uniform", out=None):
        """Counter-hash synthetic actions for step t (bench / parity), keyed by GLOBAL env id."""
        pol = {"uniform": _lib.TG_POLICY_UNIFORM, "masked": _lib.TG_POLICY_MASKED}[policy]
        out = self._act if out is None else out
        check(self._L.tg_policy_actions(self.handle, action_seed, int(t), pol, _ptr(out),
                                        self._stream()), "tg_policy_actions")
        return out

    def drain_episodes(self, out, count):
        """Asynchronous device drain: up to out.shape[0] records -> ``out`` (int64 [cap, 2],
        the raw 16-B tg_episode rows), their number -> ``count`` (int32 [1])."""
        if not (isinstance(out, torch.Tensor) and out.dtype == torch.int64 and out.dim() == 2
                and out.size(1) == 2 and out.is_contiguous() and out.device == self.device):
            raise ValueError("out must be a contiguous int64 [cap, 2] tensor on %s" % self.device)
        if not (isinstance(count, torch.Tensor) and count.dtype == torch.int32
                and count.numel() >= 1 and count.is_contiguous() and count.device == self.device):
            raise ValueError("count must be a contiguous int32 tensor of >= 1 element on %s"
                             % self.device)
        if out.size(0) >= 2**31:
            raise ValueError("out holds too many rows")
        check(self._L.tg_episodes(self.handle, _ptr(out), _ptr(count), out.shape[0],
                                  self._stream()), "tg_episodes")

    @staticmethod
    def decode_episodes(rows):
        """raw tg_episode rows (int64 [k, 2]) -> int64 [k, 3] = (env, return, length)."""
        packed = rows[:, 1]
        ret = ((packed & 0xFFFFFFFF) ^ 0x80000000) - 0x80000000  # sign-extend the i32 half
        return torch.stack([rows[:, 0], ret, packed >> 32], dim=1)

    def episodes(self, cap=None):
        """Completed (auto-reset) episodes, oldest first, up to ``cap`` of them:
        int64 [k, 3] = (global env, return, length) on the device (synchronises)."""
        cap = self.num_envs if cap is None else int(cap)
        rec = torch.empty((max(cap, 1), 2), dtype=torch.int64, device=self.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.drain_episodes(rec[:cap], cnt)
        return self.decode_episodes(rec[: int(cnt.item())])

    def errors(self):
        v = ctypes.c_uint32(0)
        check(self._L.tg_errors(self.handle, ctypes.byref(v), self._stream()), "tg_errors")
        return int(v.value)

    def set_serve(self, on=True):
        """A 1-env handle's N = 1 calls (TreasureGame.step / reset) through the resident server
        kernel (the default; tg_set_serve) or one launch + synchronisation each: identical
        results, the server without the launch and the synchronisation."""
        check(self._L.tg_set_serve(self.handle, 1 if on else 0), "tg_set_serve")

    def set_mode(self, mode="compact", run_blocks=0):
        """Step implementation: "compact" (two-pass, default), "direct" (one lane per env
        runs in place) or "flow" (as compact per step; rollout() runs up to 16 steps per launch,
        chunks advancing without a batch-wide barrier between steps); all bit-identical."""
        m = {"direct": _lib.TG_MODE_DIRECT, "compact": _lib.TG_MODE_COMPACT,
             "flow": _lib.TG_MODE_FLOW}[mode]
        check(self._L.tg_set_mode(self.handle, m, int(run_blocks)), "tg_set_mode")
        self._mode = mode

    def set_episode_capacity(self, cap):
        """Resize the completed-episode queue (discards what it holds)."""
        check(self._L.tg_set_episode_capacity(self.handle, int(cap)), "tg_set_episode_capacity")

    def predicate_table(self, x0, x1, y0, y1, door_bits):
        """The six collision predicates (IM/:232-288) evaluated on the device at every pixel
        of [x0, x1) x [y0, y1) with doors closed per door_bits: uint8 [y1-y0, x1-x0] device
        tensor, bit k = up_clear, can_go_up, can_go_down, can_go_left, can_go_right, can_fall."""
        out = torch.empty((y1 - y0, x1 - x0), dtype=torch.uint8, device=self.device)
        check(self._L.tg_predicate_table(self.handle, x0, x1, y0, y1, int(door_bits), _ptr(out),
                                         self._stream()), "tg_predicate_table")
        return out

    def set_timing(self, every=1):
        """HIP-event timing of every ``every``-th step launch (0 / False: off; True: every
        launch).  stats() then holds kernel_ms / run_ms summed over timed_launches."""
        check(self._L.tg_set_timing(self.handle, int(every)), "tg_set_timing")

    def regenerate(self):
        """Regenerate every stale MT half still queued (tg_regenerate: results never depend on
        it; a timed loop calls it at its end so that it holds its own steps' regeneration)."""
        check(self._L.tg_regenerate(self.handle, self._stream()), "tg_regenerate")

    def stats(self):
        s = _lib.Stats()
        check(self._L.tg_get_stats(self.handle, ctypes.byref(s)), "tg_get_stats")
        return s.as_dict()

    def stats_reset(self):
        check(self._L.tg_stats_reset(self.handle), "tg_stats_reset")

    def kernel_info(self):
        """{kernel: (workgroups per CU, VGPRs, LDS bytes)} of the step kernels (tg_kernel_info)"""
        out = {}
        for name, k in (("k_classify", 0), ("k_run", 1), ("k_regen", 2)):
            v = [ctypes.c_int32() for _ in range(4)]
            check(self._L.tg_kernel_info(self.handle, k, *[ctypes.byref(x) for x in v]),
                  "tg_kernel_info")
            out[name] = {"blocks_per_cu": v[0].value, "waves_per_simd": v[0].value,
                         "vgprs": v[1].value, "lds_bytes": v[3].value}
        return out

    # -- render('rgb_array') (TG/:98-105; DR/ draw_domain) ---------------------------------------
    def render_init(self, sprites=None):
        """Load the sprite sheet (uint8 [24, h, w, 4] RGBA, ``render.load_sprites`` /
        ``render.synthetic_sprites``; default: the installed reference's sprites)."""
        from . import render as R
        if sprites is None:
            sprites = R.load_sprites()
        sheet = np.ascontiguousarray(sprites, np.uint8)
        if sheet.ndim != 4 or sheet.shape[0] != _lib.TG_SPR_COUNT or sheet.shape[3] != 4:
            raise ValueError("sprite sheet must be uint8 [%d, h, w, 4]" % _lib.TG_SPR_COUNT)
        check(self._L.tg_render_init(self.handle, sheet.ctypes.data_as(ctypes.c_void_p),
                                     sheet.shape[2], sheet.shape[1]), "tg_render_init")
        h, w = ctypes.c_int32(), ctypes.c_int32()
        check(self._L.tg_frame_shape(self.handle, ctypes.byref(h), ctypes.byref(w)),
              "tg_frame_shape")
        self.frame_shape = (h.value, w.value, 3)

    def render(self, first=0, count=None, out=None):
        """render('rgb_array') of envs [first, first+count): uint8 [count, H*48, W*48, 3]
        on the device (the reference's ``rgb`` array per env, TG/:103-105)."""
        if getattr(self, "frame_shape", None) is None:
            self.render_init()
        count = self.num_envs - first if count is None else int(count)
        if out is None:
            out = torch.empty((count,) + self.frame_shape, dtype=torch.uint8, device=self.device)
        elif (out.dtype != torch.uint8 or not out.is_contiguous() or out.device != self.device
              or tuple(out.shape) != (count,) + self.frame_shape):
            raise ValueError("out must be a contiguous uint8 [%d, %d, %d, 3] tensor on %s"
                             % ((count,) + self.frame_shape[:2] + (self.device,)))
        check(self._L.tg_render(self.handle, int(first), count, _ptr(out), self._stream()),
              "tg_render")
        return out

    STATE_KEYS = ("pos", "flags", "objs", "ang", "mt", "mt_pos", "ep")

    def read_state(self, mt=False):
        """Host copy of the SoA state (checkpoints / tests); ``mt=True`` adds each env's
        ``random.getstate()`` equivalent (624 MT words + index)."""
        n = self.num_envs
        out = {"pos": np.zeros((n, 2), np.int32), "flags": np.zeros(n, np.uint32),
               "objs": np.zeros((n, 4), np.int32), "ang": np.zeros((n, 2), np.float64),
               "mt_pos": np.zeros(n, np.uint32), "ep": np.zeros((n, 2), np.int32)}
        if mt:
            out["mt"] = np.zeros((n, 624), np.uint32)

        def p(k):
            return out[k].ctypes.data_as(ctypes.c_void_p) if k in out else None

        check(self._L.tg_read_state(self.handle, *[p(k) for k in self.STATE_KEYS]),
              "tg_read_state")
        return out

    def write_state(self, state):
        """Restore a ``read_state(mt=True)`` snapshot (same num_envs): every env continues
        bit-exactly from it."""
        n = self.num_envs
        shapes = {"pos": (n, 2), "flags": (n,), "objs": (n, 4), "ang": (n, 2), "mt": (n, 624),
                  "mt_pos": (n,), "ep": (n, 2)}
        dt = {"pos": np.int32, "flags": np.uint32, "objs": np.int32, "ang": np.float64,
              "mt": np.uint32, "mt_pos": np.uint32, "ep": np.int32}
        arrs = {}
        for k in self.STATE_KEYS:
            if k not in state:
                if k == "ep":
                    continue
                raise KeyError("state lacks %r (use read_state(mt=True))" % k)
            a = np.ascontiguousarray(state[k], dt[k])
            if a.shape != shapes[k]:
                raise ValueError("state[%r] has shape %s, expected %s" % (k, a.shape, shapes[k]))
            arrs[k] = a
        torch.cuda.synchronize(self.device)
        check(self._L.tg_write_state(self.handle, *[arrs[k].ctypes.data_as(ctypes.c_void_p)
                                                    if k in arrs else None
                                                    for k in self.STATE_KEYS]), "tg_write_state")

    def save(self, path):
        """Checkpoint every env's state (np.savez)."""
        np.savez(path, **self.read_state(mt=True))

    def load(self, path):
        """Resume from a ``save`` checkpoint."""
        with np.load(path) as z:
            self.write_state({k: z[k] for k in z.files})


class GpuOption:
    """One entry of ``TreasureGame.option_list``: the reference's option object
    (``_Option`` / ``*_option``, _option.py:8-36, _move_options.py; create_options,
    _treasure_game_impl.py:484-498) for an env that lives on the GPU.

    ``can_run()`` is the device's ``can_run`` of this option for the env's current state, and
    ``run()`` runs it to completion on the device, exactly as ``TreasureGame.step(k)`` does
    (``option_list[k].run()``, TG/:91-96): it returns the summed tick rewards, or ``None``
    when the option cannot run (OP/:20-23).  ``done`` is True after a run, as in the reference.
    The per-tick ``policy_step`` is not exposed: the option's loop runs inside one kernel."""

    def __init__(self, env, k):
        self._env = env
        self.index = k
        self.name = OPTION_NAMES[k]
        self.done = False

    def can_run(self):
        return bool(self._env._mask_bits() >> self.index & 1)

    def run(self):
        r = self._env._run(self.index)[1]
        self.done = r is not None or self.done
        return r

    def __repr__(self):
        return "<%s (GPU)>" % self.name


class _GlobalMT:
    """The global ``random``'s MT19937 state read and written in place.

    ``random.getstate()`` + packing and unpacking + ``random.setstate`` cost ~50 us per call
    (a 625-int tuple each way); the drop-in exchanges the state every call.  CPython 3's
    ``_random.Random`` object is ``{PyObject_HEAD; int index; uint32_t state[624];}``
    (Modules/_randommodule.c), so two ``memmove`` of 2.5 KB do the same job, and
    ``gauss_next`` is the Python-level attribute ``random.Random`` keeps.  Enabled only after
    the layout is checked against ``random.getstate()`` (type sizes and the words, both
    directions); otherwise ``ok`` is False and the tuple path runs."""

    def __init__(self):
        self.ok = False
        try:
            self.ok = self._check()
        except Exception:
            self.ok = False

    def _check(self):
        inst = random._inst
        base_t = type(inst).__mro__[-2]  # _random.Random, the C base
        head = object.__basicsize__
        if base_t.__basicsize__ < head + 4 + 4 * 624:
            return False
        self._inst = inst
        self._index = head
        self._state = head + 4
        probe = random.getstate()
        try:
            random.random()  # a state whose index is not 0 or 624
            st = random.getstate()
            ps = _lib.PyState()
            self.load(ps)
            if list(ps.mt) + [ps.index] != list(st[1]):
                return False
            ps.mt[0] ^= 1  # round trip: a store must be what setstate would give
            self.store(ps)
            if random.getstate()[1] != tuple(list(ps.mt) + [ps.index]):
                return False
        finally:
            random.setstate(probe)
        return True

    def load(self, ps):
        base = id(self._inst)
        ctypes.memmove(ctypes.addressof(ps.mt), base + self._state, 4 * 624)
        ps.index = ctypes.c_int.from_address(base + self._index).value
        g = self._inst.gauss_next
        ps.has_gauss = g is not None
        ps.gauss_next = 0.0 if g is None else g

    def store(self, ps):
        base = id(self._inst)
        ctypes.memmove(base + self._state, ctypes.addressof(ps.mt), 4 * 624)
        ctypes.c_int.from_address(base + self._index).value = ps.index
        self._inst.gauss_next = ps.gauss_next if ps.has_gauss else None


_GLOBAL_MT = _GlobalMT()


class TreasureGame:
    """Drop-in for the reference ``TreasureGame`` (treasure_game.py:54-114), one env on the GPU.

    Same surface and Python types: ``reset() -> list[9]``, ``step(a) -> (list[9], int | None,
    bool, {})``, ``available_mask`` (np int array [9]), ``action_space`` Discrete(9),
    ``observation_space`` Box(0, 1, (9,), float32), ``option_names``.

    Random numbers, as in the reference, come by default from Python's process-global
    ``random`` (IM/:2, OB/:9 draw from the module-level ``random``): the constructor's build,
    ``reset`` and ``step`` (and ``option.run``) each read ``random.getstate()``, draw on the
    device (tg_step1_py / tg_reset1_py: one launch, one synchronisation) and store the advanced
    state back with ``random.setstate``, so ``random.seed(s); env = TreasureGame()`` replays
    the reference env draw for draw, and user code that takes its own ``random`` draws in
    between (any of them: random(), randrange, gauss, ...) sees and shapes the same shared
    stream as with the reference.  ``TreasureGame(seed=s)`` instead gives the env a private
    stream equal to ``random.seed(s); TreasureGame()`` in a fresh reference process, and leaves
    the global ``random`` untouched (``share_global_random=False`` with ``seed=None`` draws
    that seed from the global stream).
    ``render(mode='rgb_array')`` returns the frame as a uint8 numpy array [624, 672, 3]
    (TG/:98-105; the sprites are the installed reference's unless ``sprites=`` is given);
    ``mode='human'`` needs gym's image viewer and raises.
    """

    metadata = {"render.modes": ["human", "rgb_array"]}

    def __init__(self, seed=None, device=None, level_dir=None, sprites=None,
                 share_global_random=None):
        self._sprites = sprites
        if share_global_random is None:
            share_global_random = seed is None
        self._shared = bool(share_global_random)
        if self._shared and seed is not None:
            raise ValueError("share_global_random draws from the global random: no seed")
        if seed is None:
            seed = 0 if self._shared else random.getrandbits(64)
        seed = abs(int(seed))  # random.seed(s) keys on abs(s) (CPython random_seed)
        if seed >= 2**64:
            raise ValueError("seed must satisfy |seed| < 2**64 (a two-word init_by_array key)")
        self._vec = TreasureGameVec(1, seed=seed, device=device, level_dir=level_dir)
        self.option_list = [GpuOption(self, k) for k in range(_lib.NUM_ACTIONS)]
        self.option_names = list(OPTION_NAMES)
        self.action_space = Discrete(_lib.NUM_ACTIONS)
        self.observation_space = Box(np.float32(0.0), np.float32(1.0), shape=(_lib.OBS_DIM,))
        self.viewer = None
        self._h_obs = np.zeros(_lib.OBS_DIM, np.float64)  # tg_step1's host outputs
        self._h_rew, self._h_valid, self._h_done = ctypes.c_int32(), ctypes.c_uint8(), ctypes.c_uint8()
        # the step call's arguments, made once: a step is one C call and nothing else.  Its
        # stream is the null stream: every TreasureGame call returns host data, so none of this
        # env's device work is pending when a step starts.
        self._h_mask = ctypes.c_uint16()
        self._p_mask = ctypes.byref(self._h_mask)
        self._step_args = (self._h_obs.ctypes.data, ctypes.byref(self._h_rew),
                           ctypes.byref(self._h_valid), ctypes.byref(self._h_done), None)
        # the shared stream's step works in place on the global random.Random's own words and
        # index (tg_step1_pywords; _GlobalMT checked the layout): no getstate / setstate
        self._pywords = None
        if share_global_random and _GLOBAL_MT.ok:
            base = id(_GLOBAL_MT._inst)
            self._pywords = (base + _GLOBAL_MT._state, base + _GLOBAL_MT._index)
        if self._shared:
            self._py = _lib.PyState()
            # _TreasureGameImpl.__init__'s build draws from the global stream (IM/:31-53)
            self._reset_py(self._h_obs)

    # -- the reference's shared module-level random stream (default) -----------------------------
    _WORDS = struct.Struct("625I")  # tg_pystate's mt[624] + index

    def _load_global(self):
        if _GLOBAL_MT.ok:
            _GLOBAL_MT.load(self._py)
            return None
        st = random.getstate()
        self._WORDS.pack_into(self._py, 0, *st[1])
        g = st[2]
        self._py.has_gauss = g is not None
        self._py.gauss_next = 0.0 if g is None else g
        return st

    def _store_global(self):
        if _GLOBAL_MT.ok:
            _GLOBAL_MT.store(self._py)
            return
        random.setstate((3, self._WORDS.unpack_from(self._py, 0),
                         self._py.gauss_next if self._py.has_gauss else None))

    def _reset_py(self, obs):
        st = self._load_global()
        if st is None:  # in-place load: the replay's start state from the words just loaded
            st = (3, self._WORDS.unpack_from(self._py, 0),
                  self._py.gauss_next if self._py.has_gauss else None)
        check(self._vec._L.tg_reset1_py(self._vec.handle, ctypes.byref(self._py),
                                        obs.ctypes.data, self._vec._stream()), "tg_reset1_py")
        # The reset's draws (IM/:55-73): two uniform(), then gauss twice.  Their stream position
        # is the device's; gauss_next, the cached half of a gauss pair, is left in the global
        # state where user code can read it, so it must be CPython's own sin(x2pi) * g2rad
        # (glibc), not the device's (OCML; they may differ in the last ulp): the same calls are
        # replayed on a private Random from the state the reset started from.
        r = random.Random()
        r.setstate(st)
        r.random()
        r.random()
        r.gauss(0.0, 1.0)
        r.gauss(0.0, 1.0)
        out = r.getstate()
        if out[1] != self._WORDS.unpack_from(self._py, 0):
            raise TgError("tg_reset1_py: the device's stream position differs from CPython's")
        random.setstate(out)

    def reset(self):
        if self._shared:
            self._reset_py(self._h_obs)
            return self._h_obs.tolist()
        # tg_reset1: through the resident server (a reset between episodes does not stop it)
        v = self._vec
        check(v._L.tg_reset1(v.handle, self._h_obs.ctypes.data, None), "tg_reset1")
        return self._h_obs.tolist()

    def _mask_bits(self):
        # tg_available_mask1: through the resident server (a mask read between steps does not
        # stop it); the null stream, as the step
        v = self._vec
        rc = v._L.tg_available_mask1(v.handle, self._p_mask, None)
        if rc:
            check(rc, "tg_available_mask1")
        return int(self._h_mask.value) & 0x1FF

    @property
    def available_mask(self):
        m = self._mask_bits()
        return np.array([(m >> k) & 1 for k in range(_lib.NUM_ACTIONS)])

    def _run(self, a):
        """option_list[a].run() on the device + get_state + done (TG/:91-96): tg_step1 (or
        tg_step1_py over the global stream), one launch whose kernel writes the row into
        pinned host memory, one synchronisation"""
        v = self._vec
        if self._pywords is not None and random._inst is _GLOBAL_MT._inst:
            rc = v._L.tg_step1_pywords(v.handle, a, *self._pywords, *self._step_args)
            if rc:
                check(rc, "tg_step1_pywords")
        elif self._shared:
            self._load_global()
            check(v._L.tg_step1_py(v.handle, a, ctypes.byref(self._py), *self._step_args),
                  "tg_step1_py")
            self._store_global()
        else:
            rc = v._L.tg_step1(v.handle, a, *self._step_args)
            if rc:
                check(rc, "tg_step1")
        r = int(self._h_rew.value) if self._h_valid.value else None
        return self._h_obs.tolist(), r, bool(self._h_done.value)

    def step(self, action):
        a = operator.index(action)  # list indexing accepts ints only (TG/:92)
        if not -_lib.NUM_ACTIONS <= a < _lib.NUM_ACTIONS:
            raise IndexError("list index out of range")
        state, r, done = self._run(a)
        return state, r, done, {}

    def render(self, mode="human"):
        if mode != "rgb_array":
            raise NotImplementedError("render(mode=%r): only 'rgb_array' (no display / gym "
                                      "image viewer here, TG/:106-110)" % (mode,))
        if getattr(self._vec, "frame_shape", None) is None:
            self._vec.render_init(self._sprites)
        return self._vec.render().cpu().numpy()[0]

    def close(self):
        if self.viewer is not None:
            self.viewer = None
        self._vec.close()


class ObservationWrapper:
    """The reference's ``ObservationWrapper`` (treasure_game.py:38-51): reset / step return the
    rendered screen instead of the state vector, and step's info carries the state as
    ``info['world_state']``.

    Over a ``TreasureGame`` the screen is a uint8 numpy array [624, 672, 3], as in the
    reference.  Over a ``TreasureGameVec`` it is the batch's frames, a uint8 device tensor
    [N, 624, 672, 3] rendered by one kernel launch into a buffer the wrapper owns
    (overwritten each call), and step returns ``(frames, reward, valid, done, info)``.
    """

    def __init__(self, env, sprites=None):
        self.env = env
        self._vec = isinstance(env, TreasureGameVec)
        if self._vec:
            env.render_init(sprites)
            self._frames = torch.empty((env.num_envs,) + env.frame_shape, dtype=torch.uint8,
                                       device=env.device)
        else:
            if sprites is not None:
                env._sprites = sprites
            # every step renders, and a render (a full-GPU kernel) stops the resident N = 1
            # server: one launch per step costs less than a server stop + relaunch per step
            env._vec.set_serve(False)
        self.action_space = env.action_space
        self.observation_space = env.observation_space

    def __getattr__(self, name):
        return getattr(self.env, name)

    def _screen(self):
        if self._vec:
            return self.env.render(out=self._frames)
        return self.env.render(mode="rgb_array")

    def reset(self, **kwargs):
        self.env.reset(**kwargs)
        return self._screen()

    def step(self, action):
        out = self.env.step(action)
        info = out[-1]
        info["world_state"] = out[0]
        return (self._screen(),) + tuple(out[1:])


class TreasureGameVectorEnv:
    """Gymnasium-style vector env over one ``TreasureGameVec``: the batch steps
    on the device and every output is a device tensor.

    ``reset(seed=None) -> (obs f64 [N, 9], info)``; ``step(actions) -> (obs, reward f32 [N],
    terminated bool [N], truncated bool [N], info)``.  Auto-reset is same-step
    (``metadata["autoreset_mode"] == "SameStep"``): an env that terminates (TG/:95: gold held
    and back in row 0) or is truncated is reset inside the same call, ``obs`` holds its new
    episode's first observation and ``info["final_obs"]`` the last one of the finished
    episode (== ``obs`` for the others).  The reference's ``None`` reward (option could not run,
    OP/:22-23) is reward 0 with ``info["valid"] == 0``.  ``truncated`` is set only when
    ``max_episode_steps`` is given (the reference registers no TimeLimit); those envs are reset
    by a masked ``tg_reset`` on the device, with no host synchronisation.
    Env g of ``reset(seed=s)`` is ``random.seed(s + g); TreasureGame()`` (contract of
    TreasureGameVec)."""

    metadata = {"autoreset_mode": "SameStep", "render_modes": ["rgb_array"]}

    def __init__(self, num_envs, seed=0, device=None, max_episode_steps=None, level_dir=None,
                 mode="compact"):
        self.num_envs = int(num_envs)
        self._kw = dict(device=device, level_dir=level_dir, mode=mode)
        self.max_episode_steps = None if max_episode_steps is None else int(max_episode_steps)
        self.single_action_space = Discrete(_lib.NUM_ACTIONS)
        self.single_observation_space = Box(np.float32(0.0), np.float32(1.0),
                                            shape=(_lib.OBS_DIM,))
        self.action_space = MultiDiscrete([_lib.NUM_ACTIONS] * self.num_envs)
        self.observation_space = Box(np.float32(0.0), np.float32(1.0),
                                     shape=(self.num_envs, _lib.OBS_DIM))
        self._make(seed)

    def _make(self, seed):
        old = getattr(self, "env", None)
        if old is not None:
            old.close()
        # copy=True: every returned tensor is the caller's own (gymnasium loops keep obs across
        # steps: obs_t must not change when the next step writes the library's buffers)
        self.env = TreasureGameVec(self.num_envs, seed=seed, autoreset=True, copy=True, **self._kw)
        self.device = self.env.device
        self._len = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)

    def reset(self, seed=None, options=None):
        if seed is not None:
            self._make(int(seed))
        obs = self.env.reset()
        self._len.zero_()
        return obs, {}

    def step(self, actions):
        obs, rew, valid, done, info = self.env.step(actions)
        final = info["final_obs"]
        terminated = done.bool()
        self._len += 1
        self._len.masked_fill_(terminated, 0)
        if self.max_episode_steps is not None:
            truncated = self._len >= self.max_episode_steps
            self._len.masked_fill_(truncated, 0)
            obs = self.env.reset(truncated.to(torch.uint8))  # masked reset, obs of every env
        else:
            truncated = torch.zeros_like(terminated)
        return obs, rew.to(torch.float32), terminated, truncated, {"final_obs": final,
                                                                   "valid": valid}

    def available_mask(self):
        return self.env.available_mask()

    def episodes(self, cap=None):
        """(env, return, length) of the terminated episodes (device queue, TreasureGameVec)"""
        return self.env.episodes(cap)

    def close(self):
        self.env.close()


def make_vec(id="treasure_game-v0", num_envs=1, **kwargs):
    """gymnasium.make_vec stand-in: a TreasureGameVectorEnv of ``num_envs`` envs."""
    if id != "treasure_game-v0":
        raise KeyError("unknown env id %r" % (id,))
    return TreasureGameVectorEnv(num_envs, **kwargs)
