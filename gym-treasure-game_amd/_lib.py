"""ctypes binding of libtg_amd.so (the C ABI declared in include/tg_amd.h).

The library is built in-tree (``python -m gym_treasure_game_amd.build`` or
``__graft_entry__.build()``) and travels with the repository.  There is no CPU fallback: if
the library is missing or no gfx950 device is present, every entry point raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# TG_LIB_PATH: an A/B variant build (scripts/build_variant.py) in place of the product library
LIB_PATH = os.environ.get("TG_LIB_PATH") or os.path.join(HERE, "libtg_amd.so")

TG_OK = 0
TG_STEP_AUTORESET = 1
TG_POLICY_UNIFORM = 0
TG_POLICY_MASKED = 1
TG_MODE_DIRECT = 0
TG_MODE_COMPACT = 1
TG_MODE_FLOW = 2
TG_ERR_TICKCAP = 1 << 24
TG_ERR_BAG = 1 << 25
TG_ERR_ACTION = 1 << 26
TG_ERR_NEARINT = 1 << 27
TG_ERR_RENDER = 1 << 28
TG_ERR_WINDOW = 1 << 29
TG_ERR_FLOW = 1 << 30
TG_SPR_COUNT = 24
OBS_DIM = 9
NUM_ACTIONS = 9

# every symbol include/tg_amd.h declares (tests check the library exports all of them)
EXPORTS = ("tg_create", "tg_destroy", "tg_num_envs", "tg_reset", "tg_step", "tg_step1", "tg_step1_py",
           "tg_reset1_py", "tg_set_serve", "tg_step1_pywords", "tg_available_mask1", "tg_reset1", "tg_rollout", "tg_set_groups",
           "tg_available_mask",
           "tg_observe", "tg_policy_actions", "tg_episodes", "tg_errors", "tg_set_mode", "tg_set_timing", "tg_regenerate",
           "tg_set_episode_capacity", "tg_predicate_table",
           "tg_get_stats", "tg_stats_reset", "tg_kernel_info", "tg_mt_layout", "tg_probe_dispatch", "tg_read_state", "tg_write_state", "tg_render_init", "tg_frame_shape",
           "tg_render", "tg_last_error", "tg_version")


class TgError(RuntimeError):
    pass


class Episode(ctypes.Structure):
    _fields_ = [("env", ctypes.c_int64), ("ret", ctypes.c_int32), ("len", ctypes.c_int32)]


class PyState(ctypes.Structure):
    """tg_pystate: random.getstate()'s (624 words, index, gauss_next)"""
    _fields_ = [("mt", ctypes.c_uint32 * 624), ("index", ctypes.c_uint32),
                ("has_gauss", ctypes.c_uint32), ("gauss_next", ctypes.c_double)]


class Stats(ctypes.Structure):
    _fields_ = [("steps", ctypes.c_int64), ("valid_steps", ctypes.c_int64),
                ("ticks", ctypes.c_int64), ("draws", ctypes.c_int64),
                ("episodes", ctypes.c_int64), ("episodes_dropped", ctypes.c_int64),
                ("launches", ctypes.c_int64),
                ("kernel_ms", ctypes.c_double), ("regens", ctypes.c_int64),
                ("wave_ticks", ctypes.c_int64), ("timed_launches", ctypes.c_int64),
                ("run_ms", ctypes.c_double), ("regen_ms", ctypes.c_double),
                ("regen_timed", ctypes.c_int64), ("regen_launches", ctypes.c_int64),
                ("classify_ms", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def load():
    """Load libtg_amd.so and declare every signature. Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise TgError("libtg_amd.so is not built (%s); run __graft_entry__.build() or "
                      "python -m gym_treasure_game_amd.build" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P, i32, i64, u32, u64 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                             ctypes.c_uint64)
    sig = {
        "tg_create": (i32, [ctypes.POINTER(P), i64, u64, i64, i32, ctypes.c_char_p,
                            ctypes.c_char_p, ctypes.c_char_p]),
        "tg_destroy": (None, [P]),
        "tg_num_envs": (i64, [P]),
        "tg_reset": (i32, [P, P, P, P]),
        "tg_step": (i32, [P, P, P, P, P, P, P, u32, P]),
        "tg_step1": (i32, [P, i32, P, P, P, P, P]),
        "tg_step1_py": (i32, [P, i32, P, P, P, P, P, P]),
        "tg_reset1_py": (i32, [P, P, P, P]),
        "tg_set_serve": (i32, [P, i32]),
        "tg_step1_pywords": (i32, [P, i32, P, P, P, P, P, P, P]),
        "tg_available_mask1": (i32, [P, P, P]),
        "tg_reset1": (i32, [P, P, P]),
        "tg_rollout": (i32, [P, i32, u64, i64, i32, u32, P, P, P, P, P, P]),
        "tg_available_mask": (i32, [P, P, P]),
        "tg_observe": (i32, [P, P, P]),
        "tg_policy_actions": (i32, [P, u64, i64, i32, P, P]),
        "tg_episodes": (i32, [P, P, P, i32, P]),
        "tg_errors": (i32, [P, ctypes.POINTER(u32), P]),
        "tg_set_mode": (i32, [P, i32, i32]),
        "tg_set_timing": (i32, [P, i32]),
        "tg_regenerate": (i32, [P, P]),
        "tg_set_episode_capacity": (i32, [P, i32]),
        "tg_predicate_table": (i32, [P, i32, i32, i32, i32, u32, P, P]),
        "tg_get_stats": (i32, [P, ctypes.POINTER(Stats)]),
        "tg_stats_reset": (i32, [P]),
        "tg_set_groups": (i32, [P, i32, i32]),
        "tg_mt_layout": (i32, [ctypes.POINTER(ctypes.c_int32)] * 3),
        "tg_probe_dispatch": (i32, [i32, i32, P]),
        "tg_kernel_info": (i32, [P, i32, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                 ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
        "tg_read_state": (i32, [P, P, P, P, P, P, P, P]),
        "tg_write_state": (i32, [P, P, P, P, P, P, P, P]),
        "tg_render_init": (i32, [P, P, i32, i32]),
        "tg_frame_shape": (i32, [P, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "tg_render": (i32, [P, i64, i64, P, P]),
        "tg_last_error": (ctypes.c_char_p, []),
        "tg_version": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("TG_AB_LIB") and not hasattr(L, name):
            continue  # scripts/ab.py times earlier builds, which may lack newer entry points
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc, what):
    if rc != TG_OK:
        msg = load().tg_last_error()
        raise TgError("%s failed (%d): %s" % (what, rc, msg.decode() if msg else ""))
