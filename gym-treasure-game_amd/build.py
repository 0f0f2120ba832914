"""Build libtg_amd.so in-tree with hipcc for gfx950.

    python -m gym_treasure_game_amd.build [--force]

The flags matter for parity: -ffp-contract=off keeps uniform()'s a + (b-a)*r and the obs
divisions IEEE-exact (no FMA contraction), and fast-math is never enabled.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", f) for f in ("tg_amd.hip", "tg_render.hip")]
# k_flow's own unit, compiled with FLOW_FLAGS and linked into the same library (tg_flow.hip)
FLOW_SRC = os.path.join(HERE, "csrc", "tg_flow.hip")
FLOW_FLAGS = ["-mllvm", "-disable-machine-licm"]
DEPS = SRCS + [FLOW_SRC] + [os.path.join(HERE, "csrc", f) for f in ("tg_core.h", "tg_level.h", "tg_batch.h",
                                                        "tg_render.h", "tg_twist.h", "tg_flow.h")] + [
    os.path.join(os.path.dirname(HERE), "include", "tg_amd.h")]
OUT = os.path.join(HERE, "libtg_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
         "-fPIC", "-shared", "-Wall", "-Wno-unused-function", "-Wno-bitwise-instead-of-logical"]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def compile_lib(out, csrc=os.path.join(HERE, "csrc"), extra=(), verbose=False):
    """hipcc: tg_flow.hip to an object (FLOW_FLAGS), then the library from tg_amd.hip,
    tg_render.hip and that object, all with FLAGS + extra."""
    obj = out + ".flow.o"
    cflags = [f for f in FLAGS if f != "-shared"] + list(extra)
    cmds = [[HIPCC] + cflags + FLOW_FLAGS + ["-c", "-o", obj, os.path.join(csrc, "tg_flow.hip")],
            [HIPCC] + FLAGS + list(extra) + ["-o", out] +
            [os.path.join(csrc, f) for f in ("tg_amd.hip", "tg_render.hip")] + ["-x", "none", obj]]
    try:
        for cmd in cmds:
            if verbose:
                print(" ".join(cmd))
            subprocess.check_call(cmd)
    finally:
        if os.path.exists(obj):
            os.remove(obj)
    return out


def build(force=False, verbose=False):
    if not force and not needs_build():
        return OUT
    compile_lib(OUT + ".tmp", verbose=verbose)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
