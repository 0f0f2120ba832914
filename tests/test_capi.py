"""The drop-in boundary: libtg_amd.so loads and exports every entry point include/tg_amd.h
declares, and fails loudly (never silently) without a gfx950 device."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tg_amd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = header_functions()
    for must in ("tg_create", "tg_reset", "tg_step", "tg_available_mask", "tg_destroy"):
        assert must in names


def test_library_exports_every_declared_symbol(tg):
    lib = tg._lib.load()
    names = header_functions()
    assert sorted(tg._lib.EXPORTS) == names
    out = subprocess.check_output(["nm", "-D", "--defined-only", tg._lib.LIB_PATH]).decode()
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert getattr(lib, n) is not None
    assert lib.tg_version().decode().endswith("gfx950")


def test_library_has_gfx950_code_object(tg):
    blob = open(tg._lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the .hip_fatbin bundle id


def test_library_links_the_flow_unit(tg):
    """k_flow comes from its own unit (csrc/tg_flow.hip, built without MachineLICM): the
    library exports its handle accessor, and the build compiles that unit with FLOW_FLAGS and
    links the object with the other sources."""
    out = subprocess.check_output(["nm", "-D", "--defined-only", tg._lib.LIB_PATH]).decode()
    assert any("flow_kernel" in ln for ln in out.splitlines())
    from gym_treasure_game_amd import build as B
    calls = []
    orig = B.subprocess.check_call
    B.subprocess.check_call = lambda cmd: calls.append(cmd)
    try:
        B.compile_lib("/tmp/never_built.so")
    finally:
        B.subprocess.check_call = orig
    flow, lib = calls
    assert flow[-1].endswith("tg_flow.hip") and "-c" in flow
    assert " ".join(B.FLOW_FLAGS) in " ".join(flow) and " ".join(B.FLOW_FLAGS) not in " ".join(lib)
    assert lib[-3:] == ["-x", "none", "/tmp/never_built.so.flow.o"]
    assert any(a.endswith("tg_amd.hip") for a in lib) and "-shared" in lib


def test_bad_level_is_rejected_before_touching_a_device(tg):
    lib = tg._lib.load()
    h = ctypes.c_void_p()
    rc = lib.tg_create(ctypes.byref(h), 4, 0, 0, 0, b"////\n/  /\n////\n", b"door 1 1 True\n",
                       b"")
    assert rc == -1  # TG_E_INVAL: roster incomplete
    assert b"roster" in lib.tg_last_error()
    rc = lib.tg_create(ctypes.byref(h), 4, 0, 0, 0, b"x", None, None)
    assert rc == -1
    rc = lib.tg_create(ctypes.byref(h), 0, 0, 0, 0, None, None, None)
    assert rc == -1


def test_cascade_draw_bound_is_checked_at_parse(tg):
    """One INTERACT tick's random() draws are bounded per level from its trigger table
    (tg_level.h interact_draw_bound): the cascade level's 10-draw ticks parse (TG_E_NODEV here,
    no GPU: parsing comes first); a table whose cascades could draw more than the code window
    stages is rejected with a message, not run past the window."""
    lib = tg._lib.load()
    lv = os.path.join(ROOT, "tests", "golden", "levels", "cascade")
    texts = [open(os.path.join(lv, f), "rb").read()
             for f in ("domain.txt", "domain-objects.txt", "domain-interactions.txt")]
    h = ctypes.c_void_p()
    rc = lib.tg_create(ctypes.byref(h), 4, 0, 0, 0, *texts)
    assert rc in (0, -4), lib.tg_last_error()
    if rc == 0:
        lib.tg_destroy(h)
    # handle 0 toggles door 0 seven times, door 0 toggles handle 1 seven times per change
    alt = lambda src, dst: "".join("%s %s %s\n" % (src, dst, ("True", "False")[k % 2])
                                   for k in range(7))
    inter = ("".join(alt("handle 0 %s" % p, "door 0") for p in ("True", "False")) +
             "".join(alt("door 0 %s" % p, "handle 1") for p in ("True", "False")) +
             "".join(alt("handle 1 %s" % p, "door 1") for p in ("True", "False")) +
             "".join(alt("door 1 %s" % p, "handle 0") for p in ("True", "False")))
    rc = lib.tg_create(ctypes.byref(h), 4, 0, 0, 0, texts[0], texts[1], inter.encode())
    assert rc == -1
    assert b"INTERACT tick" in lib.tg_last_error()


def test_no_device_fails_loudly(tg):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = tg._lib.load()
    h = ctypes.c_void_p()
    rc = lib.tg_create(ctypes.byref(h), 4, 0, 0, 0, None, None, None)
    assert rc == -4  # TG_E_NODEV
    assert not h.value
    with pytest.raises(tg.TgError):
        tg.make(num_envs=8)
    with pytest.raises(tg.TgError):
        tg.make(seed=0)
