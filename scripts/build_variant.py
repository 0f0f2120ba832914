#!/usr/bin/env python3
"""Build an A/B variant of libtg_amd.so from the product sources with literal replacements
(diagnostics; the product is built by gym_treasure_game_amd/build.py):

    python scripts/build_variant.py NAME 'old text' 'new text' ['old2' 'new2' ...]

writes gym-treasure-game_amd/libtg_amd_NAME.so (timed by scripts/ab.py).  Every replacement
must match exactly once in one of the csrc files.  EXTRA_FLAGS (environment) is appended to
the compiler flags (e.g. '-mllvm -disable-machine-licm')."""
import os
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gym_treasure_game_amd import build as B  # noqa: E402


def main():
    name, reps = sys.argv[1], sys.argv[2:]
    assert len(reps) % 2 == 0, "pairs of old / new"
    tmp = tempfile.mkdtemp(prefix="tgvar_")
    src = os.path.join(tmp, "pkg", "csrc")
    shutil.copytree(os.path.join(ROOT, "gym-treasure-game_amd", "csrc"), src)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    files = [os.path.join(src, f) for f in os.listdir(src)]
    for old, new in zip(reps[0::2], reps[1::2]):
        hits = [f for f in files if open(f).read().count(old) == 1]
        assert len(hits) == 1, "%r matches in %d files" % (old, len(hits))
        t = open(hits[0]).read().replace(old, new)
        open(hits[0], "w").write(t)
    out = os.path.join(ROOT, "gym-treasure-game_amd", "libtg_amd_%s.so" % name)
    B.compile_lib(out, csrc=src, extra=os.environ.get("EXTRA_FLAGS", "").split())
    shutil.rmtree(tmp)
    print(out)


if __name__ == "__main__":
    main()
