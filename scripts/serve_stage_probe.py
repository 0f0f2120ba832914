#!/usr/bin/env python3
"""Which GoTable staging the N = 1 server took on a widened level (TG_SERVE_TRACE's report at
tg_destroy: 'GoTable in LDS: <stage>, <bytes> B').  Diagnostic, not the product."""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["TG_SERVE_TRACE"] = "1"
import gym_treasure_game_amd as tg  # noqa: E402

src = os.path.join(ROOT, "tests", "golden", "levels", "gen1")
rows = [r.rstrip("\n") for r in open(os.path.join(src, "domain.txt")) if r.strip()]
extra = 60 - len(rows[0])
wide = [r[:-1] + ("/" if y % 2 == 0 else " ") * extra + r[-1] for y, r in enumerate(rows)]
d = tempfile.mkdtemp()
open(os.path.join(d, "domain.txt"), "w").write("\n".join(wide) + "\n")
for f in ("domain-objects.txt", "domain-interactions.txt"):
    open(os.path.join(d, f), "w").write(open(os.path.join(src, f)).read())
env = tg.TreasureGame(seed=5, level_dir=d)
env.reset()
for t in range(20):
    env.step(t % 9)
env.close()
