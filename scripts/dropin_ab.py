#!/usr/bin/env python3
"""Interleaved A/B of the N = 1 drop-in's call latency (bench.dropin_latency: TreasureGame.step
on the shared global random stream and on a private one) across library builds, one process
per measurement: VARIANTS="name=lib,..." ROUNDS=3.  Diagnostic, not the product."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = ("import sys, json; sys.path.insert(0, %r); import bench, gym_treasure_game_amd as tg; "
        "print(json.dumps(bench.dropin_latency(tg, steps=2000)))" % ROOT)


def main():
    variants = [v.split("=", 1) for v in os.environ["VARIANTS"].split(",")]
    rounds = int(os.environ.get("ROUNDS", "3"))
    res = {}
    for r in range(rounds):
        for name, lib in variants:
            env = dict(os.environ, TG_LIB_PATH=os.path.join(ROOT, lib))
            out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True,
                                 text=True, timeout=300, check=True).stdout
            d = json.loads(out.strip().splitlines()[-1])
            res.setdefault(name, []).append((d["shared_global_random_step_us"], d["private_stream_step_us"]))
            print(name, "round", r, json.dumps(d), flush=True)
    print(json.dumps({k: {"shared_us": min(a for a, _ in v), "private_us": min(b for _, b in v)}
                      for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
