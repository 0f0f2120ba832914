#!/usr/bin/env python3
"""Generate the golden parity fixtures from the reference env (DEV-ONLY, this container only).

This script imports the unmodified reference from /root/reference with minimal ``gym`` /
``pygame`` stand-ins (neither is installed; the physics never touches them, IM/:4 imports
pygame but never calls it) and records what the reference produces.  Only the fixture files
it writes travel with the repo; the reference itself never does.  Nothing in tests/, bench.py
or __graft_entry__ imports this script.

Per-env contract (SURVEY.md §7 "RNG bit-exactness"): env ``g`` behaves like a reference env
in a fresh process after ``random.seed(seed_base + g)``:

    random.seed(s); e = TreasureGame(); e.reset(); e.step(a_0); e.step(a_1); ...

The module-global ``random`` of IM/ and OB/ (IM/:2, OB/:9) is swapped for a private
``random.Random(s)`` subclass that counts ``random()`` calls; ``check_injection`` verifies
that this is draw-for-draw identical to seeding the process-global stream.

Fixture families:
  F1  rng_kat.json        CPython MT19937 KATs: getrandbits(32), random(), uniform, gauss
  F3  traj_uniform.npz    16 envs x 1000 steps, uniform actions (full per-step vectors)
      traj_masked.npz     16 envs x 1500 steps, masked-uniform actions
      traj_autoreset.npz   8 envs x 4000 steps, masked-uniform, reset() after done
  F3h hash_uniform.npz    4096 envs x 1000 steps, per-env rolling hashes (uniform)
      hash_masked.npz     1024 envs x  600 steps, per-env rolling hashes (masked)
  F2  predicates.npz     the 6 collision predicates (IM/:232-288) at every pixel position
                          px in [-24,696), py in [-56,680) with all doors open / all closed
  F5  resets.npz          obs after construct+reset for seeds 0..9999
  F6  traj_level_<L>_{uniform,masked}.npz  16 envs x 400 uniform / 600 masked+auto-reset steps
                          on levels/<L> (corridor, gen1-3: the reference constructor pointed
                          at those files; gen* written by gen_level)

Action streams come from a counter hash (see ``action_hash``), replicated bit-for-bit by
oracle/tg_oracle.c and the device action generator.

Usage:  python tests/golden/make_golden.py [--jobs 8]
"""
import argparse
import json
import os
import random
import struct
import sys
import types
from multiprocessing import Pool

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
M64 = 0xFFFFFFFFFFFFFFFF

ACTION_SEED_UNIFORM = 0x5EED0001
ACTION_SEED_MASKED = 0x5EED0002


# ----------------------------------------------------------------------------------------
# action stream + hash (the same functions exist in oracle/tg_oracle.c and csrc/)
# ----------------------------------------------------------------------------------------
def sm64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def action_hash(a0, g, t):
    return sm64(sm64(a0 ^ sm64(g)) ^ t)


def pick_action(a0, g, t, mask_bits):
    """mask_bits None -> uniform over 0..8; else masked-uniform (k-th set bit)."""
    h = action_hash(a0, g, t)
    if mask_bits is None:
        return h % 9
    c = bin(mask_bits).count("1")
    if c == 0:
        return h % 9
    k = h % c
    for i in range(9):
        if mask_bits >> i & 1:
            if k == 0:
                return i
            k -= 1
    raise AssertionError


def rec_hash(h, obs, reward, valid, done):
    for v in obs:
        h = sm64(h ^ struct.unpack("<Q", struct.pack("<d", v))[0])
    w = (reward & 0xFFFFFFFF) | (valid << 32) | (done << 40)
    return sm64(h ^ w)


# ----------------------------------------------------------------------------------------
# reference import with stand-ins
# ----------------------------------------------------------------------------------------
def _install_stubs():
    gym = types.ModuleType("gym")

    class Env:
        pass

    class Wrapper:
        def __init__(self, env):
            self.env = env

    gym.Env, gym.Wrapper = Env, Wrapper
    spaces = types.ModuleType("gym.spaces")

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Box:
        def __init__(self, low, high, shape=None, dtype=None):
            self.low, self.high, self.shape = low, high, shape

    spaces.Discrete, spaces.Box = Discrete, Box
    envs = types.ModuleType("gym.envs")
    reg = types.ModuleType("gym.envs.registration")
    reg.register = lambda **kw: None
    cc = types.ModuleType("gym.envs.classic_control")
    rendering = types.ModuleType("gym.envs.classic_control.rendering")
    cc.rendering = rendering
    gym.spaces, gym.envs = spaces, envs
    envs.registration, envs.classic_control = reg, cc
    for n, m in [("gym", gym), ("gym.spaces", spaces), ("gym.envs", envs),
                 ("gym.envs.registration", reg), ("gym.envs.classic_control", cc),
                 ("gym.envs.classic_control.rendering", rendering)]:
        sys.modules[n] = m
    pg = types.ModuleType("pygame")
    pg.locals = types.ModuleType("pygame.locals")
    sys.modules["pygame"] = pg
    sys.modules["pygame.locals"] = pg.locals


_install_stubs()
sys.path.insert(0, REF)
from gym_treasure_game.envs import treasure_game as TG  # noqa: E402
from gym_treasure_game.envs._treasure_game_impl import _objects as OB  # noqa: E402
from gym_treasure_game.envs._treasure_game_impl import _treasure_game_impl as IM  # noqa: E402


class CountingRandom(random.Random):
    def __init__(self, seed):
        self.n = 0
        super().__init__(seed)

    def random(self):
        self.n += 1
        return super().random()


_make_path = TG.make_path


def use_level(level_dir):
    """Point the UNMODIFIED TreasureGame constructor (TG/:63-76, which reads
    make_path(dir, 'domain.txt') etc.) at another level's three files: the reference's own
    constructor, reset_game (IM/:55-73, which re-reads the same paths) and loaders run; only
    the paths differ.  None restores the default level."""
    def mp(root, *args):
        if level_dir is not None and args and str(args[-1]).endswith(".txt"):
            return os.path.join(level_dir, str(args[-1]))
        return _make_path(root, *args)
    TG.make_path = mp


def new_env(seed):
    rng = CountingRandom(seed)
    IM.random = rng
    OB.random = rng
    env = TG.TreasureGame()
    obs = env.reset()
    return env, rng, obs


def internal(env):
    """Extended per-step internal state (for debugging mismatches)."""
    md = env._env
    doors = sum(int(d.closed) << i for i, d in enumerate(md.doors))
    handles = sum(int(h.up) << i for i, h in enumerate(md.handles))
    bag = "".join("K" if isinstance(o, OB.key) else "G" for o in md.player_bag)
    keyo = [o for o in md.objects if isinstance(o, OB.key)][0]
    gold = [o for o in md.objects if isinstance(o, OB.goldcoin)][0]
    return [md.playerx, md.playery, md.jump_ticker, doors, handles, int(md.bolts[0].locked),
            keyo.cx, keyo.cy, gold.cx, gold.cy, int(md.facing_right), md.total_actions], bag


def check_injection():
    """Injected per-env Random == process-global random.seed."""
    for s in (0, 7):
        IM.random = random
        OB.random = random
        random.seed(s)
        e = TG.TreasureGame()
        o1 = [e.reset()]
        for t in range(200):
            o1.append(e.step(pick_action(ACTION_SEED_MASKED, s, t, _mask(e)))[:3])
        e2, _, o = new_env(s)
        o2 = [o]
        for t in range(200):
            o2.append(e2.step(pick_action(ACTION_SEED_MASKED, s, t, _mask(e2)))[:3])
        assert o1 == o2, "injection differs from global seeding"
    IM.random = random
    OB.random = random


def _mask(env):
    m = env.available_mask
    return int(sum(int(v) << i for i, v in enumerate(m)))


# ----------------------------------------------------------------------------------------
# F1
# ----------------------------------------------------------------------------------------
def make_rng_kat():
    seeds = [0, 1, 2, 12, 42, 123456789, 2**32 - 1, 2**32, 2**32 + 5, 2**63 + 7, 2**64 - 1]
    out = []
    for s in seeds:
        r = random.Random(s)
        words = [r.getrandbits(32) for _ in range(1300)]  # crosses three twists
        r = random.Random(s)
        rnd = [r.random() for _ in range(700)]
        r = random.Random(s)
        uni = [r.uniform(0.85, 1.0), r.uniform(0, 0.15), r.uniform(0, 1), r.uniform(-4, -2.0),
               r.uniform(2.0, 4)]
        r = random.Random(s)
        gau = []
        for _ in range(16):
            gau.append(r.gauss(0, 48 / 24))
            gau.append(r.gauss(0, 48 / 36))
        out.append({"seed": str(s),
                    "words": words,
                    "random_bits": [struct.unpack("<Q", struct.pack("<d", v))[0] for v in rnd],
                    "uniform_bits": [struct.unpack("<Q", struct.pack("<d", v))[0] for v in uni],
                    "gauss_bits": [struct.unpack("<Q", struct.pack("<d", v))[0] for v in gau]})
    with open(os.path.join(OUT, "rng_kat.json"), "w") as f:
        json.dump({"source": "CPython %s random.Random" % sys.version.split()[0], "kats": out}, f)


# ----------------------------------------------------------------------------------------
# F3 full trajectories
# ----------------------------------------------------------------------------------------
def run_traj(args):
    g, seed, steps, a0, masked, autoreset = args[:6]
    use_level(args[6] if len(args) > 6 else None)
    env, rng, obs = new_env(seed)
    T = steps
    O = np.zeros((T + 1, 9), np.float64)
    R = np.zeros(T + 1, np.int32)
    V = np.zeros(T + 1, np.uint8)
    D = np.zeros(T + 1, np.uint8)
    A = np.zeros(T + 1, np.int32)
    MK = np.zeros(T + 1, np.uint16)
    DR = np.zeros(T + 1, np.int64)
    INT = np.zeros((T + 1, 12), np.int32)
    FO = np.zeros((T + 1, 9), np.float64)
    O[0] = obs
    FO[0] = obs
    DR[0] = rng.n
    INT[0], _ = internal(env)
    MK[0] = _mask(env)
    bags = [internal(env)[1]]
    for t in range(T):
        m = _mask(env)
        a = pick_action(a0, g, t, m if masked else None)
        obs, r, d, _ = env.step(a)
        i = t + 1
        A[i] = a
        FO[i] = obs
        if autoreset and d:
            obs = env.reset()
        O[i] = obs
        R[i] = 0 if r is None else r
        V[i] = r is not None
        D[i] = d
        DR[i] = rng.n
        MK[i] = _mask(env)
        INT[i], b = internal(env)
        bags.append(b)
    return dict(obs=O, reward=R, valid=V, done=D, action=A, mask=MK, draws=DR, internal=INT,
                final_obs=FO, bag=np.array(bags))


def make_traj(name, n_envs, steps, a0, masked, autoreset, jobs, seed0=0, level_dir=None):
    with Pool(jobs) as p:
        res = p.map(run_traj, [(g, seed0 + g, steps, a0, masked, autoreset, level_dir)
                              for g in range(n_envs)])
    out = {k: np.stack([r[k] for r in res]) for k in res[0]}
    out["seed_base"] = np.int64(seed0)
    out["action_seed"] = np.uint64(a0)
    out["masked"] = np.uint8(masked)
    out["autoreset"] = np.uint8(autoreset)
    if level_dir is not None:
        out["level"] = np.array(os.path.basename(level_dir))
    np.savez_compressed(os.path.join(OUT, name), **out)
    return out


# ----------------------------------------------------------------------------------------
# F6 other levels: the reference constructor pointed at non-default level files
# ----------------------------------------------------------------------------------------
DEFAULT_INTERACTIONS = os.path.join(REF, "gym_treasure_game", "envs", "_treasure_game_impl",
                                    "domain-interactions.txt")


def gen_level(seed):
    """A random level in the reference's formats with the reference's object roster (3 doors,
    2 handles, key, bolt, gold; the default interactions file): k corridors between floors,
    ladders (some running up through the corridor above), drop holes, the exit ladder in the
    top wall.  The start is the top wall's ladder cell (the first non-wall cell, IM/:168-178)."""
    r = random.Random(seed)
    W = r.randint(12, 22)
    k = r.randint(4, 7)
    H = 2 * k + 1
    g = [["/"] * W for _ in range(H)]
    for i in range(k):
        row = 1 + 2 * i
        for x in range(1, W - 1):
            g[row][x] = " "
        if r.random() < 0.3:  # an interior wall stub splitting the corridor
            g[row][r.randint(3, W - 4)] = "/"
    g[0][r.randint(1, W - 2)] = "L"
    for i in range(k - 1):
        fl = 2 + 2 * i
        for _ in range(r.randint(1, 2)):
            c = r.randint(1, W - 2)
            g[fl][c] = "L"
            if r.random() < 0.5:
                g[fl - 1][c] = "L"
            if r.random() < 0.3:
                g[fl + 1][c] = "L"
        if r.random() < 0.6:  # a drop hole
            c = r.randint(1, W - 2)
            if g[fl][c] == "/":
                g[fl][c] = " "
    free = [(x, y) for y in range(1, H - 1, 2) for x in range(1, W - 1) if g[y][x] == " "]
    r.shuffle(free)
    cells = free[:8]
    doors, handles, (key, bolt, gold) = cells[:3], cells[3:5], cells[5:8]
    objs = ["door %d %d %s" % (x, y, r.choice(["True", "False"])) for x, y in doors]
    objs += ["handle %d %d %s" % (x, y, r.choice(["True", "False"])) for x, y in handles]
    objs += ["key %d %d" % key, "bolt %d %d True" % bolt, "gold %d %d" % gold]
    dom = "\n".join("".join(row) for row in g) + "\n"
    with open(DEFAULT_INTERACTIONS) as f:
        inter = f.read()
    return dom, "\n".join(objs) + "\n", inter


def make_levels(jobs):
    base = os.path.join(OUT, "levels")
    for i in (1, 2, 3):
        d = os.path.join(base, "gen%d" % i)
        os.makedirs(d, exist_ok=True)
        texts = gen_level(1000 + i)
        for f, t in zip(("domain.txt", "domain-objects.txt", "domain-interactions.txt"), texts):
            with open(os.path.join(d, f), "w") as fh:
                fh.write(t)
        with open(os.path.join(d, "README.md"), "w") as fh:
            fh.write("Generated test level (tests/golden/make_golden.py gen_level(%d)): the "
                     "reference's object roster and\ninteractions on a random layout.  "
                     "traj_level_gen%d_*.npz hold the reference's trajectories on it.\n"
                     % (1000 + i, i))
    # a small hand-made level whose gold lies next to the exit ladder, so that random
    # option sequences finish episodes on a non-default level (auto-reset path)
    d = os.path.join(base, "exit")
    os.makedirs(d, exist_ok=True)
    dom = "////L///////\n/          /\n///////L////\n/       L  /\n////////////\n"
    objs = ("door 9 3 True\ndoor 2 3 False\ndoor 10 1 False\nhandle 6 3 True\n"
            "handle 4 3 False\nkey 1 3\nbolt 3 3 True\ngold 7 1\n")
    with open(DEFAULT_INTERACTIONS) as f:
        inter = f.read()
    for f, t in zip(("domain.txt", "domain-objects.txt", "domain-interactions.txt"),
                    (dom, objs, inter)):
        with open(os.path.join(d, f), "w") as fh:
            fh.write(t)
    with open(os.path.join(d, "README.md"), "w") as fh:
        fh.write("Hand-made test level (not from the reference): the gold lies next to the "
                 "exit ladder, so random option\nsequences finish episodes on a non-default "
                 "level.  traj_level_exit_*.npz hold the reference's\ntrajectories on it.\n")
    for name in ("corridor", "gen1", "gen2", "gen3", "exit"):
        d = os.path.join(base, name)
        make_traj("traj_level_%s_uniform.npz" % name, 16, 400, ACTION_SEED_UNIFORM, False,
                  False, jobs, seed0=0, level_dir=d)
        make_traj("traj_level_%s_masked.npz" % name, 16, 600, ACTION_SEED_MASKED, True, True,
                  jobs, seed0=50, level_dir=d)


def make_cascade_level(jobs):
    """A hand-made level whose trigger table makes one INTERACT tick draw many times: handle
    0's lists toggle door 0 back and forth, door 0's lists toggle handle 1 back and forth, and
    process_trigger clears previously_triggered on return (OB/:76-94), so every toggle changes
    handle 1 again and wiggles it (one draw each): a successful flip of handle 0 draws up to
    10 times.  The layout is the exit level's, so episodes finish."""
    d = os.path.join(OUT, "levels", "cascade")
    os.makedirs(d, exist_ok=True)
    dom = "////L///////\n/          /\n///////L////\n/       L  /\n////////////\n"
    objs = ("door 9 3 True\ndoor 2 3 False\ndoor 10 1 False\nhandle 6 3 False\n"
            "handle 4 3 False\nkey 1 3\nbolt 3 3 True\ngold 7 1\n")
    inter = ("handle 0 True door 0 False\nhandle 0 True door 0 True\n"
             "handle 0 True door 0 False\nhandle 0 True handle 1 False\n"
             "handle 0 False door 0 True\nhandle 0 False door 0 False\n"
             "handle 0 False handle 1 True\n"
             "door 0 False handle 1 True\ndoor 0 False handle 1 False\n"
             "door 0 False handle 1 True\n"
             "door 0 True handle 1 False\ndoor 0 True handle 1 True\n"
             "handle 1 True door 1 True\nhandle 1 False door 1 False\n"
             "bolt 0 True door 2 True\nbolt 0 False door 2 False\n")
    for f, t in zip(("domain.txt", "domain-objects.txt", "domain-interactions.txt"),
                    (dom, objs, inter)):
        with open(os.path.join(d, f), "w") as fh:
            fh.write(t)
    with open(os.path.join(d, "README.md"), "w") as fh:
        fh.write("Hand-made test level (not from the reference): the exit level's layout "
                 "and a trigger table whose\ncascades change one handle many times, so one "
                 "INTERACT tick takes more than 8 random() draws.\n"
                 "traj_level_cascade_*.npz hold the reference's trajectories on it.\n")
    make_traj("traj_level_cascade_uniform.npz", 16, 400, ACTION_SEED_UNIFORM, False, False,
              jobs, seed0=0, level_dir=d)
    make_traj("traj_level_cascade_masked.npz", 16, 600, ACTION_SEED_MASKED, True, True,
              jobs, seed0=50, level_dir=d)


# ----------------------------------------------------------------------------------------
# F3h rolling hashes
# ----------------------------------------------------------------------------------------
def run_hash(args):
    seed, steps, a0, masked = args
    env, rng, obs = new_env(seed)
    h = rec_hash(seed & M64, obs, 0, 0, 0)
    valid_steps = 0
    ticks0 = 0
    ticks = 0
    for t in range(steps):
        a = pick_action(a0, seed, t, _mask(env) if masked else None)
        ticks0 = env._env.total_actions
        obs, r, d, _ = env.step(a)
        ticks += env._env.total_actions - ticks0
        h = rec_hash(h, obs, 0 if r is None else r, int(r is not None), int(d))
        valid_steps += r is not None
    return h, rng.n, valid_steps, ticks


def make_hash(name, n_envs, steps, a0, masked, jobs):
    with Pool(jobs) as p:
        res = p.map(run_hash, [(g, steps, a0, masked) for g in range(n_envs)], chunksize=8)
    np.savez_compressed(os.path.join(OUT, name),
                        hash=np.array([r[0] for r in res], np.uint64),
                        draws=np.array([r[1] for r in res], np.int64),
                        valid_steps=np.array([r[2] for r in res], np.int64),
                        ticks=np.array([r[3] for r in res], np.int64),
                        steps=np.int64(steps), action_seed=np.uint64(a0), masked=np.uint8(masked))


# ----------------------------------------------------------------------------------------
# F2 predicate truth tables
# ----------------------------------------------------------------------------------------
PRED_X0, PRED_X1, PRED_Y0, PRED_Y1 = -24, 696, -56, 680


def run_pred_rows(args):
    door_bits, ys = args
    env, _, _ = new_env(0)
    md = env._env
    for i, d in enumerate(md.doors):
        d.closed = bool(door_bits >> i & 1)
        d.update_map()
    out = np.zeros((len(ys), PRED_X1 - PRED_X0), np.uint8)
    for r, py in enumerate(ys):
        md.playery = py
        for c, px in enumerate(range(PRED_X0, PRED_X1)):
            md.playerx = px
            out[r, c] = (md.up_clear() | md.can_go_up() << 1 | md.can_go_down() << 2 |
                         md.can_go_left() << 3 | md.can_go_right() << 4 | md.can_fall() << 5)
    return out


def make_predicates(jobs):
    ys = list(range(PRED_Y0, PRED_Y1))
    chunks = [ys[i:i + 8] for i in range(0, len(ys), 8)]
    tabs = []
    with Pool(jobs) as p:
        for db in (0, 7):
            tabs.append(np.concatenate(p.map(run_pred_rows, [(db, c) for c in chunks])))
    np.savez_compressed(os.path.join(OUT, "predicates.npz"), table=np.stack(tabs),
                        door_bits=np.array([0, 7], np.uint8),
                        box=np.array([PRED_X0, PRED_X1, PRED_Y0, PRED_Y1], np.int32))


# ----------------------------------------------------------------------------------------
# F5 resets
# ----------------------------------------------------------------------------------------
def make_resets(n=10000):
    O = np.zeros((n, 9), np.float64)
    P = np.zeros((n, 2), np.int32)
    for s in range(n):
        env, rng, obs = new_env(s)
        assert rng.n == 8
        O[s] = obs
        P[s] = (env._env.playerx, env._env.playery)
    np.savez_compressed(os.path.join(OUT, "resets.npz"), obs=O, pos=P)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    check_injection()
    if not only or "kat" in only:
        make_rng_kat()
    if not only or "resets" in only:
        make_resets()
    if not only or "traj" in only:
        make_traj("traj_uniform.npz", 16, 1000, ACTION_SEED_UNIFORM, False, False, a.jobs)
        make_traj("traj_masked.npz", 16, 1500, ACTION_SEED_MASKED, True, False, a.jobs)
        make_traj("traj_autoreset.npz", 8, 4000, ACTION_SEED_MASKED, True, True, a.jobs, seed0=100)
    if not only or "pred" in only:
        make_predicates(a.jobs)
    if not only or "levels" in only:
        make_levels(a.jobs)
    if not only or "cascade" in only:
        make_cascade_level(a.jobs)
    if not only or "hash" in only:
        make_hash("hash_uniform.npz", 4096, 1000, ACTION_SEED_UNIFORM, False, a.jobs)
        make_hash("hash_masked.npz", 1024, 600, ACTION_SEED_MASKED, True, a.jobs)


if __name__ == "__main__":
    main()
