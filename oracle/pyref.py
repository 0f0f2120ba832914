"""Pure-Python restatement of the reference step path — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Written for this repository (no reference source is copied): the reference's STRUCTURE in
plain Python, so that timing it on the GPU box's host cores stands in for "the reference
Python step() timed on the box" (BASELINE.json north_star; the reference itself cannot travel
to the box).  Like the reference it keeps an object list with recursive triggers, a list-typed
bag, per-pixel probe loops for the six collision predicates, and draws from a Python
``random.Random`` (CPython's own MT19937, ``uniform``, ``gauss``), and a pixel map built as
the reference builds it (IM/:204-216, OB/:246-253).

Citations (paths under gym_treasure_game/envs/ of the reference):
TG/ treasure_game.py, IM/ _treasure_game_impl/_treasure_game_impl.py, OB/ _objects.py,
MO/ _move_options.py, OP/ _option.py.

Pinned against the reference's own trajectories (tests/test_pyref.py: traj_*.npz).
Only tests/ and bench.py's cpu_baseline leg import this module.
"""
import math
import os
import random
import time

S = 48                       # xscale == yscale (_scale.py)
WALL, OPEN, LADDER, DOOR = "/", " ", "L", "D"
NOP, UP, DOWN, LEFT, RIGHT, JUMP, INTERACT = range(7)   # _actions.py
JUMP_REWARD, STEP_REWARD = -5, -1                        # IM/:15-16
LEVEL_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         "gym-treasure-game_amd", "levels", "default")


# ---- objects (OB/) ---------------------------------------------------------------------------
class Obj:
    """_GameObject (OB/:14-94): cell, pixel position, radius, triggers."""
    kind = "obj"

    def __init__(self, cx, cy):
        self.move_to(cx, cy)
        self.radius = S / 2.0
        self.trig_true, self.trig_false = [], []
        self.previously_triggered = False

    def move_to(self, cx, cy):       # OB/:34-38
        self.cx, self.cy = cx, cy
        self.x, self.y = cx * S, cy * S

    def near_enough(self, x, y):     # OB/:46-53
        cx, cy = self.x + S / 2.0, self.y + S / 2.0
        return math.sqrt(math.pow(x - cx, 2) + math.pow(y - cy, 2)) < self.radius

    def set_trigger(self, val, other, other_val):
        (self.trig_true if val else self.trig_false).append((other, other_val))

    def process_trigger(self, val):  # OB/:76-94
        self.previously_triggered = True
        for other, ov in (self.trig_true if val else self.trig_false):
            if not other.previously_triggered:
                other.set_val(ov)
        self.previously_triggered = False

    def set_val(self, val):
        pass

    def state(self):
        return []


class Door(Obj):
    kind = "door"

    def __init__(self, cx, cy, closed, game):
        super().__init__(cx, cy)
        self.game = game
        self.closed = closed
        self.update_map()

    def update_map(self):            # OB/:246-253: the door's 48x48 pixels
        chars = [DOOR if self.closed else OPEN] * S
        for y in range(S):
            self.game.map[self.cy * S + y][self.cx * S:(self.cx + 1) * S] = chars

    def set_val(self, val):          # OB/:231-235
        if self.closed != val:
            self.closed = val
            self.update_map()
            self.process_trigger(val)


class Handle(Obj):
    kind = "handle"

    def __init__(self, cx, cy, up, rng):
        super().__init__(cx, cy)
        self.rng = rng
        self.up = up
        self.wiggle()                # OB/:111-114
        self.radius = S * 0.75       # OB/:115

    def wiggle(self):                # set_angle_wiggle OB/:127-131
        self.angle = self.rng.uniform(0.85, 1.0) if self.up else self.rng.uniform(0, 0.15)

    def flip(self):                  # OB/:117-122
        if self.rng.uniform(0, 1) <= 0.8:
            self.set_val(not self.up)
        else:
            self.wiggle()

    def set_val(self, val):          # OB/:145-149
        if self.up != val:
            self.up = val
            self.wiggle()
            self.process_trigger(val)

    def state(self):
        return [self.angle]


class Bolt(Obj):
    kind = "bolt"

    def __init__(self, cx, cy, locked):
        super().__init__(cx, cy)
        self.locked = locked

    def set_val(self, val):          # OB/:175-178
        if self.locked != val:
            self.locked = val
            self.process_trigger(val)

    def state(self):
        return [1.0 if self.locked else 0.0]


class Item(Obj):                     # key / goldcoin
    def __init__(self, cx, cy, kind, game):
        super().__init__(cx, cy)
        self.kind = kind
        self.game = game

    def state(self):
        return [float(self.x) / (self.game.W * S), float(self.y) / (self.game.H * S)]


# ---- the game (IM/) -------------------------------------------------------------------------
def read_level(level_dir=None):
    d = level_dir or LEVEL_DIR
    out = []
    for f in ("domain.txt", "domain-objects.txt", "domain-interactions.txt"):
        with open(os.path.join(d, f)) as fh:
            out.append(fh.read())
    return tuple(out)


class Game:
    """_TreasureGameImpl over one Random stream (the reference's module-global random)."""

    def __init__(self, level, rng):
        self.level, self.rng = level, rng
        self.reset_game()

    def reset_game(self):            # IM/:31-73
        dom, objs, inter = self.level
        self.desc = [list(ln.strip()) for ln in dom.split("\n")]
        while self.desc and not self.desc[-1]:
            self.desc.pop()
        self.W, self.H = len(self.desc[0]), len(self.desc)
        self.width, self.height = self.W * S, self.H * S
        self.map = []                # build_map IM/:204-216: one pixel row list per cell row,
        for row in self.desc:        # appended 48 times (the same list, as the reference does)
            px_row = [c for c in row for _ in range(S)]
            self.map += [px_row] * S
        self.objects = []
        for line in objs.split("\n"):  # read_objects IM/:119-166
            w = line.split()
            if not w:
                continue
            cx, cy = int(w[1]), int(w[2])
            if line.startswith("door"):
                self.objects.append(Door(cx, cy, w[3] == "True", self))
            elif line.startswith("key"):
                self.objects.append(Item(cx, cy, "key", self))
            elif line.startswith("bolt"):
                self.objects.append(Bolt(cx, cy, w[3] == "True"))
            elif line.startswith("gold"):
                self.objects.append(Item(cx, cy, "gold", self))
            elif line.startswith("handle"):
                self.objects.append(Handle(cx, cy, w[3] == "True", self.rng))
        lists = {k: [o for o in self.objects if o.kind == k] for k in ("door", "handle", "bolt")}
        for line in inter.split("\n"):  # extract_interactives IM/:75-117
            w = line.split()
            if w:
                lists[w[0]][int(w[1])].set_trigger(w[2] == "True", lists[w[3]][int(w[4])],
                                                   w[5] == "True")
        self.doors, self.handles, self.bolts = lists["door"], lists["handle"], lists["bolt"]
        nx = int(self.rng.gauss(0, S / 24))         # player_initial_position IM/:168-178
        ny = int(abs(self.rng.gauss(0, S / 36)))
        self.px = self.py = 0
        for y in range(self.H):
            xs = [x for x in range(self.W) if self.desc[y][x] != WALL]
            if xs:
                self.px, self.py = xs[0] * S + S // 2 + nx, y * S + ny
                break
        self.bag = []
        self.inc = S // 10
        self.jump_ticker = 0
        self.pw = S // 2
        self.facing_right = True
        self.total_actions = 0

    # map probes (IM/:218-230)
    def at(self, x, y):
        if x >= self.width or x < 0 or y >= self.height or y < 0:
            return WALL
        return self.map[y][x]

    def at_cell(self, xc, yc):
        return self.at(xc * S + S // 2, yc * S + S // 2)

    # the six predicates, pixel loops as in IM/:232-288
    def up_clear(self):
        for xo in (-self.inc, 0, self.inc):
            for yo in range(-self.inc, 0):
                if self.at(self.px + xo, self.py + yo) != OPEN:
                    return False
        return True

    def can_go_up(self):
        if self.py <= 1:
            return False
        for yo in (-self.inc, 0, S - self.inc):
            for xo in (-self.pw // 2, self.pw // 2):
                if self.at(self.px + xo, self.py + yo) == LADDER:
                    return True
        return False

    def can_go_down(self):
        for yo in range(0, S + self.inc):
            for xo in (-self.pw // 2, self.pw // 2):
                if self.at(self.px + xo, self.py + yo) == LADDER:
                    return True
        return False

    def can_go_side(self, d):
        x = self.px + d * (self.pw // 2 + self.inc)
        for yo in (self.inc, S - self.inc):
            t = self.at(x, self.py + yo)
            if t == WALL or t == DOOR:
                return False
        return True

    def can_fall(self):
        for xo in (-self.pw // 2 + 2, -2 + self.pw // 2):
            for yo in (0, S + 2):
                if self.at(self.px + xo, self.py + yo) != OPEN:
                    return False
        return True

    # bag (IM/:402-445)
    def is_object_at(self, xc, yc):
        for o in self.objects:
            if o.cx == xc and o.cy == yc and (o.kind != "door" or o.closed):
                return True
        return False

    def is_closed_door_at(self, xc, yc):
        return any(o.kind == "door" and o.closed and o.cx == xc and o.cy == yc
                   for o in self.objects)

    def got(self, kind):
        return any(o.kind == kind for o in self.bag)

    def drop_key(self):
        for o in self.bag:
            if o.kind == "key":
                self.bag.remove(o)
                o.move_to(-1, -1)
                return

    def cell(self):                  # IM/:441-445
        return self.px // S, (self.py + S // 2) // S

    def noisy(self, val):            # IM/:361-366
        mid = val / 2.0
        if val < mid:
            return int(round(self.rng.uniform(val, mid)))
        return int(round(self.rng.uniform(mid, val)))

    def tick(self, a):               # IM/:290-359
        xd = yd = 0
        self.total_actions += 1
        if a == UP:
            if self.can_go_up():
                yd = self.noisy(-self.inc)
        elif a == DOWN:
            if self.can_go_down():
                yd = self.noisy(self.inc)
        elif a == LEFT:
            if self.can_go_side(-1):
                xd = self.noisy(-self.inc)
                self.facing_right = False
        elif a == RIGHT:
            if self.can_go_side(1):
                xd = self.noisy(self.inc)
                self.facing_right = True
        elif a == JUMP:
            if not self.can_go_down() and self.up_clear():
                self.jump_ticker = 22
                if self.rng.random() > 0.25:
                    self.jump_ticker = 23
        elif a == INTERACT:
            for o in self.objects:
                if o.near_enough(self.px, self.py + S / 2):
                    if o.kind == "handle":
                        o.flip()
                    elif o.kind == "bolt" and self.got("key"):
                        o.set_val(False)  # try_unlock -> unlock
                        self.drop_key()
        if self.jump_ticker > 0:
            if self.up_clear():
                yd = -self.inc
            self.jump_ticker -= 1
        elif self.can_fall():
            self.jump_ticker = 0
            yd = self.inc
        self.px += xd
        if self.can_fall() and yd > 0:
            while yd > 0:
                self.py += 1
                yd -= 1
                if not self.can_fall():
                    yd = 0
        else:
            self.py += yd
        for o in self.objects:
            if o.kind in ("key", "gold") and o.near_enough(self.px, self.py + S / 2):
                o.move_to(self.W - 1 - len(self.bag), self.H - 1)
                self.bag.append(o)
        return JUMP_REWARD if a == JUMP else STEP_REWARD

    def get_state(self):             # IM/:368-378
        s = [float(self.px) / self.width, float(self.py) / self.height]
        for o in self.objects:
            s += o.state()
        return s


# ---- options (MO/, OP/) ---------------------------------------------------------------------
class Option:
    """One of the nine options: can_run / policy_step / run (OP/:20-36)."""

    def __init__(self, g, k):
        self.g, self.k = g, k
        self.target = None

    def _close_x(self, txc):         # MO/:69-72
        return abs(txc * S + S / 2.0 - self.g.px) < self.g.inc

    def _go_target(self, d, xc, yc):  # MO/:43-67, 115-139
        g = self.g
        x = xc + d
        while True:
            if (g.at_cell(x, yc - 1) == LADDER or g.at_cell(x, yc + 1) == LADDER or
                    g.at_cell(x + d, yc) == WALL or g.is_object_at(x, yc) or
                    g.is_closed_door_at(x + d, yc) or g.at_cell(x + d, yc + 1) == OPEN):
                return x
            x += d
            if x < 0:
                return None

    def _landing(self, xc, yc):      # MO/:281-287
        return self.g.at_cell(xc, yc) == OPEN and self.g.at_cell(xc, yc + 1) == WALL

    def can_run(self):
        g, k = self.g, self.k
        xc, yc = g.cell()
        if k in (0, 1):              # MO/:23-41, 95-113
            d = -1 if k == 0 else 1
            tc = self._go_target(d, xc, yc)
            if tc is None:
                return False
            x = xc
            while (x >= tc) if d < 0 else (x <= tc):
                if g.at_cell(x, yc) != OPEN or g.at_cell(x, yc + 1) == OPEN:
                    return False
                x += d
            return True
        if k == 2:
            return g.can_go_up()
        if k == 3:
            return g.can_go_down()
        if k == 4:                   # MO/:446-455
            for o in g.objects:
                if o.near_enough(g.px, g.py + S / 2):
                    if o.kind == "handle" or (o.kind == "bolt" and g.got("key")):
                        return True
            return False
        if k in (5, 6):              # MO/:199-209, 394-404
            d = -1 if k == 5 else 1
            return g.at_cell(xc + d, yc) == OPEN and g.at_cell(xc + d, yc + 1) == OPEN
        d = -1 if k == 7 else 1      # MO/:254-267, 324-337
        return (g.at_cell(xc, yc - 1) == OPEN and g.at_cell(xc + d, yc - 1) == OPEN and
                (self._landing(xc + d, yc - 1) or self._landing(xc + 2 * d, yc - 1)))

    def policy_step(self):
        g, k = self.g, self.k
        if k in (0, 1):              # MO/:74-85
            d = -1 if k == 0 else 1
            if self.target is None:
                xc, yc = g.cell()
                self.target = self._go_target(d, xc, yc)
            if self._close_x(self.target):
                self.done = True
                self.target = None
            return LEFT if d < 0 else RIGHT
        if k == 2:
            if not g.can_go_up():
                self.done = True
                return NOP
            return UP
        if k == 3:
            if not g.can_go_down():
                self.done = True
                return NOP
            return DOWN
        if k == 4:
            self.done = True
            return INTERACT
        if k in (5, 6):              # MO/:211-244
            d = -1 if k == 5 else 1
            if self.target is None:
                xc, yc = g.cell()
                self.target = xc + d
            if self._close_x(self.target):
                if not g.can_fall():
                    self.done = True
                    self.target = None
                return NOP
            return LEFT if d < 0 else RIGHT
        d = -1 if k == 7 else 1      # MO/:269-314
        if self.target is None:
            xc, yc = g.cell()
            self.target = xc + d if self._landing(xc + d, yc - 1) else xc + 2 * d
            return JUMP
        if self._close_x(self.target):
            if not g.can_fall():
                self.done = True
                self.target = None
            return NOP
        if not g.can_fall() and not g.can_go_side(d):
            return RIGHT if d < 0 else LEFT
        return LEFT if d < 0 else RIGHT

    def run(self):                   # OP/:20-36
        if not self.can_run():
            return None
        self.done = False
        total = 0
        while not self.done:
            total += self.g.tick(self.policy_step())
        return total


class Env:
    """TreasureGame (TG/:54-114) over a private Random(seed) — the reference env built after
    random.seed(seed)."""

    def __init__(self, seed, level=None):
        self.rng = random.Random(seed)
        self.game = Game(level or read_level(), self.rng)   # the constructor's game (4 draws)
        self.options = [Option(self.game, k) for k in range(9)]

    def reset(self):
        self.game.reset_game()
        self.options = [Option(self.game, k) for k in range(9)]
        return self.game.get_state()

    def available_mask(self):
        return [int(o.can_run()) for o in self.options]

    def step(self, a):
        r = self.options[a].run()
        g = self.game
        done = g.got("gold") and g.cell()[1] == 0
        return g.get_state(), r, done, {}


# ---- the bench's action stream (tests/golden/make_golden.py) --------------------------------
M64 = 0xFFFFFFFFFFFFFFFF


def _sm64(x):
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


def pick_action(a0, g, t, mask=None):
    h = _sm64(_sm64(a0 ^ _sm64(g)) ^ t)
    if mask is None:
        return h % 9
    c = sum(mask)
    if c == 0:
        return h % 9
    k = h % c
    for i in range(9):
        if mask[i]:
            if k == 0:
                return i
            k -= 1
    raise AssertionError


def run_env(g, steps, a0, masked, autoreset, level=None, seed_base=0):
    """Env g (seed seed_base + g) for `steps` steps of the bench's action stream; returns the
    per-step (obs, reward, done) and the post-reset obs list."""
    env = Env(seed_base + g, level)
    obs = [env.reset()]
    rew, don, fin = [None], [False], [obs[0]]
    for t in range(steps):
        a = pick_action(a0, g, t, env.available_mask() if masked else None)
        o, r, d, _ = env.step(a)
        fin.append(o)
        if autoreset and d:
            o = env.reset()
        obs.append(o)
        rew.append(r)
        don.append(d)
    return obs, fin, rew, don


# ---- CPU baseline timing (bench.py) ---------------------------------------------------------
def _work(args):
    """steps of env g, g+stride, ... until `seconds` pass; returns env-steps done"""
    first, stride, seconds, policy, a0 = args
    masked = policy == "masked"
    level = read_level()
    done = 0
    t_end = time.perf_counter() + seconds
    g = first
    while time.perf_counter() < t_end:
        env = Env(g, level)
        env.reset()
        for t in range(200):
            a = pick_action(a0, g, t, env.available_mask() if masked else None)
            o, r, d, _ = env.step(a)
            if d:
                env.reset()
            done += 1
            if (t & 15) == 15 and time.perf_counter() >= t_end:
                break
        g += stride
    return done


def throughput(seconds, policy, a0):
    """env-steps/s of this restatement on 1 process and on one process per host core
    (len(os.sched_getaffinity(0))), each for ~`seconds` of wall time."""
    from multiprocessing import get_context
    cores = len(os.sched_getaffinity(0))
    t0 = time.perf_counter()
    n1 = _work((0, 1, seconds / 2, policy, a0))
    v1 = n1 / (time.perf_counter() - t0)
    procs = max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores))))
    with get_context("fork").Pool(procs) as p:
        t0 = time.perf_counter()
        nn = sum(p.map(_work, [(r, procs, seconds / 2, policy, a0) for r in range(procs)]))
        vn = nn / (time.perf_counter() - t0)
    return {"value_1proc": v1, "value": vn, "procs": procs, "unit": "env-steps/s",
            "kind": "port", "cores": procs,
            "sample": "oracle/pyref.py (pure-Python structural restatement of the reference: "
                      "pixel-loop predicates, object graph, CPython random), envs 0.. x <=200 "
                      "%s steps, auto-reset, %.0f s on 1 process + %.0f s on %d processes"
                      % (policy, seconds / 2, seconds / 2, procs)}
