#!/usr/bin/env python3
"""Benchmark: batched Treasure Game env-steps/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs ENVS_PER_GPU]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N`` without an external launcher starts its N ranks itself (fresh child processes,
before anything touches a GPU; dist.spawn_ranks) and returns rank 0's exit code.

One "step" = one TreasureGame.step() (TG/:91-96) of EVERY env of the batch: the on-device
synthetic policy writes the actions (uniform over the 9 options, counter hash keyed by the
global env index), tg_step runs each env's option to completion with auto-reset (k_classify
then k_run).  Every G steps (--gather-every, default 10) the completed episodes are drained
from the device queue and all-gathered over RCCL (dist.gather_padded: the one collective of
SURVEY §8e); rank 0 keeps them and reports their number and an order-independent digest of
(env, return, length), which does not depend on the number of GPUs.  Per-GPU work is fixed
(1,048,576 envs per GPU = config C3; C4 at 8 GPUs), so scaling is weak.  Inputs are resident
in HBM when the timed region starts.

Before timing: W warm-up steps, then ``--burn-in`` steps (default 3,000 uniform / 1,500
masked) so that the batch is in its steady state when timing starts: the envs' positions in
their MT19937 generations are spread out, so the timed steps regenerate generations at the
steady-state rate (N x draws per env-step / 312 per step; the line reports the measured and
the expected rate), and episodes complete and flow through the gather at their steady-state
rate (the first episodes end after ~550 masked / ~2,000 uniform steps).  The gathered records
of global envs [0, E) are compared with the oracle's replay of those envs over every step of
the run (``episode_check``).

Prints ONE JSON line (rank 0) with the driver's fields plus ``roofline`` (tg_step's kernels:
algorithmic bytes per launch over their HIP-event-timed duration vs the 8 TB/s HBM peak),
``cpu_baseline`` (the C oracle timed on this box's host cores, a bounded sample) and, at
N = 1, ``parity_check`` (4,096 envs x 200 steps replayed on the GPU and compared bit-for-bit
with the oracle's run in the cpu_baseline leg), ``masked_policy`` (the same measurement
with the masked-uniform policy: every step runs an option) and ``dropin_n1`` (the N = 1
drop-in's TreasureGame.step latency through the resident server kernel, with the same calls
launch-per-call beside it).

``--workload c5`` is config C5 instead: 65,536 envs per GPU whose step also renders every
env's screen (ObservationWrapper, TG/:38-51: tg_render -> k_render, 1,257,984 B per frame,
synthetic sprite sheet); its roofline is k_render's frame bytes over its HIP-event time.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node) at 1M batched envs, 1/2/4/8 MI355X; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ACTION_SEED = 0x5EED0001
PREGEN_BYTES = 8 << 30  # pre-generated action rows for the timed steps, at most this much HBM
EP_CAP = 4096          # episode records gathered per rank per step of a drain interval (padded)
KST_MAX = 512          # step launches whose kernel spans the library records (tg_amd.hip)
# algorithmic bytes of one tg_step for THIS data layout, per kernel:
#   k_classify, every env: action 4 + state word 16 + angles 16 + episode 8 read (44)
#     reward-None env: obs 72 + reward/valid/done 6 written (78; its episode word holds the
#     return and the episode's start step, unchanged by a reward-None step)
#     valid env: worklist index 4 + state 16 + angles 16 + episode 8 written (44)
#     stale MT half: its refill-list entry 4 written (a half is MT_HALF_GENS generations)
#   k_run, valid env: the worklist row 44 read; state 16 + angles 16 + episode 8 + obs 72 +
#     rows 6 written (118); random() draw: its 1-B code (tg_core.h draw_code)
#   k_regen (every 16 compact steps, tg_regenerate), per MT generation regenerated (tg_core.h:
#     halves of MT_HALF_GENS = 8 generations, chained in LDS): 312 codes + the words the build
#     stores (round 4: the even generations, so 624 words every other generation; tg_mt_layout)
#     written, an eighth of the source generation's 624 words, of the 4-B list entry and of the
#     env's 4-B state word read and written
#   k_step (direct mode): one kernel, the same without the worklist round trip
MT_HALF_GENS = 8
CLS_ENV, CLS_INVALID, CLS_VALID, CLS_REGEN = 44, 78, 44, 4 / MT_HALF_GENS
RUN_VALID, RUN_DRAW = 162, 1
FLOW_VALID = 4  # k_flow (TG_MODE_FLOW): a valid env's list entry (its state is not copied)
DIRECT_ENV, DIRECT_INVALID, DIRECT_VALID = 44, 78, 118
# per generation regenerated, set by set_layout from the loaded library (round 3's layout, which
# stored every generation's words, lacks tg_mt_layout)
REGEN_GEN = DIRECT_REGEN = 0.0


def set_layout(L):
    """REGEN_GEN / DIRECT_REGEN for the loaded library's MT storage."""
    global REGEN_GEN, DIRECT_REGEN
    stored = 1.0
    if hasattr(L, "tg_mt_layout"):
        ring, kept = ctypes.c_int32(), ctypes.c_int32()
        L.tg_mt_layout(ctypes.byref(ring), ctypes.byref(kept), None)
        stored = kept.value / ring.value
    REGEN_GEN = 2496 * stored + 312 + (2496 + 4 + 8) / MT_HALF_GENS
    DIRECT_REGEN = 2496 * stored + 312 + 2496 / MT_HALF_GENS
    return stored
BYTES_DRAW = RUN_DRAW
# SURVEY.md §8(d)'s layout-independent count per env-step: action 4 + obs 72 + reward 4 +
# valid 1 + done 1 + state read/write 2 x 40 = 162, plus 24 per random() draw (8 B of MT words
# read + 16 B amortised twist read/write)
SURVEY_BYTES_STEP, SURVEY_BYTES_DRAW = 162, 24
# algorithmic bytes of one k_render launch per env: the frame written (H*48 x W*48 x 3 =
# 1,257,984 for the default level) + the env's state words read (st4 16 + angles 16)
BYTES_RENDER_STATE = 32
MT_DRAWS_PER_GEN = 312  # random() values per MT19937 generation


def alg_bytes(st, mode="compact"):
    """algorithmic bytes of the counted steps per kernel: (k_classify, k_run, k_regen), or
    (0, k_step, 0) in the direct mode (k_step regenerates the halves its envs left itself)"""
    inval = st["steps"] - st["valid_steps"]
    if mode == "direct":
        return 0, (DIRECT_ENV * st["steps"] + DIRECT_INVALID * inval +
                   DIRECT_VALID * st["valid_steps"] + BYTES_DRAW * st["draws"] +
                   DIRECT_REGEN * st["regens"]), 0
    # flow: k_flow's lists carry the 4-B env index, its option waves gather the 40 B of state
    # from the env arrays (the same 162 B per valid env as k_run's 44-B worklist row + 118)
    cls = (CLS_ENV * st["steps"] + CLS_INVALID * inval +
           (FLOW_VALID if mode == "flow" else CLS_VALID) * st["valid_steps"] +
           CLS_REGEN * st["regens"])
    run = RUN_VALID * st["valid_steps"] + RUN_DRAW * st["draws"]
    return cls, run, REGEN_GEN * st["regens"]


def survey_bytes(st):
    return SURVEY_BYTES_STEP * st["steps"] + SURVEY_BYTES_DRAW * st["draws"]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--burn-in", type=int, default=None,
                    help="untimed steps after the warm-up so that MT regenerations and episode "
                         "completions reach their steady-state rates (default 3000 uniform / "
                         "1500 masked; 0 disables)")
    ap.add_argument("--workload", default="c3", choices=["c3", "c5"],
                    help="c3: vector-obs step (default, the headline); c5: step + RGB render")
    ap.add_argument("--envs", type=int, default=None,
                    help="envs per GPU (default 1,048,576 for c3, 65,536 for c5)")
    ap.add_argument("--policy", default="uniform", choices=["uniform", "masked"])
    ap.add_argument("--level", default=None,
                    help="a level directory in the reference's three-file format (default: the "
                         "reference's own level)")
    ap.add_argument("--no-autoreset", action="store_true")
    ap.add_argument("--mode", default="compact", choices=["compact", "direct", "flow"],
                    help="step implementation (bit-identical): two-pass compacted, one-pass, or "
                         "flow (with --rollout: k_flow, chunks advancing without a batch-wide "
                         "barrier between steps, DESIGN.md 9.2)")
    ap.add_argument("--run-blocks", type=int, default=0, help="k_run workgroups (0 = default)")
    ap.add_argument("--rollout", type=int, default=0,
                    help="K > 0: tg_rollout, K steps per call with the policy evaluated inside "
                         "the step kernels (episodes drained / gathered every K steps); 0: the "
                         "per-step API (tg_policy_actions + tg_step per step)")
    ap.add_argument("--groups", type=int, default=1,
                    help="with --rollout: step the batch as G groups on G streams (tg_set_groups)")
    ap.add_argument("--stagger", action="store_true",
                    help="with --groups: group g + 1 starts after group g's first k_classify")
    ap.add_argument("--actions-in-loop", action="store_true",
                    help="generate the uniform policy's actions inside the timed loop "
                         "(tg_policy_actions before every tg_step) instead of before it")
    ap.add_argument("--gather-every", type=int, default=10,
                    help="per-step API: drain and gather the completed episodes every G steps "
                         "(SURVEY §8e: batched gather; 1 = every step); --rollout K drains "
                         "every K steps")
    ap.add_argument("--progress", action="store_true",
                    help="a line on stderr every 500 untimed steps (profiler runs)")
    ap.add_argument("--timing-every", type=int, default=1,
                    help="kernel spans of every k-th timed step (in-kernel s_memrealtime stamps: "
                         "nothing goes on the stream) for the roofline")
    ap.add_argument("--no-spin", dest="spin", action="store_false",
                    help="wait for the timed region's end in torch.cuda.synchronize alone (the "
                         "default polls the end event first, then synchronizes)")
    ap.add_argument("--secondary-steps", type=int, default=30,
                    help="N = 1, c3: steps of the masked-policy line (0 disables it)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target duration of the CPU-baseline sample (0 disables it and the "
                         "parity check)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC-derived HBM bytes per tg_step (default profiles/"
                         "traffic_step_<policy>.json), if measured")
    ap.add_argument("--episode-envs", type=int, default=None,
                    help="episode_check: the oracle replays global envs [0, E) over the whole "
                         "run (default 16384 uniform / 8192 masked; 0 disables)")
    return ap.parse_args(argv)


# ---- CPU legs (the oracle is loaded here only: bench's cpu_baseline leg) ------------------
def dropin_latency(tg, steps=300, seed=0):
    """The N=1 drop-in's own hot call: TreasureGame.step(a) (TG/:91-96) from Python, one env on
    the GPU, uniform random actions from a host RNG, resetting when done; mean µs per call.
    Both construction modes: TreasureGame() draws from Python's global random as the reference
    does (tg_step1_pywords: the global Random's words and index in place), TreasureGame(seed=s)
    from the env's own stream (tg_step1).  Each call is served by the resident server kernel
    (k_serve1, the default); the ``launch_per_call`` figures are the same calls with serving
    off (one launch and one synchronisation each, tg_set_serve(0))."""
    import random
    out = {"steps": steps, "api": "TreasureGame.step, host RNG actions, synchronous"}
    saved = random.getstate()
    try:
        for serve in (True, False):
            for mode in ("shared_global_random", "private_stream"):
                random.seed(seed)
                env = tg.TreasureGame() if mode == "shared_global_random" else tg.TreasureGame(seed=seed)
                env._vec.set_serve(serve)
                env.reset()
                r = random.Random(seed)
                for _ in range(20):
                    env.step(r.randrange(9))
                t0 = time.perf_counter()
                for _ in range(steps):
                    if env.step(r.randrange(9))[2]:
                        env.reset()
                key = mode + "_step_us" if serve else "launch_per_call_" + mode + "_step_us"
                out[key] = (time.perf_counter() - t0) / steps * 1e6
                if mode == "shared_global_random":  # an agent reading the mask before each step
                    t0 = time.perf_counter()
                    for _ in range(steps):
                        m = env.available_mask
                        if env.step(r.randrange(9))[2]:
                            env.reset()
                    key = "mask_and_step_us" if serve else "launch_per_call_mask_and_step_us"
                    out[key] = (time.perf_counter() - t0) / steps * 1e6
                    del m
                env.close()
    finally:
        random.setstate(saved)
    out["step_us"] = out["shared_global_random_step_us"]  # the default TreasureGame()
    return out


def cpu_baseline(seconds, policy, parity_envs=0):
    """The C oracle (oracle/, the CPU restatement of the reference) on this box's host cores:
    a bounded sample of the same workload (same seeds, action stream and auto-reset).  Also
    returns the per-env rolling hashes of the first ``parity_envs`` envs after 200 steps."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402 — bench's cpu_baseline leg only
    O.build()
    cores = len(os.sched_getaffinity(0))
    threads = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    pol = 1 if policy == "masked" else 0
    steps = 200
    n = 4096
    t0 = time.perf_counter()
    O.run(0, 0, n, steps, ACTION_SEED, pol, True, full=False, nthreads=threads)
    dt = time.perf_counter() - t0
    n = max(threads * 64, parity_envs, int(n * seconds / max(dt, 1e-3)))
    t0 = time.perf_counter()
    r = O.run(0, 0, n, steps, ACTION_SEED, pol, True, full=False, nthreads=threads)
    dt = time.perf_counter() - t0
    out = {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
           "sample": "C oracle (oracle/tg_oracle.c, CPU restatement of the reference step path), "
                     "envs 0..%d x %d steps, %s policy, auto-reset, %d OpenMP threads, %.1f s"
                     % (n - 1, steps, policy, threads, dt)}
    return out, r["hash"][:parity_envs], steps


def oracle_episodes(policy, steps, t_from, envs, level=None):
    """(count, digest) of the auto-reset episodes of global envs [0, envs) that end at step
    index >= t_from, from the C oracle's replay of the run (bench's cpu leg only)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402 — bench's cpu_baseline leg only
    O.build()
    cores = len(os.sched_getaffinity(0))
    threads = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    return O.run_episodes(0, 0, envs, steps, ACTION_SEED, 1 if policy == "masked" else 0, t_from,
                          threads, level_dir=level)


def python_baseline(seconds, policy):
    """The pure-Python structural restatement of the reference step path (oracle/pyref.py:
    the reference's pixel loops, object graph and random module), on 1 process and on one
    process per host core, same seeds / actions / auto-reset."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyref  # noqa: E402 — bench's cpu_baseline leg only
    return pyref.throughput(seconds, policy, ACTION_SEED)


def cpu_baseline_render(seconds, policy):
    """C5's CPU leg: the oracle's renderer restatement (plus construct/reset and one step per
    env) on this box's host cores, synthetic sprites."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: E402 — bench's cpu_baseline leg only
    from gym_treasure_game_amd.render import synthetic_sprites
    O.build()
    cores = len(os.sched_getaffinity(0))
    threads = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    pol = 1 if policy == "masked" else 0
    sprites = synthetic_sprites(seed=1)
    n = threads * 4
    t0 = time.perf_counter()
    O.run_render(0, np.arange(n), 1, ACTION_SEED, pol, True, sprites, nthreads=threads)
    dt = time.perf_counter() - t0
    n = int(min(max(n, n * seconds / max(dt, 1e-3)), 20000))
    t0 = time.perf_counter()
    O.run_render(0, np.arange(n), 1, ACTION_SEED, pol, True, sprites, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "env-steps/s (rendered frames/s)", "cores": threads,
            "kind": "port",
            "sample": "C oracle renderer (oracle/tg_oracle.c tgo_run_render: construct, reset, 1 "
                      "%s step, render('rgb_array')) for envs 0..%d, %d OpenMP threads, %.1f s"
                      % (policy, n - 1, threads, dt)}


# ---- parity spot check: the product on the GPU, hashed like tests/golden/make_golden.py -----
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _sm64(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _rec_hash(h, obs, rew, valid, done):
    bits = np.ascontiguousarray(obs).view(np.uint64)
    with np.errstate(over="ignore"):
        for k in range(9):
            h = _sm64(h ^ bits[:, k])
        w = (rew.astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)) | \
            (valid.astype(np.uint64) << np.uint64(32)) | (done.astype(np.uint64) << np.uint64(40))
        return _sm64(h ^ w)


def gpu_hashes(tg, n, steps, policy, mode, dev):
    """Per-env rolling hashes of envs 0..n-1 (seed 0, the bench's action stream, auto-reset)
    after ``steps`` steps, through the product API."""
    vec = tg.TreasureGameVec(n, seed=0, autoreset=True, mode=mode, device=dev)
    h = np.arange(n, dtype=np.uint64)
    z32, z8 = np.zeros(n, np.int32), np.zeros(n, np.uint8)
    h = _rec_hash(h, vec.reset().cpu().numpy(), z32, z8, z8)
    for t in range(steps):
        o, r, v, d, info = vec.step(vec.policy_actions(t, ACTION_SEED, policy))
        h = _rec_hash(h, info["final_obs"].cpu().numpy(), r.cpu().numpy(), v.cpu().numpy(),
                      d.cpu().numpy())
    errs = vec.errors()
    vec.close()
    return h, errs


# ---- the measured loop ------------------------------------------------------------------------
class Runner:
    """One rank's batch and its step loop (per-step API or tg_rollout), with the episode
    drain + gather every G steps."""

    def __init__(self, tg, D, args, policy, count, offset, world, dev, keep_log):
        self.tg, self.D, self.args, self.world, self.dev = tg, D, args, world, dev
        self.count = count
        self.autoreset = not args.no_autoreset
        vec = tg.TreasureGameVec(count, seed=0, global_offset=offset, autoreset=False, device=dev,
                                 level_dir=args.level)
        vec.set_mode(args.mode, args.run_blocks)
        vec.autoreset = self.autoreset  # final_obs is not requested: obs/reward/valid/done only
        vec.reset()
        self.vec = vec
        self.K = args.rollout
        self.G = self.K if self.K else args.gather_every
        if self.G < 1:
            raise SystemExit("--gather-every must be >= 1")
        self.ep_cap = EP_CAP * self.G  # records per rank per drain (padded; the rest stays queued)
        self.ep_rows = torch.zeros((self.ep_cap, 2), dtype=torch.int64, device=dev)
        self.ep_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        self.all_rows = self.all_cnt = None
        if world > 1:
            self.all_rows = torch.empty((world * self.ep_cap, 2), dtype=torch.int64, device=dev)
            self.all_cnt = torch.empty(world, dtype=torch.int32, device=dev)
        drains = args.steps // self.G + 2
        self.log = D.EpisodeLog(drains, world, self.ep_cap, dev, keep=keep_log)
        L, h = vec._L, vec.handle
        self.L, self.h = L, h
        self.mt_stored = set_layout(L)
        self.flags = tg._lib.TG_STEP_AUTORESET if self.autoreset else 0
        p = self.p
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        self.pol = tg._lib.TG_POLICY_MASKED if policy == "masked" else tg._lib.TG_POLICY_UNIFORM
        self.args_step = (h, p(vec._act), p(vec._obs), p(vec._rew), p(vec._valid), p(vec._done),
                          None, self.flags, self.stream)
        # the timed steps' actions (inputs) sit in HBM before timing starts: a uniform-policy
        # action depends on (env, t) only, so [t0, t0 + steps) is generated untimed, one row per
        # step (4 B per env-step); the masked policy reads the state and stays in the loop
        self.pre, self.pre_t0 = None, 0
        if (policy == "uniform" and not self.K and not args.actions_in_loop
                and args.steps * count * 4 <= PREGEN_BYTES):
            self.pre = torch.empty((max(args.steps, 1), count), dtype=torch.int32, device=dev)
        if self.K:
            if args.workload == "c5":
                raise SystemExit("--rollout K: c3 only")
            self.roll = [torch.empty((self.K, count), dtype=d, device=dev)
                         for d in (torch.int32, torch.uint8, torch.uint8)]
            if args.groups > 1:
                tg._lib.check(L.tg_set_groups(h, args.groups, 1 if args.stagger else 0),
                              "tg_set_groups")
        self.frames, self.rev, self.timing, self.render_on = None, [], False, True
        self.timing_every = args.timing_every
        if args.workload == "c5":  # ObservationWrapper.step: render every env after its step
            vec.render_init(tg.synthetic_sprites(seed=1))
            self.frames = torch.empty((count,) + vec.frame_shape, dtype=torch.uint8, device=dev)

    @staticmethod
    def p(t):
        return ctypes.c_void_p(t.data_ptr())

    def drain(self, log=True):
        """one drain of the device queue, gathered to rank 0's log: written in place into the
        log's next slot (one launch at one rank, the drain and the all-gather beyond)"""
        chk, L, p = self.tg._lib.check, self.L, self.p
        if log and self.world == 1:
            rows, cnt = self.log.target()
            chk(L.tg_episodes(self.h, p(rows), p(cnt), self.ep_cap, self.stream), "episodes")
            self.log.commit()
            return cnt
        chk(L.tg_episodes(self.h, p(self.ep_rows), p(self.ep_cnt), self.ep_cap, self.stream),
            "episodes")
        if log:
            rows, cnt = self.log.target()
            self.D.gather_padded(self.ep_rows, self.ep_cnt, rows, cnt)
            self.log.commit()
            return cnt
        _, cnt = self.D.gather_padded(self.ep_rows, self.ep_cnt, self.all_rows, self.all_cnt)
        return cnt

    def drain_all(self, log):
        """drain until every rank's queue is empty (untimed; synchronises)"""
        while True:
            cnt = self.drain(log)
            if int(cnt.sum().item()) == 0:
                return

    def roll_steps(self, t, k):
        """steps t .. t+k-1 in one tg_rollout call (k <= K), then the episode drain"""
        p = self.p
        self.tg._lib.check(self.L.tg_rollout(self.h, k, ACTION_SEED, t, self.pol, self.flags,
                                             None, None, p(self.roll[0]), p(self.roll[1]),
                                             p(self.roll[2]), self.stream), "rollout")
        self.drain()

    def advance(self, t, nsteps):
        """nsteps steps from t: rollout calls of K steps (the last one shorter), or per step"""
        if self.K:
            done = 0
            while done < nsteps:
                k = min(self.K, nsteps - done)
                self.roll_steps(t + done, k)
                done += k
        else:
            for j in range(nsteps):
                self.step(t + j)
        return t + nsteps

    def step(self, t):
        chk, L, p = self.tg._lib.check, self.L, self.p
        K = self.K
        if K:
            raise AssertionError("rollout mode steps through advance()")
        elif self.timing and self.pre is not None:  # actions generated before timing
            chk(L.tg_step(self.h, self.pre_ptr[t - self.pre_t0], *self.args_step[2:]), "tg_step")
        else:
            chk(L.tg_policy_actions(self.h, ACTION_SEED, t, self.pol, p(self.vec._act),
                                    self.stream), "actions")
            chk(L.tg_step(*self.args_step), "tg_step")
        if (t + 1) % self.G == 0:
            self.drain()
        if self.frames is not None and self.render_on:
            if self.timing:  # k_render alone, on the stream it is launched on
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            chk(L.tg_render(self.h, 0, self.count, p(self.frames), self.stream), "tg_render")
            if self.timing:
                ev[1].record()
                self.rev.append(ev)

    def probe_region(self, steps):
        """The platform's share of a timed region: the same number of dependent
        launches as the region held (2 step kernels per step + the k_regen launches + the final
        drain), as EMPTY kernels of the step kernels' grid (tg_probe_dispatch), timed exactly as
        the region is (synchronize, wall clock + event pair, end event polled, synchronize).
        Untimed by the line itself; reported beside it."""
        n = 2 * steps + -(-steps // 16) + 1
        blocks = min(4096, max(1, self.count // 256))
        out = []
        for _ in range(3):
            torch.cuda.synchronize(self.dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            self.tg._lib.check(self.L.tg_probe_dispatch(n, blocks, self.stream), "probe")
            e1.record()
            if self.args.spin:
                while not e1.query():
                    pass
            torch.cuda.synchronize(self.dev)
            out.append(((time.perf_counter() - t0) * 1e3, e0.elapsed_time(e1)))
        w, e = sorted(out)[1]
        return {"kernels": n, "blocks": blocks, "wall_ms": w, "events_ms": e, "wall_minus_events_ms": w - e}

    def measure(self, warmup, burn_in, steps):
        """warm-up + burn-in (untimed), then EXACTLY ``steps`` timed steps between barriers;
        returns the max-over-ranks wall time and this rank's stats."""
        t = 0
        if self.K:
            t = self.advance(t, warmup)
            for j in range(0, burn_in, 500):
                t = self.advance(t, min(500, burn_in - j))
                if self.args.progress:
                    print("untimed step %d of %d" % (t, warmup + burn_in), file=sys.stderr,
                          flush=True)
        for j in range(warmup + burn_in if not self.K else 0):
            self.render_on = j < warmup  # c5: the burn-in only advances the envs
            self.step(t)
            t += 1
            if self.args.progress and j % 500 == 499:
                print("untimed step %d of %d" % (j + 1, warmup + burn_in), file=sys.stderr,
                      flush=True)
        self.render_on = True
        if self.pre is not None:  # the timed steps' inputs, resident before timing
            self.pre_t0 = t
            # their device addresses as call arguments, made once (a torch view and a ctypes
            # pointer per step cost the host ~10 us, most visibly before the region's first
            # launch)
            self.pre_ptr = [self.p(self.pre[j]) for j in range(steps)]
            for j in range(steps):
                self.tg._lib.check(self.L.tg_policy_actions(
                    self.h, ACTION_SEED, t + j, self.pol, self.p(self.pre[j]), self.stream),
                    "actions")
        self.drain_all(log=False)  # the timed region's records are its own
        # no MT regeneration pending from the untimed steps: the timed region does exactly the
        # regeneration work of its own steps (the deferred lists drained again at its end)
        self.tg._lib.check(self.L.tg_regenerate(self.h, self.stream), "tg_regenerate")
        torch.cuda.synchronize(self.dev)
        self.log.reset()
        vec = self.vec
        vec.stats_reset()
        # the library keeps KST_MAX = 512 step records and would flush (a device sync and a
        # copy) inside the timed region past them: sample every k-th step so that the timed
        # steps' records fit
        self.timing_every = (max(self.args.timing_every, -(-steps // KST_MAX))
                             if self.args.timing_every else 0)
        vec.set_timing(self.timing_every)
        self.timing = True
        if self.world > 1:
            dist.barrier()
        # HIP events on the step's stream (torch's current stream, which the steps use) around
        # the whole timed region: two records, none between kernels
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if os.environ.get("TG_BENCH_PRESPIN", "1") != "0":
            # the synchronisation before the region as a spin on an event: a blocking wait let
            # the host thread sleep, and the region's first launch then ran on a cold core
            # (~58 us from ev0 to the first kernel's GPU start)
            evs = torch.cuda.Event()
            evs.record()
            while not evs.query():
                pass
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        ev0.record()
        if self.K:
            t = self.advance(t, steps)
        else:
            for _ in range(steps):
                self.step(t)
                t += 1
        self.tg._lib.check(self.L.tg_regenerate(self.h, self.stream), "tg_regenerate")
        ev1.record()
        t_launched = time.perf_counter()
        if self.args.spin:  # a blocking wait's wake-up costs tens of us after the last kernel
            while not ev1.query():
                pass
        torch.cuda.synchronize(self.dev)
        t_synced = time.perf_counter()
        if self.world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        self.events_ms = ev0.elapsed_time(ev1)
        self.host_ms = {"launch": (t_launched - t0) * 1e3, "wait": (t_synced - t_launched) * 1e3,
                        "spin": bool(self.args.spin)}
        self.timing = False
        vec.set_timing(0)
        self.region_probe = self.probe_region(steps)
        st = vec.stats()
        self.drain_all(log=True)  # records of the timed steps still queued (untimed)
        if self.world > 1:
            dt_t = torch.tensor([dt], dtype=torch.float64, device=self.dev)
            dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
            dt = float(dt_t.item())
        return dt, st


def node_totals(st, world, dev):
    keys = ["steps", "ticks", "draws", "valid_steps", "episodes", "episodes_dropped",
            "wave_ticks", "regens"]
    if world == 1:
        return {k: st[k] for k in keys}
    tot = torch.tensor([st[k] for k in keys], dtype=torch.int64, device=dev)
    dist.all_reduce(tot)
    return dict(zip(keys, tot.tolist()))


def default_burn_in(policy):
    """untimed steps before timing: the batch's steady state (module docstring)"""
    return 3000 if policy == "uniform" else 1500


def default_episode_envs(policy):
    return 16384 if policy == "uniform" else 8192


def load_pmc(path, envs, policy, mode, regens_per_step, burn_in):
    """profiles/traffic_step_<policy>.json (scripts/prof_summary.py) when its PMC source run
    matches this run: same envs, policy and step mode, and a regeneration rate within 10 %."""
    if path is None:
        path = os.path.join(ROOT, "profiles", "traffic_step_%s.json" % policy)
    if not os.path.exists(path):
        return None
    tj = json.load(open(path))
    if (tj.get("envs") != envs or tj.get("policy") != policy or tj.get("mode") != mode):
        return None
    ref = tj.get("regens_per_step")
    if ref is None or abs(regens_per_step - ref) > 0.1 * max(ref, 1.0):
        return None
    return tj


def step_line(args, runner, dt, st, node, world, total):
    """the bench line's roofline / counters for the c3 step measurement: the dominant kernel
    (k_run; k_step in the direct mode) over its own duration, the step's kernels beside.

    Durations: the kernels of every --timing-every-th timed step (default every step) and every
    k_regen launch record their span, from the first wave's start to the last wave's end, by
    in-kernel s_memrealtime stamps (tg_amd.hip kst_end: two returnless atomics per wave, nothing
    on the stream); a HIP event pair on the step's stream brackets the whole timed region.  The
    rocprofv3 kernel trace of the same command agrees with the spans (profiles/<tag>*)."""
    env_steps = total * args.steps
    assert node["steps"] == env_steps, (node, env_steps)
    launches = max(st["launches"], 1)
    timed = max(st["timed_launches"], 1)
    run_s = st["run_ms"] / 1e3 / timed          # k_run's span (k_step's in the direct mode)
    cls_s = st["classify_ms"] / 1e3 / timed     # k_classify's span
    cls_b, run_b, regen_b = (b / launches for b in alg_bytes(st, args.mode))
    flow = args.mode == "flow" and args.rollout > 0
    if flow:  # one kernel does both passes; its span per step is its launch's / K (run_ms)
        cls_b, run_b = 0.0, cls_b + run_b
    if args.rollout and args.groups > 1:  # the spans are group 0's kernels: its share
        cls_b, run_b, regen_b = cls_b / args.groups, run_b / args.groups, regen_b / args.groups
    rl = st.get("regen_launches", 0)
    rt = st.get("regen_timed", 0)
    grouped = bool(args.rollout and args.groups > 1)
    if grouped:  #  only the handle's own k_regen launches stamp spans, while every
        # group's drains count as launches: no regeneration figures for grouped runs
        rl, rt, regen_b = 0, 0, 0.0
    regen_launch_s = st["regen_ms"] / 1e3 / rt if rt else 0.0
    regen_s = regen_launch_s * rl / launches    # per step
    surv = survey_bytes(st) / launches
    d = node["draws"] / max(node["steps"], 1)
    regens = st["regens"] / launches
    regens_expected = runner.count * d / MT_DRAWS_PER_GEN
    lane_eff = node["ticks"] / max(64 * node["wave_ticks"], 1)
    pmc = load_pmc(args.traffic_json, args.envs, args.policy_used, args.mode, regens,
                   args.burn_in_used)
    run_name = "k_flow" if flow else "k_run" if args.mode != "direct" else "k_step"
    kp = pmc.get("kernels", {}) if pmc else {}
    run_pmc = next((v for k, v in kp.items() if k.split("<")[0] == run_name), None)
    cls_pmc = next((v for k, v in kp.items() if k.split("<")[0] == "k_classify"), None)
    info = runner.vec.kernel_info()

    def kern(name, alg, sec, pm, traffic=None):
        ach = alg / sec / 1e9 if sec > 0 else None
        out = {"kernel": name, "alg_bytes_per_launch": alg, "kernel_ms": sec * 1e3,
               "achieved": ach, "frac": ach / HBM_PEAK_GBS if ach else None,
               "traffic": traffic if traffic is not None else (pm["hbm_bytes"] if pm else None)}
        if pm:
            out.update({"traffic_gbs": out["traffic"] / sec / 1e9 if sec > 0 else None,
                        "valu_util": pm.get("valu_util"), "wait_frac": pm.get("wait_frac"),
                        "limiter": pm.get("limiter"), "rocprof_ms": (pm.get("avg_ns") or 0) / 1e6})
        if name in info:
            out["occupancy"] = info[name]
        return out

    run_k = kern(run_name, run_b, run_s, run_pmc)
    # "bound" names the roofline the fraction is taken against: HBM, the only one this integer
    # path has (no MFMA); what the counters say limits the kernel is "limiter"
    roof = {"bound": "hbm", "kernel": run_name + " (the step's dominant kernel)",
            "achieved": run_k["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": run_k["frac"], "traffic": run_k["traffic"],
            "traffic_source": pmc["source"] if pmc else None,
            "kernel_ms": run_s * 1e3, "alg_bytes_per_launch": run_b,
            "timed_launches": st["timed_launches"],
            "timing": "every %d-th timed step: the kernel's span from its first wave's start to "
                      "its last wave's end (in-kernel s_memrealtime stamps); HIP events on the "
                      "step's stream around the timed region (events_ms)" % runner.timing_every,
            "rocprof_ms": run_k.get("rocprof_ms"),
            "limiter": run_k.get("limiter"), "valu_util": run_k.get("valu_util"),
            "wait_frac": run_k.get("wait_frac"), "lane_efficiency": lane_eff,
            "bound_basis": "the HBM roofline (no MFMA on this integer path); the kernel is "
                           "limited by what `limiter` says (rocprofv3 counters)",
            "note": "dominant kernel by time; latency-bound option loops that move few bytes "
                    "(the MT regeneration is k_regen's: step.kernels.regen; the whole step: "
                    "step.frac) (DESIGN.md 3.6)"}
    kernels = {"run": run_k}
    if grouped:
        kernels["regen"] = {"note": "not reported with --groups > 1: the groups' k_regen launches "
                                    "are not stamped (the step figures leave it out)"}
    if args.mode != "direct":
        if not flow:
            kernels["classify"] = kern("k_classify", cls_b, cls_s, cls_pmc)
        if rl:
            regen_pmc = next((v for k, v in kp.items() if k.split("<")[0] == "k_regen"), None)
            gens_launch = st["regens"] / rl  # MT generations regenerated per k_regen launch
            # the PMC traffic per generation regenerated (its source run: 16 steps per launch),
            # scaled to this run's launches
            tr_gen = None
            if regen_pmc and pmc.get("regens_per_step"):
                tr_gen = regen_pmc["hbm_bytes"] / (pmc["regens_per_step"] * 16.0)
            kernels["regen"] = kern("k_regen", regen_b * launches / rl, regen_launch_s, regen_pmc,
                                    traffic=tr_gen * gens_launch if tr_gen else None)
            kernels["regen"].update({
                "launches": rl, "steps_per_launch": launches / rl,
                "generations_per_launch": gens_launch,
                "alg_bytes_per_generation": REGEN_GEN,
                "traffic_per_generation": tr_gen,
                "ms_per_1k_generations": regen_launch_s * 1e3 / gens_launch * 1e3
                if gens_launch else None})
    all_b, all_s = cls_b + run_b + regen_b, cls_s + run_s + regen_s
    ms_step = dt / args.steps * 1e3
    roof["step"] = {"kernel": "tg_step = " + (" + ".join(
                        ["k_flow / steps per launch", "k_regen / steps per launch"] if flow else
                        ["k_classify", "k_run", "k_regen / steps per launch"]
                        if args.mode != "direct" else ["k_step"])),
                    "alg_bytes_per_launch": all_b, "kernel_ms": all_s * 1e3,
                    "events_ms_per_step": runner.events_ms / args.steps,
                    "host_ms": runner.host_ms,
                    # the region's wall clock minus its event pair, beside the same for a region
                    # of as many empty dependent kernels
                    "region_wall_minus_events_ms": dt * 1e3 - runner.events_ms,
                    "region_probe": runner.region_probe,
                    "gaps_ms": ms_step - all_s * 1e3,
                    "achieved": all_b / all_s / 1e9 if all_s else None,
                    "frac": all_b / all_s / 1e9 / HBM_PEAK_GBS if all_s else None,
                    "frac_wall": all_b / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBS,
                    "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
                    "alg_bytes_per_launch_survey": surv,
                    "frac_survey": surv / all_s / 1e9 / HBM_PEAK_GBS if all_s else None,
                    "frac_survey_wall": surv / (ms_step / 1e3) / 1e9 / HBM_PEAK_GBS,
                    "kernels": kernels}
    return {
        "ticks_per_s": node["ticks"] / dt,
        # ticks executed / lane-ticks issued by the tick loops' wavefronts
        "lane_efficiency": lane_eff,
        "valid_step_frac": node["valid_steps"] / max(node["steps"], 1),
        "draws_per_step": d,
        "regens_per_step": regens,
        "regens_per_step_steady_state": regens_expected,
        "roofline": roof,
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0 and args.gpus > 1:
        # no external launcher: start the ranks as fresh processes before any GPU call
        import gym_treasure_game_amd.dist as D
        sys.exit(D.spawn_ranks(args.gpus, sys.argv[1:]))
    world = max(world, 1)
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
    c5 = args.workload == "c5"
    if args.envs is None:
        args.envs = 65536 if c5 else 1 << 20
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    import gym_treasure_game_amd as tg
    import gym_treasure_game_amd.dist as D

    total = args.envs * world
    offset, count = D.shard(total, rank, world)
    args.policy_used = args.policy
    args.burn_in_used = (args.burn_in if args.burn_in is not None
                         else default_burn_in(args.policy))
    ep_envs = (args.episode_envs if args.episode_envs is not None
               else default_episode_envs(args.policy))
    ep_envs = min(ep_envs, total)
    run = Runner(tg, D, args, args.policy, count, offset, world, dev, keep_log=(rank == 0))
    dt, st = run.measure(args.warmup, args.burn_in_used, args.steps)
    node = node_totals(st, world, dev)
    errs = run.vec.errors()
    rec, digest = run.log.digest() if rank == 0 else (None, None)
    autoreset = run.autoreset
    # (policy, warmup, burn-in, steps, E, the gathered records of envs [0, E) and their digest)
    checks = []
    if rank == 0 and autoreset and ep_envs > 0:
        checks.append((args.policy, args.warmup, args.burn_in_used, args.steps, ep_envs,
                       run.log.digest(env_below=ep_envs), "line"))

    line = None
    if rank == 0:
        env_steps = total * args.steps
        if autoreset:
            # every episode the step kernels counted reached rank 0 through the gather
            assert rec == node["episodes"] - node["episodes_dropped"], (rec, node)
        workload = ("C3/C4: %d batched treasure_game-v0 envs per GPU, vector obs, %s random "
                    "options, auto-reset%s%s" % (args.envs, args.policy,
                                                 " + RCCL episode gather" if world > 1 else "",
                                                 ", level %s" % args.level if args.level else ""))
        extra = step_line(args, run, dt, st, node, world, total)
        if c5:
            fh, fw, _ = run.vec.frame_shape
            r_ms = sum(a.elapsed_time(b) for a, b in run.rev) / max(len(run.rev), 1)
            r_alg = count * (fh * fw * 3 + BYTES_RENDER_STATE)
            r_ach = r_alg / (r_ms / 1e3) / 1e9
            r_traffic = None
            tj_path = os.path.join(ROOT, "profiles", "traffic_render.json")
            if os.path.exists(tj_path):
                tj = json.load(open(tj_path))
                if tj.get("envs") == count:
                    r_traffic = tj.get("hbm_bytes_per_launch")
            extra["step_roofline"] = extra.pop("roofline")
            extra["roofline"] = {"bound": "hbm", "kernel": "k_render (tg_render)",
                                 "achieved": r_ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": r_ach / HBM_PEAK_GBS, "traffic": r_traffic,
                                 "kernel_ms": r_ms, "alg_bytes_per_launch": r_alg}
            workload = ("C5: %d batched treasure_game-v0 envs per GPU, ObservationWrapper RGB "
                        "render (%dx%dx3 u8 frames, synthetic sprites) after every step, %s "
                        "random options, auto-reset" % (args.envs, fh, fw, args.policy))
            extra["frames_per_s"] = env_steps / dt
            extra["frame_bytes"] = fh * fw * 3
        line = {
            "metric": METRIC, "value": env_steps / dt, "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int32+f64", "data": "synthetic",
            "config": {"workload": workload,
                       "envs_per_gpu": args.envs, "total_envs": total, "policy": args.policy,
                       "autoreset": autoreset, "step_mode": args.mode,
                       "api": ("tg_rollout x%d (policy inside the step kernels%s)"
                               % (args.rollout, ", %d groups on %d streams%s" % (
                                   args.groups, args.groups,
                                   ", staggered" if args.stagger else "")
                                  if args.groups > 1 else "")
                               if args.rollout else
                               "tg_step per step, the timed steps' actions generated in HBM "
                               "before timing (tg_policy_actions)" if run.pre is not None else
                               "tg_policy_actions + tg_step per step"),
                       "parallelism": "env-shard x%d" % world},
            "burn_in": args.burn_in_used,
        }
        line.update(extra)
        line.update({"episodes": node["episodes"], "episodes_dropped": node["episodes_dropped"],
                     "episodes_gathered": rec, "episode_digest": digest,
                     "gather_every": run.G, "error_flags": errs})
    run.vec.close()
    del run

    if rank == 0 and world == 1 and not c5 and args.secondary_steps > 0:
        # the masked-uniform policy: every step runs an option (report it beside
        # the uniform headline), same batch size, its own burn-in
        other = "masked" if args.policy == "uniform" else "uniform"
        a2 = parse(sys.argv[1:])
        a2.envs, a2.policy, a2.policy_used = args.envs, other, other
        a2.steps = args.secondary_steps
        a2.burn_in_used = default_burn_in(other)
        w2 = min(args.warmup, 5)
        r2 = Runner(tg, D, a2, other, count, offset, world, dev, keep_log=True)
        dt2, st2 = r2.measure(w2, a2.burn_in_used, a2.steps)
        n2 = node_totals(st2, 1, dev)
        sec = {"policy": other, "value": total * a2.steps / dt2, "unit": "env-steps/s",
               "steps": a2.steps, "burn_in": a2.burn_in_used,
               "ms_per_step": dt2 / a2.steps * 1e3}
        sec.update(step_line(a2, r2, dt2, st2, n2, 1, total))
        rec2, dig2 = r2.log.digest()
        assert rec2 == n2["episodes"] - n2["episodes_dropped"], (rec2, n2)
        sec.update({"episodes": n2["episodes"], "episodes_dropped": n2["episodes_dropped"],
                    "episodes_gathered": rec2, "episode_digest": dig2})
        e2 = min(default_episode_envs(other), total)
        if r2.autoreset and e2 > 0 and args.episode_envs != 0:
            checks.append((other, w2, a2.burn_in_used, a2.steps, e2, r2.log.digest(env_below=e2),
                           other + "_policy"))
        r2.vec.close()
        line[other + "_policy"] = sec
        line["dropin_n1"] = dropin_latency(tg)

    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        if c5:
            line["cpu_baseline"] = cpu_baseline_render(args.cpu_seconds, args.policy)
        else:
            pe, ps = 4096, 200
            cb, ref_h, steps_h = cpu_baseline(args.cpu_seconds, args.policy, parity_envs=pe)
            try:
                cb["reference_python"] = python_baseline(min(args.cpu_seconds, 10.0), args.policy)
            except ImportError:
                cb["reference_python"] = None
            if cb["reference_python"] and "dropin_n1" in line:  # the same call, on one core
                line["dropin_n1"]["reference_python_step_us"] = \
                    1e6 / cb["reference_python"]["value_1proc"]
            line["cpu_baseline"] = cb
            got, gerr = gpu_hashes(tg, pe, steps_h, args.policy, args.mode, dev)
            bad = int(np.count_nonzero(got != ref_h))
            line["parity_check"] = {"envs": pe, "steps": steps_h, "policy": args.policy,
                                    "autoreset": True, "mismatched_envs": bad,
                                    "error_flags": gerr, "bit_exact": bad == 0 and gerr == 0}
        for pol, w, b, k, e, got, where in checks:
            want = oracle_episodes(pol, w + b + k, w + b, e, args.level)
            chk = {"envs": e, "policy": pol, "steps": [w + b, w + b + k],
                   "gathered": got[0], "digest": got[1],
                   "oracle": want[0], "oracle_digest": want[1],
                   "match": tuple(got) == tuple(want),
                   "what": "episodes of global envs [0, E) ending in the timed steps, gathered "
                           "(tg_episodes -> dist.gather_padded -> EpisodeLog) vs the oracle's "
                           "auto-reset replay of those envs over every step of the run"}
            (line if where == "line" else line[where])["episode_check"] = chk
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
