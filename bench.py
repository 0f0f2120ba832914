#!/usr/bin/env python3
"""Benchmark: batched Treasure Game env-steps/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs ENVS_PER_GPU]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One "step" = one TreasureGame.step() (TG/:91-96) of EVERY env of the batch: the on-device
synthetic policy writes the actions (uniform over the 9 options, counter hash keyed by the
global env index), tg_step runs each env's option to completion with auto-reset (k_classify
then k_run).  Every G steps (--gather-every, default 10) the completed episodes are drained
from the device queue and, for N > 1, all-gathered over RCCL.  Per-GPU work is fixed (1,048,576 envs per GPU = config C3, C4 at 8 GPUs), so scaling
is weak.  Inputs are resident in HBM when the timed region starts.

Prints ONE JSON line (rank 0) with the driver's fields plus ``roofline`` (tg_step's kernels:
algorithmic bytes per launch over their HIP-event-timed duration vs the 8 TB/s HBM peak) and
``cpu_baseline`` (the C oracle timed on this box's host cores, a bounded sample).

``--workload c5`` is config C5 instead: 65,536 envs per GPU whose step also renders every
env's screen (ObservationWrapper, TG/:38-51: tg_render -> k_render, 1,257,984 B per frame,
synthetic sprite sheet); its roofline is k_render's frame bytes over its HIP-event time.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (whole node) at 1M batched envs, 1/2/4/8 MI355X; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ACTION_SEED = 0x5EED0001
EP_CAP = 4096          # episode records gathered per rank per step of a drain interval (padded)
# algorithmic bytes of one tg_step, per launch:
#   every env: action 4 + state word 16 read (classify)
#   reward-None env: angles 16 + episode 8 read; episode 8 + obs 72 + reward/valid/done 6 written
#   valid env: worklist index 4 + 4, state 16 + 16, angles 16 + 16, episode 8 + 8, obs 72, rows 6
#   random() draw: one 8-B value (the pre-twisted generation's doubles)
#   MT regeneration: 624 words read, 624 words + 312 values written
BYTES_ENV, BYTES_INVALID, BYTES_VALID, BYTES_DRAW, BYTES_REGEN = 20, 110, 166, 8, 7488
# algorithmic bytes of one k_render launch per env: the frame written (H*48 x W*48 x 3 =
# 1,257,984 for the default level) + the env's state words read (st4 16 + angles 16)
BYTES_RENDER_STATE = 32


def alg_bytes(st):
    inval = st["steps"] - st["valid_steps"]
    return (BYTES_ENV * st["steps"] + BYTES_INVALID * inval + BYTES_VALID * st["valid_steps"] +
            BYTES_DRAW * st["draws"] + BYTES_REGEN * st["regens"])


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="c3", choices=["c3", "c5"],
                    help="c3: vector-obs step (default, the headline); c5: step + RGB render")
    ap.add_argument("--envs", type=int, default=None,
                    help="envs per GPU (default 1,048,576 for c3, 65,536 for c5)")
    ap.add_argument("--policy", default="uniform", choices=["uniform", "masked"])
    ap.add_argument("--no-autoreset", action="store_true")
    ap.add_argument("--mode", default="compact", choices=["compact", "direct"],
                    help="step implementation (bit-identical): two-pass compacted or one-pass")
    ap.add_argument("--run-blocks", type=int, default=0, help="k_run workgroups (0 = default)")
    ap.add_argument("--rollout", type=int, default=0,
                    help="K > 0: tg_rollout, K steps per call with the policy evaluated inside "
                         "the step kernels (episodes drained / gathered every K steps); 0: the "
                         "per-step API (tg_policy_actions + tg_step per step)")
    ap.add_argument("--gather-every", type=int, default=10,
                    help="per-step API: drain (and, N > 1, all-gather) the completed episodes "
                         "every G steps (SURVEY §8e: batched gather; 1 = every step). "
                         "--rollout K drains every K steps")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target duration of the CPU-baseline sample (0 disables it)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_step.json"),
                    help="PMC-derived HBM bytes per tg_step (profiles/), if measured")
    return ap.parse_args()


def cpu_baseline(seconds, policy):
    """The C oracle (oracle/, the CPU restatement of the reference) on this box's host cores:
    a bounded sample of the same workload (same seeds, action stream and auto-reset)."""
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
    n = max(threads * 64, int(n * seconds / max(dt, 1e-3)))
    t0 = time.perf_counter()
    O.run(0, 0, n, steps, ACTION_SEED, pol, True, full=False, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "C oracle (oracle/tg_oracle.c, CPU restatement of the reference step path), "
                      "envs 0..%d x %d steps, %s policy, auto-reset, %d OpenMP threads, %.1f s"
                      % (n - 1, steps, policy, threads, dt),
            "reference_python_1core_measured_in_build_container": 14400.0}


def cpu_baseline_render(seconds, policy):
    """C5's CPU leg: the oracle's renderer restatement (plus construct/reset and one step per
    env) on this box's host cores, synthetic sprites."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
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


def main():
    args = parse()
    c5 = args.workload == "c5"
    if args.envs is None:
        args.envs = 65536 if c5 else 1 << 20
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus %d needs torch.distributed.run with %d processes"
                             % (args.gpus, args.gpus))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    import gym_treasure_game_amd as tg
    import gym_treasure_game_amd.dist as D

    total = args.envs * world
    offset, count = D.shard(total, rank, world)
    autoreset = not args.no_autoreset
    vec = tg.TreasureGameVec(count, seed=0, global_offset=offset, autoreset=False, device=dev)
    vec.set_mode(args.mode, args.run_blocks)
    vec.autoreset = autoreset  # final_obs is not requested: obs/reward/valid/done only
    vec.reset()
    K = args.rollout
    G = K if K else args.gather_every
    if G < 1:
        raise SystemExit("--gather-every must be >= 1")
    ep_cap = EP_CAP * G  # records per rank per drain (padded; the rest stays queued)
    ep_rows = torch.empty((ep_cap, 2), dtype=torch.int64, device=dev)
    ep_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    gathered = torch.zeros(1, dtype=torch.int64, device=dev)  # records seen by this rank
    if world > 1:
        all_rows = torch.empty((world * ep_cap, 2), dtype=torch.int64, device=dev)
        all_cnt = torch.empty(world, dtype=torch.int32, device=dev)
    L, h = vec._L, vec.handle
    obs, rew, val, don = vec._obs, vec._rew, vec._valid, vec._done
    act = vec._act
    flags = tg._lib.TG_STEP_AUTORESET if autoreset else 0
    import ctypes
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    pol = tg._lib.TG_POLICY_MASKED if args.policy == "masked" else tg._lib.TG_POLICY_UNIFORM
    args_step = (h, p(act), p(obs), p(rew), p(val), p(don), None, flags, stream)

    frames, rev = None, []
    if c5:  # ObservationWrapper.step: render every env's screen after its step
        vec.render_init(tg.synthetic_sprites(seed=1))
        frames = torch.empty((count,) + vec.frame_shape, dtype=torch.uint8, device=dev)
    timing = [False]

    if K:
        if c5 or args.steps % K or args.warmup % K:
            raise SystemExit("--rollout K: c3 only, with --steps and --warmup multiples of K")
        roll = [torch.empty((K, count), dtype=d, device=dev)
                for d in (torch.int32, torch.uint8, torch.uint8)]

    def one_step(t):
        if K:  # steps t .. t+K-1 in one call
            if t % K:
                return
            tg._lib.check(L.tg_rollout(h, K, ACTION_SEED, t, pol, flags, None, None,
                                       p(roll[0]), p(roll[1]), p(roll[2]), stream), "rollout")
        else:
            tg._lib.check(L.tg_policy_actions(h, ACTION_SEED, t, pol, p(act), stream), "actions")
            tg._lib.check(L.tg_step(*args_step), "tg_step")
        if (t + 1) % G == 0 or K:
            drain()
        if c5:
            if timing[0]:  # k_render alone, on the stream it is launched on
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            tg._lib.check(L.tg_render(h, 0, count, p(frames), stream), "tg_render")
            if timing[0]:
                ev[1].record()
                rev.append(ev)

    def drain():
        tg._lib.check(L.tg_episodes(h, p(ep_rows), p(ep_cnt), ep_cap, stream), "episodes")
        if world > 1:  # the one collective: completed episodes over RCCL/xGMI
            dist.all_gather_into_tensor(all_cnt, ep_cnt)
            dist.all_gather_into_tensor(all_rows, ep_rows)
            gathered.add_(all_cnt.sum())
        else:
            gathered.add_(ep_cnt[0])

    for t in range(args.warmup):
        one_step(t)
    drain()  # empty the queue, so the timed region's records are its own
    torch.cuda.synchronize(dev)
    gathered.zero_()
    vec.stats_reset()
    vec.set_timing(True)
    timing[0] = True
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + args.steps):
        one_step(t)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = vec.stats()
    errs = vec.errors()
    if world > 1:
        dt_t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dt = float(dt_t.item())
        keys = ["steps", "ticks", "draws", "valid_steps", "episodes", "wave_ticks"]
        tot = torch.tensor([st[k] for k in keys], dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        node = dict(zip(keys, tot.tolist()))
    else:
        node = {k: st[k] for k in ("steps", "ticks", "draws", "valid_steps", "episodes",
                                   "wave_ticks")}

    if rank == 0:
        env_steps = total * args.steps
        assert node["steps"] == env_steps, (node, env_steps)
        launches = max(st["launches"], 1)
        kern_s = st["kernel_ms"] / 1e3 / launches
        alg = alg_bytes(st) / launches
        achieved = alg / kern_s / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            tj = json.load(open(args.traffic_json))
            if (tj.get("envs") == args.envs and tj.get("policy") == args.policy
                    and tj.get("mode", "direct") == args.mode):
                traffic = tj.get("hbm_bytes_per_launch")
        roof = {"bound": "hbm",
                "kernel": ("tg_step = k_classify + k_run" if args.mode == "compact"
                           else "tg_step = k_step"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic, "kernel_ms": kern_s * 1e3,
                "alg_bytes_per_launch": alg}
        workload = ("C3/C4: %d batched treasure_game-v0 envs per GPU, vector obs, %s random "
                    "options, auto-reset%s" % (args.envs, args.policy,
                                               " + RCCL episode gather" if world > 1 else ""))
        extra = {}
        if c5:
            fh, fw, _ = vec.frame_shape
            r_ms = sum(a.elapsed_time(b) for a, b in rev) / max(len(rev), 1)
            r_alg = count * (fh * fw * 3 + BYTES_RENDER_STATE)
            r_ach = r_alg / (r_ms / 1e3) / 1e9
            r_traffic = None
            tj_path = os.path.join(ROOT, "profiles", "traffic_render.json")
            if os.path.exists(tj_path):
                tj = json.load(open(tj_path))
                if tj.get("envs") == count:
                    r_traffic = tj.get("hbm_bytes_per_launch")
            extra["step_roofline"] = roof
            roof = {"bound": "hbm", "kernel": "k_render (tg_render)", "achieved": r_ach,
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": r_ach / HBM_PEAK_GBS,
                    "traffic": r_traffic, "kernel_ms": r_ms, "alg_bytes_per_launch": r_alg}
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
                       "api": ("tg_rollout x%d (policy inside the step kernels)" % K if K
                               else "tg_policy_actions + tg_step per step"),
                       "parallelism": "env-shard x%d" % world},
            "ticks_per_s": node["ticks"] / dt,
            # ticks executed / lane-ticks issued by the tick loops' wavefronts
            "lane_efficiency": node["ticks"] / max(64 * node["wave_ticks"], 1),
            "valid_step_frac": node["valid_steps"] / max(node["steps"], 1),
            "draws_per_step": node["draws"] / max(node["steps"], 1),
            "episodes": node["episodes"], "error_flags": errs,
            "gather_every": G, "episodes_gathered": int(gathered.item()),
            "regens_per_step": st["regens"] / launches,
            "roofline": roof,
        }
        line.update(extra)
        if args.cpu_seconds > 0 and world == 1:
            line["cpu_baseline"] = (cpu_baseline_render if c5 else cpu_baseline)(
                args.cpu_seconds, args.policy)
        print(json.dumps(line), flush=True)
    vec.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
