"""Multi-GPU sharding of the env batch (one process per GPU, torch.distributed over RCCL).

The envs share nothing, so the batch partitions into contiguous shards with no data-path
collective: rank r owns global envs [offset, offset + count) and seeds/acts by GLOBAL index,
so every env's trajectory is the same for any world size.  The only exchange is the gather of
completed-episode records (env, return, length) that auto-reset produces:

* ``gather_padded`` — the bench's collective: every rank's drained queue (a fixed-size buffer
  of raw 16-B ``tg_episode`` rows + its record count, written on the device by
  ``tg_episodes``) is all-gathered as two fixed-size tensors, so no host sync sits between
  the drain and the collective;
* ``EpisodeLog`` — rank 0 keeps every gathered buffer on the device during the timed loop and
  reduces them afterwards to a record count and an order-independent digest of
  (env, return, length), which must not depend on the world size;
* ``spawn_ranks`` — ``bench.py --gpus N`` without an external launcher starts its N ranks as
  fresh child processes (before anything touches the GPU) with the torch.distributed
  environment of ``torch.distributed.run``.

All of it runs on gloo with CPU tensors too (tests/test_dist.py runs the exact functions the
bench calls, world sizes 1-3).
"""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def shard(n_total, rank, world):
    """Contiguous shard of ``n_total`` envs for ``rank``: (global_offset, count)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n_total), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


# ---- the bench's gather ---------------------------------------------------------------------
def gather_padded(rows, count, all_rows=None, all_count=None, group=None):
    """All-gather one drain of every rank's episode queue.

    ``rows``: int64 [cap, 2], the raw ``tg_episode`` records (env; return | length << 32) of
    this rank, of which the first ``count[0]`` are valid; ``count``: int32 [1].  Both sizes
    are fixed, so the collective needs no host-side count.  Returns ``(all_rows [world*cap,
    2], all_count [world])``: rank r's records are ``all_rows[r*cap : r*cap + all_count[r]]``.
    With one rank (or no process group) it returns the inputs, reshaped.  ``all_rows`` /
    ``all_count`` may be given preallocated (the bench does, outside its timed loop)."""
    if rows.dim() != 2 or rows.size(1) != 2 or rows.dtype != torch.int64:
        raise ValueError("rows must be int64 [cap, 2]")
    if count.numel() != 1 or count.dtype != torch.int32:
        raise ValueError("count must be int32 [1]")
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world == 1:
        return rows, count.view(1)
    if all_rows is None:
        all_rows = rows.new_empty((world * rows.size(0), 2))
    if all_count is None:
        all_count = count.new_empty(world)
    dist.all_gather_into_tensor(all_count, count.view(1), group=group)
    dist.all_gather_into_tensor(all_rows, rows, group=group)
    return all_rows, all_count


def _sm64(x):
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def episode_digest(rows, counts, cap, env_below=None):
    """(records, digest) of gathered episode buffers: ``rows`` int64 [k*cap, 2] raw records
    and ``counts`` [k] valid records per cap-sized segment (any device).  The digest is the
    sum mod 2^64 of sm64(sm64(env) ^ (return | length << 32)) over the valid records, so it
    depends on the set of (env, return, length) only: not on their order, on the ranks that
    produced them or on the drain interval.  ``env_below``: only the records of global envs
    [0, env_below) (the bench compares those with the oracle's replay)."""
    r = rows.detach().cpu().numpy().reshape(-1, cap, 2)
    c = counts.detach().cpu().numpy().astype(np.int64).reshape(-1)
    if len(c) != r.shape[0]:
        raise ValueError("counts must have one entry per cap-sized segment")
    if np.any(c < 0) or np.any(c > cap):
        raise ValueError("a segment count is outside [0, cap]")
    valid = np.arange(cap)[None, :] < c[:, None]
    v = r[valid]
    if env_below is not None:
        v = v[v[:, 0] < env_below]
    v = v.view(np.uint64)
    with np.errstate(over="ignore"):
        h = _sm64(_sm64(v[:, 0]) ^ v[:, 1])
        digest = int(np.sum(h, dtype=np.uint64))
    return len(v), digest


def records_digest(env, ret, length):
    """episode_digest of explicit (env, return, length) arrays (tests, host checks)."""
    env = np.asarray(env, np.int64)
    packed = (np.asarray(ret, np.int64) & 0xFFFFFFFF) | (np.asarray(length, np.int64) << 32)
    rows = np.stack([env, packed], 1) if len(env) else np.zeros((0, 2), np.int64)
    cap = max(len(env), 1)
    pad = np.zeros((cap, 2), np.int64)
    pad[:len(env)] = rows
    return episode_digest(torch.from_numpy(pad), torch.tensor([len(env)]), cap)


class EpisodeLog:
    """Rank 0's record of every gathered drain, kept on the device during the timed loop (one
    device copy per drain, no host sync) and reduced to (records, digest) afterwards."""

    def __init__(self, drains, world, cap, device, keep=True):
        self.cap, self.world, self.keep = int(cap), int(world), bool(keep)
        n = max(int(drains), 1) if keep else 1
        self.rows = torch.zeros((n, world * cap, 2), dtype=torch.int64, device=device)
        self.counts = torch.zeros((n, world), dtype=torch.int32, device=device)
        self.records = torch.zeros(1, dtype=torch.int64, device=device)
        self.used = 0

    def target(self):
        """``(rows [world*cap, 2], counts [world])``: the next drain's slot, for the drain
        (``tg_episodes``) or the all-gather to write in place, then ``commit()``: one launch
        per drain instead of a drain, its gather and two copies (the bench)."""
        if not self.keep:
            return self.rows[0], self.counts[0]
        if self.used >= self.rows.size(0):  # more drains than sized for: grow (allocates)
            self.rows = torch.cat([self.rows, torch.zeros_like(self.rows)])
            self.counts = torch.cat([self.counts, torch.zeros_like(self.counts)])
        return self.rows[self.used], self.counts[self.used]

    def commit(self):
        """the slot from ``target()`` now holds a drain"""
        if self.keep:
            self.used += 1
        else:  # one reused slot: its count is added up at once
            self.records.add_(self.counts[0].sum())

    def add(self, all_rows, all_count):
        """a drain gathered elsewhere, copied into the next slot"""
        rows, counts = self.target()
        if self.keep or rows.data_ptr() != all_rows.data_ptr():
            rows.copy_(all_rows, non_blocking=True)
            counts.copy_(all_count, non_blocking=True)
        self.commit()

    def reset(self):
        self.records.zero_()
        self.used = 0

    def digest(self, env_below=None):
        """(records, digest) over every drain added since the last reset (synchronises);
        ``env_below``: of the records of global envs [0, env_below) only."""
        if not self.keep:
            return int(self.records.item()), None
        n = self.used
        return episode_digest(self.rows[:n].reshape(-1, 2), self.counts[:n].reshape(-1), self.cap,
                              env_below)


# ---- the launcher ---------------------------------------------------------------------------
def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, script=None, env=None, poll_s=0.2):
    """Start ``n`` ranks of ``script`` (default: the running script) as fresh child processes
    with the environment torch.distributed.run would give them (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), wait for them, and return rank 0's
    exit code.  The parent must not have touched the GPU (it only forks plain processes).
    If a rank fails, the others are terminated (they would wait forever in a collective) and
    the failing code is returned."""
    script = script or os.path.abspath(sys.argv[0])
    port = free_port()
    procs = []
    for r in range(n):
        e = dict(os.environ if env is None else env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                  "LOCAL_WORLD_SIZE": str(n), "GROUP_RANK": "0",
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=e))
    rcs = [None] * n
    failed = None
    while any(rc is None for rc in rcs):
        for r, p in enumerate(procs):
            if rcs[r] is None:
                rcs[r] = p.poll()
                if rcs[r] not in (None, 0) and failed is None:
                    failed = rcs[r]
        if failed is not None:
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    p.terminate()
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    try:
                        rcs[r] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[r] = p.wait()
            return failed
        time.sleep(poll_s)
    return rcs[0]


# ---- variable-length gather (host-side helper) -----------------------------------------------
def gather_episodes(records, group=None):
    """All-gather variable-length int64 [k, 3] (env, return, length) records from every rank.

    Returns the concatenation (rank order) on every rank.  Works on gloo (CPU tensors) and on
    the RCCL-backed ``nccl`` backend (device tensors).  Synchronises on the counts; the bench
    uses ``gather_padded`` instead."""
    world = dist.get_world_size(group)
    if records.dim() != 2 or records.size(1) != 3:
        raise ValueError("records must be [k, 3]")
    dev = records.device
    k = torch.tensor([records.size(0)], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(k) for _ in range(world)]
    dist.all_gather(counts, k, group=group)
    counts = [int(c.item()) for c in counts]
    cap = max(counts)
    if cap == 0:
        return records.new_zeros((0, 3))
    pad = records.new_zeros((cap, 3))
    pad[: records.size(0)] = records
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[:c] for o, c in zip(outs, counts)], dim=0)
