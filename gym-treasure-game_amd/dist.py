"""Multi-GPU sharding of the env batch (one process per GPU, torch.distributed over RCCL).

The envs share nothing, so the batch partitions into contiguous shards with no data-path
collective: rank r owns global envs [offset, offset + count) and seeds/acts by GLOBAL index,
so every env's trajectory is the same for any world size.  The only exchange is the gather of
completed-episode records (env, return, length) that auto-reset produces: a count exchange
followed by one padded all-gather (a few KB per step over xGMI).
"""
import torch
import torch.distributed as dist


def shard(n_total, rank, world):
    """Contiguous shard of ``n_total`` envs for ``rank``: (global_offset, count)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n_total), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_episodes(records, group=None):
    """All-gather variable-length int64 [k, 3] episode records from every rank.

    Returns the concatenation (rank order) on every rank.  Works on gloo (CPU tensors) and on
    the RCCL-backed ``nccl`` backend (device tensors)."""
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
