"""Document sharding across GPUs (one process per GPU).

Documents are independent (each SharedString replays its own sequenced op stream), so a multi-GPU job
partitions them by a hash of the document index and never exchanges data on the replay path.  The only
collective is a counter reduction after the timed region (ops applied, errors, parity mismatches, and
the max elapsed time over ranks), done by `reduce_counters` on whichever process group the caller
initialised (RCCL on the GPU box, gloo in the CPU tests).
"""


def fnv32(x: int) -> int:
    """FNV-1a over the 8 little-endian bytes of a document index."""
    h = 2166136261
    for b in int(x).to_bytes(8, "little"):
        h = ((h ^ b) * 16777619) & 0xFFFFFFFF
    return h


def shard_docs(total_docs: int, world: int, rank: int):
    """Global document indices owned by `rank` (hash(doc) mod world)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    return [g for g in range(total_docs) if fnv32(g) % world == rank]


def reduce_counters(dist, device, elapsed: float, counters):
    """MAX-reduce `elapsed` and SUM-reduce the integer `counters` over the process group.

    Returns (elapsed_max, [summed counters]).  `dist` is torch.distributed (already initialised).
    """
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([int(x) for x in counters], dtype=torch.int64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(x) for x in c.tolist()]
