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


MASK64 = (1 << 64) - 1


def _as_i64(x: int) -> int:
    v = int(x) & MASK64
    return v - (1 << 64) if v >= (1 << 63) else v


def reduce_counters(dist, device, elapsed: float, counters):
    """MAX-reduce `elapsed` and SUM-reduce the integer `counters` (mod 2^64) over the process group.

    The counters are unsigned 64-bit values: ops applied, errors, bytes and the per-rank checksum (the sum
    of its documents' state digests mod 2^64), carried in int64 two's complement so that
    one all-reduce (RCCL on the GPU box, gloo in the CPU tests) sums them with wrap-around.
    Returns (elapsed_max, [summed counters]).  `dist` is torch.distributed (already initialised).
    """
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([_as_i64(x) for x in counters], dtype=torch.int64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(x) & MASK64 for x in c.tolist()]
