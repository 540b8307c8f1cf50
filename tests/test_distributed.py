"""Multi-process (gloo, world_size 2, CPU) checks of the document sharding used by bench.py.

The replay path has no collective: each rank owns hash(doc) mod N.  These tests check that the shards
partition the documents exactly, and that the post-timing counter reduction (MAX of elapsed, SUM of
counters) gives the same totals as a single process replaying every document.  The per-rank replay here
is the CPU oracle (test infrastructure); on the GPU box the same host code drives the HIP engine.
"""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total_docs, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist
    from fluidframework_amd.sharding import reduce_counters, shard_docs
    from pyloggen import LogBatch, make_cfg
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard_docs(total_docs, world, rank)
        shards = [None] * world
        dist.all_gather_object(shards, mine)
        cfg = make_cfg(seed=7, n_clients=4, n_ops=300, lag=16)
        ops = 0
        csum = 0
        for g in mine:
            lb = LogBatch(cfg, g, g + 1, threads=1)
            ops += lb.docs[0].ops_applied
            csum = (csum + lb.docs[0].digest) % (1 << 64)  # the per-rank checksum bench.py reduces
        el, (ops_t, csum_t, nd) = reduce_counters(dist, "cpu", float(rank + 1), [ops, csum, len(mine)])
        q.put((rank, shards, el, ops_t, csum_t, nd))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_and_reduction():
    total = 40
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    shards = res[0][1]
    flat = sorted(g for s in shards for g in s)
    assert flat == list(range(total))                   # complete
    assert len(set(shards[0]) & set(shards[1])) == 0    # disjoint
    assert min(len(s) for s in shards) > 0
    for r in res:
        assert r[2] == 2.0                              # MAX over ranks
    # single-process totals
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from pyloggen import LogBatch, make_cfg
    cfg = make_cfg(seed=7, n_clients=4, n_ops=300, lag=16)
    ops = 0
    csum = 0
    for g in range(total):
        lb = LogBatch(cfg, g, g + 1, threads=1)
        ops += lb.docs[0].ops_applied
        csum = (csum + lb.docs[0].digest) % (1 << 64)
    for r in res:
        assert r[3] == ops and r[5] == total
        assert r[4] == csum  # reduced checksum (uint64 wrap-around) == the single-process one


def test_shard_docs_rejects_bad_rank():
    from fluidframework_amd.sharding import shard_docs
    with pytest.raises(ValueError):
        shard_docs(10, 2, 2)
    assert shard_docs(10, 1, 0) == list(range(10))
