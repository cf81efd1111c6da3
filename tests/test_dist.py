"""Multi-rank path on CPU (gloo, world_size 2): the round-robin object
partition covers every object exactly once, per-rank results combine into
the single-process result, and the timing reduction is max-over-ranks.
The per-object work here is the CPU oracle (no GPU on this host); on the
GPU box bench.py runs the same partition with one HIP context per rank.
"""
import hashlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from storb_amd import partition

NOBJ = 23
OBJ_LEN = 5000


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def obj_digest(i):
    from oracle import coracle
    data = coracle.splitmix_bytes(0x5709B + i, OBJ_LEN)
    h = hashlib.sha256()
    for off, ln in partition.chunks_of(OBJ_LEN, 2048):
        from oracle import zfec_np
        k, m = zfec_np.get_k_and_m(ln)
        shares, _, _ = coracle.encode(k, m, data[off:off + ln])
        h.update(shares.tobytes())
    return h.digest()


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = list(partition.objects_for_rank(NOBJ, rank, world))
    digests = {i: obj_digest(i) for i in mine}
    gathered = [None] * world
    dist.all_gather_object(gathered, digests)
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        merged = {}
        for d in gathered:
            assert not set(d) & set(merged), "object encoded twice"
            merged.update(d)
        q.put((merged, float(t.item()), [len(d) for d in gathered]))
    dist.barrier()
    dist.destroy_process_group()


def test_partition_helpers():
    for world in (1, 2, 3, 8):
        seen = []
        for r in range(world):
            seen += list(partition.objects_for_rank(10000, r, world))
            assert all(partition.owner(i, world) == r
                       for i in partition.objects_for_rank(10000, r, world))
        assert sorted(seen) == list(range(10000))
    with pytest.raises(ValueError):
        partition.objects_for_rank(5, 2, 2)
    assert partition.chunks_of(10, 4) == [(0, 4), (4, 4), (8, 2)]
    assert partition.aggregate_rate([100, 100], [1.0, 2.0]) == 100.0


def test_two_rank_gloo_partition_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged, tmax, counts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(merged) == list(range(NOBJ))
    assert counts == [12, 11]
    assert tmax == 1.5
    for i in (0, 7, NOBJ - 1):
        assert merged[i] == obj_digest(i)
