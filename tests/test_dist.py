"""CPU (gloo) tests of the multi-GPU stream sharding and the stats all-gather that builds
the global frame index. The per-stream stats come from the oracle here (no
GPU); on a GPU box the same drp_dist calls run over RCCL with libdrp's kernels (bench.py)."""
import os
import random
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
import drp_dist  # noqa: E402

import _oracle as O  # noqa: E402
import _streams as S  # noqa: E402


def _streams(n, seed):
    rng = random.Random(seed)
    out = []
    for s in range(n):
        if s % 3 == 0:
            out.append(S.c2_stream(rng.randint(0, 40), seed=s, start=s * 100).tobytes())
        else:
            out.append(S.random_stream(rng, rng.randint(0, 30), blob_p=0.1, blob_max=300))
    return out


def _stats(wire):
    r = O.decode_batch(wire)
    ty = r["type"] & 0x3F
    return [r["nframes"], int((ty == 1).sum()), int((ty == 2).sum()), r["consumed"]]


@pytest.mark.parametrize("n,world", [(10, 3), (8192, 8), (5, 8), (0, 2), (7, 1)])
def test_shard_range_partitions(n, world):
    got = [drp_dist.shard_range(n, world, r) for r in range(world)]
    assert got[0][0] == 0 and got[-1][1] == n
    for (a, b), (c, d) in zip(got, got[1:]):
        assert b == c and a <= b
    sizes = [b - a for a, b in got]
    assert max(sizes) - min(sizes) <= 1
    assert max(sizes) == drp_dist.per_rank_slots(n, world)


def _worker(rank, world, port, nstreams, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        streams = _streams(nstreams, seed=42)
        lo, hi = drp_dist.shard_range(nstreams, world, rank)
        local = torch.tensor([_stats(w) for w in streams[lo:hi]] or np.zeros((0, 4)),
                             dtype=torch.int64).reshape(-1, 4)
        table = drp_dist.gather_stats(local, nstreams)
        base = np.concatenate([[0], np.cumsum(table[:, 0].numpy())[:-1]]) if nstreams else []
        q.put((rank, table.numpy().tolist(), list(map(int, base))))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,nstreams", [(2, 9), (3, 10)])
def test_gather_builds_global_index(world, nstreams):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nstreams, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process expectation: stats of every stream in global order + exclusive prefix
    streams = _streams(nstreams, seed=42)
    exp_table = [_stats(w) for w in streams]
    exp_base = [0]
    for st in exp_table[:-1]:
        exp_base.append(exp_base[-1] + st[0])
    # the global index is where each stream's frames start when all streams are decoded as one
    # concatenation of independently framed streams
    for rank, table, base in got:
        assert table == exp_table, rank
        assert base == exp_base, rank
