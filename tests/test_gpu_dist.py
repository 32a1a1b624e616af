"""GPU: the multi-GPU index chain with libdrp's own stats.

- drp_index_allgather (RCCL inside libdrp) on a one-rank communicator and drp_comm_init_all on
  one device: the gathered table equals the local one and the index is its exclusive scan.
- Two ranks (gloo, both on this GPU: RCCL refuses two ranks on one device), each decoding its
  contiguous block of streams with libdrp (drp_decode_device -> drp_stream_stats_from_results),
  gathering the stats and scanning them with drp_index_scan: every stream's global index and
  counts equal a single-process decode of all streams."""
import ctypes as C
import os
import random
import sys

import numpy as np
import pytest
import torch

import _streams as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _streams(n, seed=5):
    rng = random.Random(seed)
    out = []
    for s in range(n):
        k = s % 3
        if k == 0:
            out.append(S.c2_stream(rng.randint(0, 300), seed=s).tobytes())
        elif k == 1:
            out.append(S.random_stream(rng, rng.randint(0, 50), blob_p=0.1, blob_max=5000))
        else:
            w = S.random_stream(rng, rng.randint(1, 40))
            out.append(w[:rng.randint(0, len(w))])
    return out


def _decode_stats(ctx, streams, dev):
    import drp_dist
    from _gpu import drp_amd
    offs = np.concatenate([[0], np.cumsum([len(w) for w in streams])]).astype(np.int64)
    wire = np.frombuffer(b"".join(streams), np.uint8)
    wire_t = torch.from_numpy(wire.copy()).to(dev) if wire.size else torch.zeros(16, dtype=torch.uint8, device=dev)
    so_t = torch.from_numpy(offs).to(dev)
    cap = int(wire.size) // 2 + 64
    outs = {"payload_off": torch.zeros(cap, dtype=torch.int64, device=dev),
            "payload_len": torch.zeros(cap, dtype=torch.int32, device=dev),
            "type": torch.zeros(cap, dtype=torch.uint8, device=dev),
            "flags": torch.zeros(cap, dtype=torch.uint8, device=dev)}
    for k in drp_amd.COLS32:
        outs[k] = torch.zeros(cap, dtype=torch.int32, device=dev)
    for k in drp_amd.COLS64:
        outs[k] = torch.zeros(cap, dtype=torch.int64, device=dev)
    res_t = torch.zeros(len(streams) * C.sizeof(drp_amd.StreamResult), dtype=torch.uint8, device=dev)
    ctx.decode_device(wire_t, so_t, None, outs, cap, res_t)
    return drp_dist.local_stats_device(ctx, res_t, so_t)


def test_rccl_allgather_one_rank():
    import drp_dist  # noqa: F401
    from _gpu import drp_amd
    dev = torch.device("cuda", 0)
    streams = _streams(57)
    with drp_amd.Ctx(0) as ctx:
        stats = _decode_stats(ctx, streams, dev)
        comm = drp_amd.Comm(ctx, drp_amd.Comm.new_id(), 1, 0)
        try:
            table = torch.empty_like(stats)
            base = torch.empty(stats.shape[0], dtype=torch.int64, device=dev)
            comm.allgather_index(ctx, stats, table, base)
        finally:
            comm.close()
        # one process driving its devices (here one): drp_comm_init_all + the grouped form
        comms = (C.c_void_p * 1)()
        ctxs = (C.c_void_p * 1)(ctx.h)
        drp_amd._chk("drp_comm_init_all", ctx.L.drp_comm_init_all(ctxs, 1, comms))
        try:
            table2 = torch.empty_like(stats)
            base2 = torch.empty(stats.shape[0], dtype=torch.int64, device=dev)
            ptr = lambda t: (C.c_void_p * 1)(t.data_ptr())
            ctx.order_after_torch(stats)
            drp_amd._chk("drp_index_allgather_multi",
                         ctx.L.drp_index_allgather_multi(ctxs, comms, 1, ptr(stats), stats.shape[0], ptr(table2),
                                                         ptr(base2)))
        finally:
            ctx.L.drp_comm_destroy(comms[0])
    f = stats[:, 0]
    exp = torch.cumsum(f, 0) - f
    assert torch.equal(table, stats) and torch.equal(base, exp)
    assert torch.equal(table2, stats) and torch.equal(base2, exp)


def _rank(rank, world, port, streams, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        sys.path.insert(0, os.path.join(ROOT, "dat-replication-protocol_amd", "python"))
        import torch.distributed as dist
        import _gpu  # noqa: F401  (torch's HIP runtime first)
        import drp_dist
        from _gpu import drp_amd
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        lo, hi = drp_dist.shard_range(len(streams), world, rank)
        with drp_amd.Ctx(0) as ctx:
            stats = _decode_stats(ctx, streams[lo:hi], dev)
            table = drp_dist.gather_stats(stats, len(streams))
            base = drp_dist.global_index_device(ctx, table)
        q.put((rank, table.cpu().numpy(), base.cpu().numpy()))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put((rank, repr(e), None))


def test_two_ranks_gloo_libdrp_stats():
    import torch.multiprocessing as mp
    from _gpu import drp_amd  # noqa: F401
    dev = torch.device("cuda", 0)
    streams = _streams(101, seed=9)
    with drp_amd.Ctx(0) as ctx:
        ref = _decode_stats(ctx, streams, dev).cpu().numpy()
    ref_base = np.cumsum(ref[:, 0]) - ref[:, 0]
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = 29500 + random.Random().randint(0, 2000)
    procs = [mpc.Process(target=_rank, args=(r, 2, port, streams, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, table, base in got:
        assert base is not None, table
        np.testing.assert_array_equal(table, ref, err_msg=f"rank {rank}")
        np.testing.assert_array_equal(base, ref_base, err_msg=f"rank {rank}")
