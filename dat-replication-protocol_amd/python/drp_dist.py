"""Multi-GPU sharding of independent replication streams.

One process per GPU, launched by torch.distributed. Streams are sharded in contiguous blocks,
so the all-gathered per-stream stats table is already in global stream order and its
exclusive prefix over `frames` is the global index of every stream's first frame. The gather
of the 32-byte `drp_stream_stats` records is the only collective: the data path itself never
crosses ranks (weak scaling).

Two transports for that one gather:
- `global_index_rccl`: libdrp's own RCCL communicator (drp_index_allgather, the C ABI a Node
  or C host uses too); torch.distributed only hands the RCCL unique id to every rank.
- `gather_stats` + `global_index_device`: torch.distributed's all_gather ("gloo" in the CPU
  tests and for rehearsing several ranks on one GPU, where RCCL refuses duplicate devices).
"""
import ctypes as C

import torch
import torch.distributed as dist

STATS_WORDS = 4  # drp_stream_stats: frames, changes, blobs, wire_bytes (u64 each)


def shard_range(nstreams, world, rank):
    """Contiguous block [lo, hi) of the global stream ids owned by `rank`; blocks differ in
    size by at most one stream."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    base, extra = divmod(nstreams, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def per_rank_slots(nstreams, world):
    """Slots per rank in the gathered table (the largest block; short blocks are padded)."""
    return -(-nstreams // world) if nstreams else 0


def gather_stats(local_stats, nstreams, group=None):
    """All-gather every rank's (n_local, 4) int64 stats into one (nstreams, 4) table in
    global stream order. Works for CUDA tensors (RCCL) and CPU tensors (gloo)."""
    world = dist.get_world_size(group)
    slots = per_rank_slots(nstreams, world)
    # gloo has no device all-gather: rehearsal runs of several ranks on one GPU stage via host
    cdev = torch.device("cpu") if dist.get_backend(group) == "gloo" else local_stats.device
    send = torch.zeros((slots, STATS_WORDS), dtype=torch.int64, device=cdev)
    send[: local_stats.shape[0]] = local_stats.to(cdev)
    recv = torch.empty((world * slots, STATS_WORDS), dtype=torch.int64, device=cdev)
    dist.all_gather_into_tensor(recv, send, group=group)
    keep = []
    for r in range(world):
        lo, hi = shard_range(nstreams, world, r)
        keep.append(recv[r * slots: r * slots + (hi - lo)])
    out = torch.cat(keep) if keep else recv[:0]
    return out.to(local_stats.device)


def global_index_device(ctx, table):
    """Exclusive prefix of frames over the gathered (nstreams, 4) CUDA table with libdrp's
    index-scan kernel: the global index of each stream's first frame."""
    from drp_amd import _chk  # local import: the CPU-only tests never need libdrp

    n = table.shape[0]
    base = torch.empty(n, dtype=torch.int64, device=table.device)
    if n:
        ctx.order_after_torch(table)  # the gather / cat / copy producing `table` ran on torch's stream
        _chk("drp_index_scan", ctx.L.drp_index_scan(ctx.h, C.c_void_p(table.data_ptr()), n,
                                                    C.c_void_p(base.data_ptr())))
        _chk("drp_synchronize", ctx.L.drp_synchronize(ctx.h))
    return base


def local_stats_device(ctx, results_t, stream_off_t):
    """(n_local, 4) int64 CUDA stats from a drp_decode_device result array."""
    n = stream_off_t.numel() - 1
    stats = torch.zeros((n, STATS_WORDS), dtype=torch.int64, device=stream_off_t.device)
    if n:
        from drp_amd import _chk

        ctx.order_after_torch(stats)  # the zero fill of `stats` ran on torch's stream
        _chk("drp_stream_stats_from_results",
             ctx.L.drp_stream_stats_from_results(ctx.h, C.c_void_p(results_t.data_ptr()),
                                                 C.c_void_p(stream_off_t.data_ptr()), n,
                                                 C.c_void_p(stats.data_ptr())))
        _chk("drp_synchronize", ctx.L.drp_synchronize(ctx.h))
    return stats


_comms = {}


def comm_for(ctx, group=None):
    """libdrp's RCCL communicator for this process group (created once): rank 0 makes the
    unique id, torch.distributed broadcasts its bytes, every rank joins with its ctx."""
    from drp_amd import Comm
    key = (id(group), ctx.h.value)
    if key not in _comms:
        obj = [Comm.new_id() if dist.get_rank(group) == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        _comms[key] = Comm(ctx, obj[0], dist.get_world_size(group), dist.get_rank(group))
    return _comms[key]


def close_comms():
    for c in _comms.values():
        c.close()
    _comms.clear()


def global_index_rccl(ctx, local_stats, nstreams, group=None):
    """All-gather of the (n_local, 4) int64 CUDA stats through drp_index_allgather (RCCL) and
    the global index scan on this GPU; returns (table, base) in global stream order."""
    world = dist.get_world_size(group)
    slots = per_rank_slots(nstreams, world)
    dev = local_stats.device
    send = torch.zeros((slots, STATS_WORDS), dtype=torch.int64, device=dev)
    send[: local_stats.shape[0]] = local_stats
    table = torch.empty((world * slots, STATS_WORDS), dtype=torch.int64, device=dev)
    base = torch.empty(world * slots, dtype=torch.int64, device=dev)
    comm_for(ctx, group).allgather_index(ctx, send, table, base)
    keep = [torch.arange(r * slots, r * slots + (hi - lo), device=dev)
            for r, (lo, hi) in ((r, shard_range(nstreams, world, r)) for r in range(world))]
    idx = torch.cat(keep) if keep else torch.zeros(0, dtype=torch.int64, device=dev)
    return table[idx], base[idx]
