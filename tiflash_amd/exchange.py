"""MPP exchange between ranks (one process per GPU) — the ExchangeSender -> ExchangeReceiver
repartition of the reference (Flash/Mpp/HashPartitionWriter.cpp:139-204 -> MPPTunnelSet ->
Flash/Mpp/ExchangeReceiver.cpp:626-945) as collectives over torch.distributed ("nccl" = RCCL
over xGMI on MI355X; "gloo" on CPU for the multi-process tests).

The sender side is tfg_hash_partition (weak hash -> fillSelector -> stable scatter): its output is
partition-major, partition p = rows [offsets[p], offsets[p+1]), which is exactly an all-to-all
send buffer, so an exchange is one counts all-to-all plus one all_to_all_single per column.
"""
from typing import List, Sequence

import torch
import torch.distributed as dist


def exchange_partitions(cols: Sequence[torch.Tensor], offsets: Sequence[int], group=None) -> List[torch.Tensor]:
    """Sends rows [offsets[p], offsets[p+1]) of every column to rank p; returns the received
    columns, rows from rank 0 first (ExchangeReceiver's concatenation order is unspecified in
    the reference; consumers must not depend on it)."""
    world = dist.get_world_size(group)
    if len(offsets) != world + 1:
        raise ValueError(f"need {world + 1} partition offsets, got {len(offsets)}")
    dev = cols[0].device
    if dev.type != "cpu" and dist.get_backend(group) == "gloo":
        # gloo moves host memory only: stage through the host (rehearsal of the N>1 path on one
        # GPU; the production backend is "nccl" = RCCL, which exchanges device buffers directly)
        outs = exchange_partitions([c.cpu() for c in cols], offsets, group)
        return [o.to(dev) for o in outs]
    send_counts = [int(offsets[p + 1] - offsets[p]) for p in range(world)]
    send = torch.tensor(send_counts, dtype=torch.int64, device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    recv_counts = recv.tolist()
    outs = []
    for c in cols:
        c = c[: int(offsets[world])]
        o = torch.empty((sum(recv_counts),) + tuple(c.shape[1:]), dtype=c.dtype, device=dev)
        dist.all_to_all_single(o, c.contiguous(), recv_counts, send_counts, group=group)
        outs.append(o)
    return outs


def two_phase_merge_keys(ctx, partial, final, group=None, collators=None):
    """ExchangeSender -> ExchangeReceiver of a two-phase GROUP BY over String / several keys
    (C5): the partial aggregation's rows are routed by the reference's hash of the key columns
    (IColumn::updateWeakHash32 -> fillSelector, HashBaseWriterHelper.cpp:46-84), travel as packed
    16-byte keys plus states, and the final aggregation merges them (mergeOnBlock).  `partial` and
    `final` are tiflash_amd.KeysAggregator objects of the same signature."""
    import tiflash_amd as tfa
    world = dist.get_world_size(group)
    packed = partial.result_packed()
    cols = partial.result()
    n = packed["keys"].shape[0]
    h = torch.empty(n, dtype=torch.int32, device=packed["keys"].device)
    tfa.check(tfa.lib().tfg_weak_hash_init(ctx.h, tfa._p(h), tfa.ctypes.c_int64(n)))
    for j, (t, k, kn) in enumerate(zip(partial.key_types, cols["keys"], cols["key_null"])):
        if t == tfa.STRING:
            tfa.weak_hash_string(ctx, k[0], k[1], h, nullmap=kn, collator=(collators or [0] * 4)[j])
        else:
            tfa.weak_hash(ctx, [k], types=[t], nullmaps=[kn], h=h)
    sel = tfa.fill_selector(ctx, h, world)
    perm, offs = tfa.partition(ctx, sel, world)
    send = tfa.gather(ctx, perm, [packed["keys"]] + list(packed["states"]))
    recv = exchange_partitions(send, offs, group)
    final.consume_partial_packed(recv[0], recv[1:])
