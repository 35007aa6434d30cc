"""MPP exchange between ranks (one process per GPU) — the ExchangeSender -> ExchangeReceiver
repartition of the reference (Flash/Mpp/HashPartitionWriter.cpp:139-204 -> MPPTunnelSet ->
Flash/Mpp/ExchangeReceiver.cpp:626-945).

The sender side is tfg_hash_partition (weak hash -> fillSelector -> stable scatter): its output is
partition-major, partition p = rows [offsets[p], offsets[p+1]) of every column.  An exchange moves
any number of columns and row sets ("sides", e.g. a join's build and probe sides, or a String
column's chars next to its rows) — the same exchange as the C++ boundary's tfa::MPPExchange
(host/operators.cpp), over the same ABI calls:

* ONE counts exchange (rows of each side per rank pair: tfg_alltoall_counts_n), one host read;
* ONE zero-copy exchange (tfg_exchange_slices: one RCCL group over xGMI): every (peer, column)
  slice is sent from where it lies in the partitioned column and received straight into the
  output column at its row offset — no pack / unpack copy, no packet encode / decode.

The RCCL communicator (tfg_comm) is made once per process group and context, its unique id
broadcast over torch.distributed.  On CPU tensors (gloo: the multi-process tests) the same
exchange is built with torch slicing and all_to_all_single; device tensors under gloo (a
rehearsal of the N>1 path on one GPU) are staged through the host.
"""
import ctypes
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist


def _row_width(c: torch.Tensor) -> int:
    """Bytes per row of a column, from its schema (dtype, trailing shape), not from its data, so
    a rank with no rows agrees with its peers on the layout."""
    w = c.element_size()
    for d in c.shape[1:]:
        w *= int(d)
    return w


def _row_bytes(c: torch.Tensor, n: int) -> torch.Tensor:
    """The first n rows of a column as an [n, row_bytes] uint8 view (copy only if strided)."""
    if n == 0:  # empty tensors may carry 0 strides, which view() refuses
        return torch.empty((0, _row_width(c)), dtype=torch.uint8, device=c.device)
    c = c[:n]
    if not c.is_contiguous():
        c = c.contiguous()
    return c.view(torch.uint8).reshape(n, _row_width(c))


_CTX = {}


class _Comm:
    """A tfg_comm owned by its context: destroyed by Context.close() (before tfg_ctx_destroy), so
    no communicator outlives the stream it enqueues on."""

    def __init__(self, h, group):
        self.h = h
        self.group = group  # held: the cache key is id(group), which must not be reused while we live

    def close(self):
        import tiflash_amd as tfa
        if self.h is not None and self.h.value:
            tfa.lib().tfg_comm_destroy(self.h)
        self.h = None


def _tfg_comm(ctx, group):
    """The tfg_comm (RCCL communicator) of a process group on a context; collective on first use.
    Cached on the context object itself (ctx._comms), so a closed context's communicators are gone
    with it and a new context never finds a stale one."""
    import tiflash_amd as tfa
    comms = ctx.__dict__.setdefault("_comms", {})
    key = id(group)
    if key not in comms:
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            tfa.check(tfa.lib().tfg_comm_unique_id(uid, ctypes.c_size_t(128)))
        obj = [bytes(uid)]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        tfa.check(tfa.lib().tfg_comm_init(ctx.h, ctypes.c_int(world), ctypes.c_int(rank), buf, ctypes.c_size_t(128),
                                          ctypes.byref(h)))
        c = _Comm(h, group)
        comms[key] = c
        ctx._children.add(c)
    return comms[key].h


class _Slice(ctypes.Structure):  # tfg_slice
    _fields_ = [("peer", ctypes.c_int), ("ptr", ctypes.c_void_p), ("bytes", ctypes.c_uint64)]


def _default_ctx(dev):
    """A tfg context on the current stream of `dev` (one per device and stream)."""
    import tiflash_amd as tfa
    st = torch.cuda.current_stream(dev)
    key = (dev.index, st.cuda_stream)
    if key not in _CTX:
        _CTX[key] = tfa.Context(dev.index if dev.index is not None else 0, stream=st)
    return _CTX[key]


def _empty_col(rows, dt, shp, dev):
    return torch.empty((rows,) + shp, dtype=dt, device=dev)


def exchange_sides(sides: Sequence[Tuple[Sequence[torch.Tensor], Sequence[int]]], group=None,
                   ctx=None) -> List[List[torch.Tensor]]:
    """sides: [(columns, offsets)], each side's rows partition-major (rows [offsets[p],
    offsets[p+1]) go to rank p; offsets are host ints).  Returns, per side, the received columns
    (rows from rank 0 first; ExchangeReceiver's concatenation order is unspecified in the
    reference and consumers must not depend on it).  ctx: the tfg context of device columns (a
    context on the current stream when None)."""
    world = dist.get_world_size(group)
    for _, offs in sides:
        if len(offs) != world + 1:
            raise ValueError(f"need {world + 1} partition offsets, got {len(offs)}")
    dev = sides[0][0][0].device
    if dev.type != "cpu" and dist.get_backend(group) == "gloo":
        # gloo moves host memory only: stage through the host (rehearsal of the N>1 path on one
        # GPU; the production backend is "nccl" = RCCL, which exchanges device buffers directly)
        outs = exchange_sides([([c.cpu() for c in cols], offs) for cols, offs in sides], group)
        return [[o.to(dev) for o in side] for side in outs]
    S = len(sides)
    # the planes, side by side, each side's columns in turn
    planes, widths, side_of, specs = [], [], [], []
    for s, (cols, offs) in enumerate(sides):
        n = int(offs[world])
        for c in cols:
            planes.append(_row_bytes(c, n))
            widths.append(_row_width(c))
            side_of.append(s)
            specs.append((c.dtype, tuple(c.shape[1:])))
    NP = len(planes)
    send_counts = [[int(offs[p + 1] - offs[p]) for _, offs in sides] for p in range(world)]
    if dev.type == "cpu":
        cnt = torch.tensor(send_counts, dtype=torch.int64).reshape(-1)
        rcnt = torch.empty_like(cnt)
        dist.all_to_all_single(rcnt, cnt, group=group)
        recv_counts = rcnt.reshape(world, S).tolist()
    else:
        import tiflash_amd as tfa
        ctx = ctx or _default_ctx(dev)
        cur = torch.cuda.current_stream(dev)
        if ctx.stream.cuda_stream != cur.cuda_stream:  # the slices move on ctx's stream
            ctx.stream.wait_stream(cur)
        comm = _tfg_comm(ctx, group)
        sc = (ctypes.c_uint64 * (world * S))(*[send_counts[p][s] for p in range(world) for s in range(S)])
        rc = (ctypes.c_uint64 * (world * S))()
        tfa.check(tfa.lib().tfg_alltoall_counts_n(comm, ctypes.c_int(S), sc, rc))
        recv_counts = [[int(rc[p * S + s]) for s in range(S)] for p in range(world)]
    total_rows = [sum(recv_counts[p][side_of[k]] for p in range(world)) for k in range(NP)]
    outs = [_empty_col(total_rows[k], specs[k][0], specs[k][1], dev) for k in range(NP)]
    if dev.type == "cpu":
        send_bytes = [sum(send_counts[p][side_of[k]] * widths[k] for k in range(NP)) for p in range(world)]
        recv_bytes = [sum(recv_counts[p][side_of[k]] * widths[k] for k in range(NP)) for p in range(world)]
        send = torch.cat([planes[k][int(sides[side_of[k]][1][p]):int(sides[side_of[k]][1][p + 1])].reshape(-1)
                          for p in range(world) for k in range(NP)] + [torch.empty(0, dtype=torch.uint8)])
        recv = torch.empty(sum(recv_bytes), dtype=torch.uint8)
        dist.all_to_all_single(recv, send, recv_bytes, send_bytes, group=group)
        pos, r0 = 0, [0] * NP
        for p in range(world):
            for k in range(NP):
                r = recv_counts[p][side_of[k]]
                if r:
                    dst = outs[k].reshape(-1).view(torch.uint8)
                    dst[r0[k] * widths[k]:(r0[k] + r) * widths[k]] = recv[pos:pos + r * widths[k]]
                pos += r * widths[k]
                r0[k] += r
    else:  # zero copy: every slice from its partitioned column straight into its output column
        sends = (_Slice * max(1, world * NP))()
        recvs = (_Slice * max(1, world * NP))()
        r0 = [0] * NP
        for p in range(world):
            for k in range(NP):
                o0 = int(sides[side_of[k]][1][p])
                r = send_counts[p][side_of[k]]
                sends[p * NP + k] = _Slice(p, planes[k].data_ptr() + o0 * widths[k] if r else 0, r * widths[k])
                rr = recv_counts[p][side_of[k]]
                recvs[p * NP + k] = _Slice(p, outs[k].data_ptr() + r0[k] * widths[k] if rr else 0, rr * widths[k])
                r0[k] += rr
        tfa.check(tfa.lib().tfg_exchange_slices(comm, ctypes.c_int(world * NP), sends, ctypes.c_int(world * NP), recvs))
        if ctx.stream.cuda_stream != cur.cuda_stream:  # the caller's stream sees the received columns,
            cur.wait_stream(ctx.stream)               # and the allocator keeps both sides alive until then
            for t in planes + outs:
                t.record_stream(ctx.stream)
    res, k = [], 0
    for cols, _ in sides:
        res.append(outs[k:k + len(cols)])
        k += len(cols)
    return res


def exchange_partitions(cols: Sequence[torch.Tensor], offsets: Sequence[int], group=None, ctx=None) -> List[torch.Tensor]:
    """One side: sends rows [offsets[p], offsets[p+1]) of every column to rank p in one fused
    exchange; returns the received columns."""
    return exchange_sides([(cols, offsets)], group, ctx)[0]


def exchange_string_rows(ctx, perm, offs, row_cols, strings, group=None):
    """Rows with String columns: the fixed-width row columns plus each String's row lengths
    travel as one side, every String's chars as a side of 1-byte rows cut at the partitions'
    byte boundaries — all in the same single data all-to-all.  perm / offs: the stable partition
    (tfa.partition).  strings: [(chars, end offsets)].  Returns (row columns, [(chars, end
    offsets)]) of the received rows."""
    import tiflash_amd as tfa
    world = len(offs) - 1
    rows = tfa.gather(ctx, perm, list(row_cols)) if row_cols else []
    lens, chars_sides = [], []
    for chars, ends in strings:
        gc, ge = tfa.gather_string(ctx, perm, chars, ends)
        starts = torch.cat([ge.new_zeros(1), ge[:-1]]) if ge.numel() else ge
        lens.append(ge - starts)
        # byte offset of each partition boundary (one small host read)
        idx = torch.tensor([int(o) - 1 for o in offs[1:]], dtype=torch.int64, device=ge.device)
        ends_at = torch.where(idx >= 0, ge[idx.clamp(min=0)] if ge.numel() else idx * 0, idx * 0)
        boff = [0] + [int(x) for x in ends_at.tolist()]
        chars_sides.append(([gc], boff))
    got = exchange_sides([(rows + lens, offs)] + chars_sides, group, ctx)
    rcols = got[0][:len(rows)]
    rlens = got[0][len(rows):]
    out_strings = []
    for ln, side in zip(rlens, got[1:]):
        out_strings.append((side[0], torch.cumsum(ln, 0)))
    return rcols, out_strings


def two_phase_merge_keys(ctx, partial, final, group=None, collators=None):
    """ExchangeSender -> ExchangeReceiver of a two-phase GROUP BY over String / several keys
    (C5): the partial aggregation's rows are routed by the reference's hash of the key columns
    (IColumn::updateWeakHash32 -> fillSelector, HashBaseWriterHelper.cpp:46-84) and the final
    aggregation merges them (mergeOnBlock).  Keys travel packed (16 bytes) while the partial
    aggregator holds them packed: its result is written ONCE, packed, and the weak hash of the key
    columns is computed from the packed keys (tfg_agg_weak_hash_packed) — no unpacked copy of the
    partial groups.  Once it has moved to the serialized method (a String sort key over 15 bytes,
    String + fixed keys, wide tuples), or a state is a String (min / max / first_row of a String),
    the groups travel as their key columns — Strings as chars + lengths — with the states, still in
    one data all-to-all.  `partial` and `final` are tiflash_amd.KeysAggregator objects of the same
    signature."""
    import tiflash_amd as tfa
    world = dist.get_world_size(group)
    str_states = any((t & 0xFF) == tfa.STRING and k in (tfa.AGG_MIN, tfa.AGG_MAX, tfa.AGG_FIRST_ROW)
                     for k, t in partial.aggs)  # the type word's low byte (collator / precision above)
    if partial.holds_packed() and not str_states:
        packed = partial.result_packed()
        keys16 = packed["keys"]
        n = keys16.shape[0]
        h = torch.empty(n, dtype=torch.int32, device=keys16.device)
        tfa.check(tfa.lib().tfg_weak_hash_init(ctx.h, tfa._p(h), tfa.ctypes.c_int64(n)))
        partial.weak_hash_packed(keys16, h)
        sel = tfa.fill_selector(ctx, h, world)
        perm, offs = tfa.partition(ctx, sel, world)
        ns = len(packed["states"])
        send = tfa.gather(ctx, perm, [keys16] + list(packed["states"]) + list(packed["state_null"]))
        recv = exchange_partitions(send, offs, group, ctx)
        final.consume_partial_packed(recv[0], recv[1:1 + ns], state_nullmaps=recv[1 + ns:])
        return
    cols = partial.result()
    n = partial.size()
    dev = cols["key_null"][0].device
    h = torch.empty(n, dtype=torch.int32, device=dev)
    tfa.check(tfa.lib().tfg_weak_hash_init(ctx.h, tfa._p(h), tfa.ctypes.c_int64(n)))
    for j, (t, k, kn) in enumerate(zip(partial.key_types, cols["keys"], cols["key_null"])):
        if t == tfa.STRING:
            tfa.weak_hash_string(ctx, k[0], k[1], h, nullmap=kn, collator=(collators or [0] * 4)[j])
        else:
            tfa.weak_hash(ctx, [k], types=[t], nullmaps=[kn], h=h)
    sel = tfa.fill_selector(ctx, h, world)
    perm, offs = tfa.partition(ctx, sel, world)
    fixed = [k for t, k in zip(partial.key_types, cols["keys"]) if t != tfa.STRING]
    strings = [k for t, k in zip(partial.key_types, cols["keys"]) if t == tfa.STRING]
    # String states (min / max / first_row of a String) travel like String keys: offsets + chars
    is_str = [isinstance(st, (tuple, list)) for st in cols["states"]]
    fstates = [st for st, x in zip(cols["states"], is_str) if not x]
    strings += [st for st, x in zip(cols["states"], is_str) if x]
    row_cols = fixed + list(cols["key_null"]) + fstates + list(cols["state_null"])
    rcols, rstr = exchange_string_rows(ctx, perm, offs, row_cols, strings, group)
    nk, nkeys, ns, nsk = len(fixed), len(partial.key_types), len(fstates), len(strings) - sum(is_str)
    rfixed, rknull = rcols[:nk], rcols[nk:nk + nkeys]
    rfstates, rsnull = rcols[nk + nkeys:nk + nkeys + ns], rcols[nk + nkeys + ns:]
    keys, fi, si = [], 0, 0
    for t in partial.key_types:
        if t == tfa.STRING:
            keys.append(rstr[si])
            si += 1
        else:
            keys.append(rfixed[fi])
            fi += 1
    rstates, fi, si = [], 0, nsk
    for x in is_str:
        if x:
            rstates.append(rstr[si])
            si += 1
        else:
            rstates.append(rfstates[fi])
            fi += 1
    final.consume_partial(keys, rstates, key_nullmaps=rknull, state_nullmaps=rsnull)
