"""Multi-process (world_size 2, gloo, CPU) tests of the N>1 path: hash repartition -> all-to-all
exchange -> local operator, as bench.py --gpus N runs it over RCCL.

The per-rank device kernels (tfg_hash_partition, the aggregator, the join) are replaced here by
the CPU restatement so the distributed logic runs without a GPU: weak hash + fillSelector routing
(HashBaseWriterHelper.cpp:46-84), the exchange itself (tiflash_amd.exchange), and the merge of
partial aggregation states (two-phase agg) / the local join after repartitioning
(C4).  Results are compared with a single-process run over the union of all ranks' data."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _partition(orc, key, parts):
    """tfg_hash_partition on the CPU: weak hash of the key column -> selector -> stable perm."""
    h = orc.weak_hash([key])
    sel = orc.fill_selector(h, parts)
    perm, offsets = orc.partition(sel, parts)
    return perm, [int(x) for x in offsets], sel


def _agg_data(rank, n=20000, groups=3000):
    rng = np.random.default_rng(100 + rank)
    k = rng.integers(-groups // 2, groups // 2, n, dtype=np.int64)
    v = rng.integers(-10**6, 10**6, n, dtype=np.int64)
    return k, v


def _two_phase_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    from tiflash_amd.exchange import exchange_partitions
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        k, v = _agg_data(rank)
        # phase 1: partial aggregation of this rank's rows
        part = orc.Agg(orc.INT64, [(0, orc.INT64), (2, 0)])
        part.consume(k, [v, None])
        r = part.result()
        pk = r["keys"].view(np.int64)
        ps, pc = r["states"][0], r["states"][1].view(np.int64)
        # ExchangeSender: route partial rows by the reference's hash of the key
        perm, offs, _ = _partition(orc, pk, world)
        cols = [torch.from_numpy(np.ascontiguousarray(x[perm])) for x in (pk, ps, pc)]
        rk, rs, rc = exchange_partitions(cols, offs)
        rk, rs, rc = rk.numpy(), rs.numpy(), rc.numpy()
        # every received key belongs to this rank under fillSelector
        _, _, sel = _partition(orc, rk, world) if len(rk) else (None, None, np.array([], dtype=np.uint32))
        assert (sel == rank).all()
        # phase 2: final aggregation = sum of partial sums and counts per key
        fin = orc.Agg(orc.INT64, [(0, orc.INT64), (0, orc.INT64)])
        fin.consume(rk, [rs, rc])
        fr = fin.result()
        res = {int(a): (int(b), int(c)) for a, b, c in zip(fr["keys"].view(np.int64), fr["states"][0], fr["states"][1])}
        allres = [None] * world
        dist.all_gather_object(allres, res)
        if rank == 0:
            merged = {}
            for d in allres:
                assert not (set(d) & set(merged)), "a key was finalised on two ranks"
                merged.update(d)
            q.put(merged)
        dist.destroy_process_group()
    except Exception as e:  # surface the failure to the parent
        q.put(repr(e))
        raise


def test_two_phase_aggregation_gloo():
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_phase_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert isinstance(got, dict), got
    # single-process reference over the union of both ranks' rows
    ks, vs = zip(*[_agg_data(r) for r in range(WORLD)])
    ref = orc.Agg(orc.INT64, [(0, orc.INT64), (2, 0)])
    ref.consume(np.concatenate(ks), [np.concatenate(vs), None])
    rr = ref.result()
    want = {int(a): (int(b), int(c)) for a, b, c in zip(rr["keys"].view(np.int64), rr["states"][0],
                                                         rr["states"][1].view(np.int64))}
    assert got == want


def _join_data(rank, nb=4000, npr=16000):
    rng = np.random.default_rng(200 + rank)
    bk = (rng.permutation(nb).astype(np.int64) * 2 + rank) * 4 + 1        # unique over ranks
    bpay = rng.integers(0, 1 << 40, nb, dtype=np.int64)
    all_b = np.concatenate([(np.arange(nb, dtype=np.int64) * 2 + r) * 4 + 1 for r in range(WORLD)])
    hit = rng.random(npr) < 0.5
    pk = np.where(hit, all_b[rng.integers(0, len(all_b), npr)], rng.integers(0, 1 << 30, npr) * 4 + 3)
    ppay = rng.integers(0, 1 << 40, npr, dtype=np.int64)
    return bk, bpay, pk.astype(np.int64), ppay


def _join_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    from tiflash_amd.exchange import exchange_partitions
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        bk, bpay, pk, ppay = _join_data(rank)
        # repartition both sides by the key (C4: ExchangeSender of build and probe)
        perm, offs, _ = _partition(orc, bk, world)
        rbk, rbp = [x.numpy() for x in exchange_partitions([torch.from_numpy(bk[perm]), torch.from_numpy(bpay[perm])], offs)]
        perm, offs, _ = _partition(orc, pk, world)
        rpk, rpp = [x.numpy() for x in exchange_partitions([torch.from_numpy(pk[perm]), torch.from_numpy(ppay[perm])], offs)]
        j = orc.JoinRef(orc.INT64)
        j.build(rbk)
        pi, bi = j.probe(rpk, kind=0)
        rows = sorted(zip(rpk[pi].tolist(), rpp[pi].tolist(), rbp[bi].tolist()))
        allrows = [None] * world
        dist.all_gather_object(allrows, rows)
        if rank == 0:
            q.put(sorted(sum(allrows, [])))
        dist.destroy_process_group()
    except Exception as e:
        q.put(repr(e))
        raise


def test_repartitioned_join_gloo():
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_join_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert isinstance(got, list), got
    data = [_join_data(r) for r in range(WORLD)]
    bk = np.concatenate([d[0] for d in data])
    bpay = np.concatenate([d[1] for d in data])
    pk = np.concatenate([d[2] for d in data])
    ppay = np.concatenate([d[3] for d in data])
    j = orc.JoinRef(orc.INT64)
    j.build(bk)
    pi, bi = j.probe(pk, kind=0)
    want = sorted(zip(pk[pi].tolist(), ppay[pi].tolist(), bpay[bi].tolist()))
    assert len(want) > 1000
    assert got == want


# ---- C5: two-phase GROUP BY a String key, partial rows exchanged as packed 16-byte keys ----------
def _str_data(rank, n=20000, groups=5000):
    rng = np.random.default_rng(300 + rank)
    ids = rng.integers(0, groups, n)
    strs = [b"k%08d" % i for i in ids]
    d = rng.integers(0, 10**9, n, dtype=np.int64)
    return strs, d


def _str_col(strs):
    chars = np.frombuffer(b"".join(s + b"\0" for s in strs), dtype=np.uint8).copy()
    return chars, np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64)


def _pack(strs):
    """The packed key form partial rows travel in (tfg_agg_create_keys, key_string): bytes, zero
    padded, byte 15 = length."""
    out = np.zeros((len(strs), 16), dtype=np.uint8)
    for i, s in enumerate(strs):
        out[i, :len(s)] = np.frombuffer(s, np.uint8)
        out[i, 15] = len(s)
    return out


def _unpack(a):
    return [bytes(r[:r[15]]) for r in a]


def _two_phase_string_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as orc
    from tiflash_amd.exchange import exchange_partitions
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        strs, d = _str_data(rank)
        part = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
        part.consume([_str_col(strs)], [d, None])
        groups = part.result()
        keys = [k[0] for k, _ in groups]
        sums = np.array([[s & (2**64 - 1), s >> 64] for (_, (s, _c)) in groups], dtype=np.uint64).view(np.int64)
        cnts = np.array([c for (_, (_s, c)) in groups], dtype=np.int64)
        # ExchangeSender: route by ColumnString::updateWeakHash32 of the key -> fillSelector
        chars, offs = _str_col(keys)
        h = orc.weak_hash_string(chars, offs, np.full(len(keys), 0xFFFFFFFF, dtype=np.uint32))
        sel = orc.fill_selector(h, world)
        perm, poffs = orc.partition(sel, world)
        packed = _pack(keys)[perm].view(np.int64)
        rk, rs, rc = [x.numpy() for x in exchange_partitions(
            [torch.from_numpy(np.ascontiguousarray(packed)), torch.from_numpy(np.ascontiguousarray(sums[perm])),
             torch.from_numpy(np.ascontiguousarray(cnts[perm]))], [int(x) for x in poffs])]
        rstr = _unpack(rk.view(np.uint8).reshape(-1, 16))
        if rstr:
            c2, o2 = _str_col(rstr)
            h2 = orc.weak_hash_string(c2, o2, np.full(len(rstr), 0xFFFFFFFF, dtype=np.uint32))
            assert (orc.fill_selector(h2, world) == rank).all()
        # final: merge partial states (sum of Decimal128 partial sums, sum of counts)
        fin = orc.AggKeys([orc.STRING], [(0, orc.DECIMAL128), (0, orc.INT64)])
        if rstr:
            fin.consume([_str_col(rstr)], [np.ascontiguousarray(rs), np.ascontiguousarray(rc)])
        res = {k[0]: (s, c) for k, (s, c) in fin.result()}
        allres = [None] * world
        dist.all_gather_object(allres, res)
        if rank == 0:
            merged = {}
            for r in allres:
                assert not (set(r) & set(merged)), "a key was finalised on two ranks"
                merged.update(r)
            q.put(merged)
        dist.destroy_process_group()
    except Exception as e:
        q.put(repr(e))
        raise


def test_two_phase_string_aggregation_gloo():
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_two_phase_string_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert isinstance(got, dict), got
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    for r in range(WORLD):
        strs, d = _str_data(r)
        ref.consume([_str_col(strs)], [d, None])
    want = {k[0]: (s, c) for k, (s, c) in ref.result()}
    assert len(want) > 1000
    assert got == want


def _sides_worker(rank, world, port, q, empty=False):
    """exchange_sides: three sides in one data all-to-all — (Int64, UInt8, 2-word) rows, Float64
    rows, and a byte side (String chars) cut at per-partition byte offsets.  empty: rank 1 has no
    rows on the first side and no chars on the third (a partial GROUP BY with no groups, an empty
    join side), which must not change the record layout its peers expect."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, ROOT)
    from tiflash_amd.exchange import exchange_sides
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        rng = np.random.default_rng(500 + rank)
        sides, sent = [], []
        for s, (n, mk) in enumerate(((3000, "a"), (1700, "b"), (9000, "c"))):
            if empty and rank == 1 and mk in ("a", "c"):
                n = 0
            dest = np.sort(rng.integers(0, world, n))  # partition-major rows
            if rank == 0 and s == 1:
                dest[:] = 0  # a side that sends nothing to the other ranks
            offs = [0] + [int(np.searchsorted(dest, p, side="right")) for p in range(world)]
            if mk == "a":
                cols = [rng.integers(-2**62, 2**62, n, dtype=np.int64), rng.integers(0, 255, n).astype(np.uint8),
                        rng.integers(-2**62, 2**62, (n, 2), dtype=np.int64)]
            elif mk == "b":
                cols = [rng.random(n)]
            else:
                cols = [rng.integers(0, 255, n).astype(np.uint8)]
            sides.append(([torch.from_numpy(c) for c in cols], offs))
            sent.append((cols, offs))
        got = exchange_sides(sides)
        # what each rank should receive: its slice of every side from every rank, rank order
        allsent = [None] * world
        dist.all_gather_object(allsent, sent)
        for s in range(3):
            for j in range(len(sent[s][0])):
                exp = np.concatenate([allsent[r][s][0][j][allsent[r][s][1][rank]:allsent[r][s][1][rank + 1]]
                                      for r in range(world)])
                g = got[s][j].numpy()
                assert g.dtype == exp.dtype and g.shape == exp.shape, (s, j, g.shape, exp.shape)
                assert np.array_equal(g, exp), (s, j)
        q.put("ok")
        dist.destroy_process_group()
    except Exception as e:
        q.put(repr(e))
        raise


@pytest.mark.parametrize("world,empty", [(2, False), (3, False), (2, True), (3, True)])
def test_fused_exchange_sides_gloo(world, empty):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sides_worker, args=(r, world, port, q, empty)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert res == ["ok"] * world, res
