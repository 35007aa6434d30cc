"""One rank of the world-2 GPU test (tests/test_gpu_multirank.py): the N>1 path of bench.py with
the HIP kernels on every rank — ranks share cuda:0 and exchange over gloo (the RCCL path needs
one GPU per rank; gloo stages the same partition-major buffers through the host).

Per rank, on the device through the C-ABI:
  C4  tfg_hash_partition of the build and probe sides (weak hash -> fillSelector -> stable
      scatter, HashPartitionWriter.cpp:139-204) -> all-to-all -> tfg_join build_rows / finalize ->
      materialising INNER probe;
  C5  KeysAggregator over a nullable String key with sum(Decimal(15,2)) + count(*) -> weak hash
      of the partial rows' keys -> all-to-all of packed keys + states -> final KeysAggregator
      (two-phase, gtest_compute_server.cpp:738-812);
  C5L the same with String keys past 15 bytes (the serialized method: keys travel as chars +
      lengths in the fused exchange), and C5M with a (String, Int64) key pair;
  C2  Aggregator Int64 key, fused f < 96 filter, sum(Float64) + count -> hash_partition of the
      partial rows -> all-to-all -> consume_partial (bench.py's N>1 step).
The join's build and probe sides travel in ONE fused exchange (exchange_sides).
Results (and the rows each rank received) are written to <out>/rank<r>.npz; the test compares
them with the oracle over the union of both ranks' inputs.

Run as: RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/multirank_worker.py <out>
Not collected by pytest (no test_ prefix); imported by the test for the data generators only.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def join_data(rank, world=2, nb=40_000, npr=150_000):
    """C3 distributions over the global key space; ~5% of build keys repeat (RowRefList chains)."""
    rng = np.random.default_rng(70 + rank)
    bk = (rng.permutation(nb).astype(np.int64) + rank * nb) * 4 + 1
    dup = rng.random(nb) < 0.05
    bk[dup] = (rng.integers(0, nb * world, int(dup.sum())) * 4 + 1).astype(np.int64)
    bpay = rng.integers(0, 1 << 40, nb, dtype=np.int64)
    hit = rng.random(npr) < 0.5
    pk = np.where(hit, rng.integers(0, nb * world, npr) * 4 + 1, rng.integers(0, 1 << 40, npr) * 4 + 3).astype(np.int64)
    ppay = rng.integers(0, 1 << 40, npr, dtype=np.int64)
    return bk, bpay, pk, ppay


def string_column(strs):
    """ColumnString layout: chars with a '\\0' after every row + UInt64 end offsets."""
    bs = [s.encode() + b"\0" for s in strs]
    chars = np.frombuffer(b"".join(bs), dtype=np.uint8).copy()
    offs = np.cumsum([len(b) for b in bs]).astype(np.uint64)
    return chars, offs


def agg_data(rank, n=60_000, groups=5_000):
    """C5 shape: String keys (k%08d and shorter variable-length forms), 2% NULL keys,
    Decimal(15,2) values as Int64 in [-1e9, 1e9)."""
    rng = np.random.default_rng(110 + rank)
    ids = rng.integers(0, groups, n)
    strs = [("k%08d" % i) if i % 3 else ("x%d" % i) for i in ids]
    chars, offs = string_column(strs)
    nulls = (rng.random(n) < 0.02).astype(np.uint8)
    v = rng.integers(-10**9, 10**9, n, dtype=np.int64)
    return chars, offs, nulls, v


def long_agg_data(rank, n=40_000, groups=3_000):
    """String keys of 1-40 bytes, most past the 15 bytes of the packed key, 2% NULL; an Int64
    second key column (C5M) with 7 values."""
    rng = np.random.default_rng(130 + rank)
    ids = rng.integers(0, groups, n)
    strs = [("customer#%012d/%s" % (i, "x" * (i % 17))) if i % 4 else ("s%d" % i) for i in ids]
    chars, offs = string_column(strs)
    nulls = (rng.random(n) < 0.02).astype(np.uint8)
    k2 = (ids % 7 - 3).astype(np.int64)
    v = rng.integers(-10**9, 10**9, n, dtype=np.int64)
    return chars, offs, nulls, k2, v


def c2_data(rank, n=300_000, groups=20_000):
    rng = np.random.default_rng(1 + rank)
    f = rng.integers(0, 100, n, dtype=np.int64)
    k = rng.integers(0, groups, n, dtype=np.int64)
    v = rng.integers(0, 1 << 20, n).astype(np.float64) / 256.0  # dyadic: exact in any order
    return f, k, v


def main():
    out_dir = sys.argv[1]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import tiflash_amd as tfa
    from tiflash_amd.exchange import exchange_partitions, exchange_sides, two_phase_merge_keys

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)

    def T(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    res = {}
    with tfa.Context(0) as ctx:
        # ---- C4: repartitioned join
        bk, bpay, pk, ppay = join_data(rank, world)
        bcols, boffs = tfa.hash_partition(ctx, [T(bk), T(bpay)], [0], world)
        res["send_build_keys"] = bcols[0].cpu().numpy()
        res["send_build_offs"] = np.array(boffs, dtype=np.int64)
        pcols, poffs = tfa.hash_partition(ctx, [T(pk), T(ppay)], [0], world)
        lb, lp = exchange_sides([(bcols, boffs), (pcols, poffs)])
        res["recv_build_keys"] = lb[0].cpu().numpy()
        res["recv_probe_keys"] = lp[0].cpu().numpy()
        j = tfa.Join(ctx, tfa.INT64, expected_build_rows=int(lb[0].shape[0]))
        j.build(lb[0], payload=[lb[1]])
        j.finalize()
        op, ob, _ = j.probe_rows(lp[0], [lp[0], lp[1]], 1)
        res["join_rows"] = np.stack([op[0].cpu().numpy(), op[1].cpu().numpy(), ob[0].cpu().numpy()], axis=1)
        j.close()

        # ---- C5: two-phase GROUP BY String key, sum(Decimal(15,2)) + count(*)
        chars, offs, nulls, v = agg_data(rank)
        aggs = [(tfa.AGG_SUM, tfa.prec(tfa.DECIMAL64, 15)), (tfa.AGG_COUNT_ALL, 0)]
        part = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=10_000)
        fin = tfa.KeysAggregator(ctx, [tfa.STRING], aggs, expected_groups=10_000)
        part.consume([(T(chars), T(offs.astype(np.int64)))], [T(v), None], key_nullmaps=[T(nulls)])
        two_phase_merge_keys(ctx, part, fin)
        r = fin.result()
        (kc, ko), = r["keys"]
        res["c5_chars"] = kc.cpu().numpy()
        res["c5_offs"] = ko.cpu().numpy()
        res["c5_key_null"] = r["key_null"][0].cpu().numpy()
        res["c5_sum"] = r["states"][0].cpu().numpy()
        res["c5_cnt"] = r["states"][1].cpu().numpy()
        part.close()
        fin.close()

        # ---- C5L / C5M: String keys past 15 bytes (serialized), and String + Int64 keys
        chars, offs, nulls, k2, v = long_agg_data(rank)
        for tag, types in (("c5l", [tfa.STRING]), ("c5m", [tfa.STRING, tfa.INT64])):
            part = tfa.KeysAggregator(ctx, types, aggs, expected_groups=10_000)
            fin = tfa.KeysAggregator(ctx, types, aggs, expected_groups=10_000)
            keys = [(T(chars), T(offs.astype(np.int64)))] + ([T(k2)] if len(types) > 1 else [])
            knull = [T(nulls)] + ([T(np.zeros(len(k2), np.uint8))] if len(types) > 1 else [])
            part.consume(keys, [T(v), None], key_nullmaps=knull)
            two_phase_merge_keys(ctx, part, fin)
            r = fin.result()
            (kc, ko) = r["keys"][0]
            res[tag + "_chars"] = kc.cpu().numpy()
            res[tag + "_offs"] = ko.cpu().numpy()
            res[tag + "_key_null"] = r["key_null"][0].cpu().numpy()
            if len(types) > 1:
                res[tag + "_k2"] = r["keys"][1].cpu().numpy()
            res[tag + "_sum"] = r["states"][0].cpu().numpy()
            res[tag + "_cnt"] = r["states"][1].cpu().numpy()
            part.close()
            fin.close()

        # ---- C2: two-phase filter -> GROUP BY Int64 key
        f, k, vv = c2_data(rank)
        a2 = [(tfa.AGG_SUM, tfa.FLOAT64), (tfa.AGG_COUNT_ALL, 0)]
        agg = tfa.Aggregator(ctx, tfa.INT64, a2, expected_groups=40_000)
        final = tfa.Aggregator(ctx, tfa.INT64, a2, expected_groups=40_000)
        agg.consume_filtered(T(f), tfa.LT, 96, T(k), [T(vv), None])
        pr = agg.result()
        cols, coffs = tfa.hash_partition(ctx, [pr["keys"], pr["states"][0], pr["states"][1]], [0], world)
        outs = exchange_partitions(cols, coffs)
        final.consume_partial(outs[0], [outs[1], outs[2]])
        fr = final.result()
        res["c2_keys"] = fr["keys"].cpu().numpy()
        res["c2_sum"] = fr["states"][0].cpu().numpy()
        res["c2_cnt"] = fr["states"][1].cpu().numpy()
        agg.close()
        final.close()
        ctx.sync()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
