"""World-2 GPU test of the N>1 path (SURVEY §8(e), configs[3] / configs[4]): two ranks, each
running the HIP kernels through the C-ABI on cuda:0 and exchanging over gloo (the RCCL path
needs one GPU per rank; the 8-GPU run is the driver's).  tests/multirank_worker.py is one rank.

Checked against the CPU oracle over the union of both ranks' inputs:
  * routing — every row a rank receives hashes to that rank under the reference's weak hash +
    fillSelector (HashBaseWriterHelper.cpp:46-62), and the sender's partitions equal the
    oracle's stable partition (IColumn::scatter order);
  * C4 — the joined rows (probe key, probe payload, build payload) of all ranks = the oracle
    join of the union (JoinRef, Join.cpp semantics), as multisets;
  * C5 — the final groups of all ranks (String key incl. NULL, exact Decimal sum, count) = the
    oracle's GROUP BY of the union, and no key is finalised on two ranks;
  * C5L / C5M — the same with String keys past 15 bytes (serialized keys through the exchange)
    and with a (String, Int64) key pair;
  * C2 — two-phase Int64-key GROUP BY with the fused filter = the oracle's.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import multirank_worker as W  # noqa: E402

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def ranks(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("multirank"))
    port = _free_port()
    procs = []
    for r in range(WORLD):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "multirank_worker.py"), out],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=100)
            logs.append(o)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-4000:]}"
    return [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(WORLD)]


def _selector(orc, keys):
    return orc.fill_selector(orc.weak_hash([keys]), WORLD)


@pytest.mark.gpu
def test_routing_matches_reference_selector(ranks, orc):
    for r, d in enumerate(ranks):
        bk = W.join_data(r, WORLD)[0]
        sel = _selector(orc, bk)
        perm, offs = orc.partition(sel, WORLD)
        assert list(d["send_build_offs"]) == [int(x) for x in offs]
        assert np.array_equal(d["send_build_keys"], bk[perm]), "sender partition order != stable scatter"
        for name in ("recv_build_keys", "recv_probe_keys"):
            keys = d[name]
            assert (_selector(orc, keys) == r).all(), f"rank {r} received rows of another partition ({name})"
    all_b = np.concatenate([W.join_data(r, WORLD)[0] for r in range(WORLD)])
    got_b = np.concatenate([d["recv_build_keys"] for d in ranks])
    assert np.array_equal(np.sort(all_b), np.sort(got_b))


@pytest.mark.gpu
def test_repartitioned_join_matches_oracle(ranks, orc):
    parts = [W.join_data(r, WORLD) for r in range(WORLD)]
    bk = np.concatenate([p[0] for p in parts])
    bpay = np.concatenate([p[1] for p in parts])
    pk = np.concatenate([p[2] for p in parts])
    ppay = np.concatenate([p[3] for p in parts])
    jr = orc.JoinRef(orc.INT64)
    jr.build(bk)
    pi, bi = jr.probe(pk)
    exp = np.stack([pk[pi], ppay[pi], bpay[bi]], axis=1)
    got = np.concatenate([d["join_rows"] for d in ranks])
    assert got.shape == exp.shape
    order = lambda a: a[np.lexsort(a.T[::-1])]  # noqa: E731
    assert np.array_equal(order(got), order(exp))


@pytest.mark.gpu
def test_two_phase_string_decimal_groupby_matches_oracle(ranks, orc):
    ref = orc.AggKeys([orc.STRING], [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    for r in range(WORLD):
        chars, offs, nulls, v = W.agg_data(r)
        ref.consume([(chars, offs)], [v, None], key_nulls=[nulls])
    exp = {}
    for key, vals in ref.result():
        exp[key[0]] = (vals[0], vals[1])
    got = {}
    for d in ranks:
        chars, offs, knull = d["c5_chars"], d["c5_offs"], d["c5_key_null"]
        s = 0
        for i in range(len(offs)):
            e = int(offs[i])
            key = None if knull[i] else bytes(chars[s:e - 1])
            s = e
            lo, hi = int(d["c5_sum"][i][0]) & ((1 << 64) - 1), int(d["c5_sum"][i][1])
            val = lo | (hi << 64)
            assert key not in got, f"group {key!r} finalised on two ranks"
            got[key] = (val, int(d["c5_cnt"][i]))
    assert got == exp


@pytest.mark.gpu
def test_two_phase_filter_groupby_matches_oracle(ranks, orc):
    ref = orc.Agg(orc.INT64, [(0, orc.FLOAT64), (2, 0)])
    for r in range(WORLD):
        f, k, v = W.c2_data(r)
        ref.consume(k, [v, None], mask=(f < 96).astype(np.uint8))
    rr = ref.result()
    exp = sorted(zip(rr["keys"].view(np.int64).tolist(), rr["states"][0].tolist(), rr["states"][1].tolist()))
    got = []
    for d in ranks:
        got += list(zip(d["c2_keys"].tolist(), d["c2_sum"].tolist(), d["c2_cnt"].tolist()))
    assert len(set(k for k, _, _ in got)) == len(got), "a key was finalised on two ranks"
    assert sorted(got) == exp


@pytest.mark.gpu
@pytest.mark.parametrize("tag", ["c5l", "c5m"])
def test_two_phase_long_string_keys_match_oracle(ranks, orc, tag):
    types = [orc.STRING] + ([orc.INT64] if tag == "c5m" else [])
    ref = orc.AggKeys(types, [(0, orc.prec(orc.DECIMAL64, 15)), (2, 0)])
    for r in range(WORLD):
        chars, offs, nulls, k2, v = W.long_agg_data(r)
        keys = [(chars, offs)] + ([k2] if tag == "c5m" else [])
        ref.consume(keys, [v, None], key_nulls=[nulls] + ([None] if tag == "c5m" else []))
    exp = {}
    for key, vals in ref.result():
        exp[tuple(key)] = (vals[0], vals[1])
    got = {}
    long_keys = 0
    for d in ranks:
        chars, offs, knull = d[tag + "_chars"], d[tag + "_offs"], d[tag + "_key_null"]
        s = 0
        for i in range(len(offs)):
            e = int(offs[i])
            key = None if knull[i] else bytes(chars[s:e - 1])
            long_keys += key is not None and len(key) > 15
            s = e
            lo, hi = int(d[tag + "_sum"][i][0]) & ((1 << 64) - 1), int(d[tag + "_sum"][i][1])
            k = (key,) + ((int(d[tag + "_k2"][i]),) if tag == "c5m" else ())
            assert k not in got, f"group {k!r} finalised on two ranks"
            got[k] = (lo | (hi << 64), int(d[tag + "_cnt"][i]))
    assert long_keys > 0
    assert got == exp
