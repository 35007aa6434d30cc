"""MPP packet codec (§8 f1): CHBlockChunkCodec / CHBlockChunkCodecV1 with CompressionMethod::NONE
(LZ4 packets: tests/test_codec_lz4.py).

CPU: the oracle (oracle/codec.c) against hand-derived packets — the byte layout written out from
the reference's text (CHBlockChunkCodecV1.cpp:45-58,293-312,370-432; CHBlockChunkCodec.cpp:134-166;
IO/VarInt.h:224-240; DataTypeString.cpp:93-117,339-430; DataTypeNullable.cpp:66-89).  The
reference's own codec gtests are round trips of random blocks (gtest_block_chunk_codec.cpp), so
the format is pinned by these hand-derived vectors, not by reference-produced fixtures.
GPU: the HIP encoder is byte-identical to the oracle; the HIP decoder returns the original
columns for oracle packets (one part and several parts), every type, NULLs, empty strings,
multi-byte varints, long strings (the sequential fallback) and legacy String columns spanning
many parse chunks.
"""
import struct

import numpy as np
import pytest

CHB, V1 = 0, 1


def strings_to_column(strs):
    """ColumnString layout: chars with a '\\0' after every row, UInt64 end offsets."""
    chars = b"".join(s + b"\0" for s in strs)
    offs = np.cumsum([len(s) + 1 for s in strs]).astype(np.uint64) if strs else np.zeros(0, np.uint64)
    return np.frombuffer(chars, np.uint8).copy() if chars else np.zeros(0, np.uint8), offs


def vu(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def sb(s):
    return vu(len(s)) + s


# ------------------------------------------------------------------ CPU: oracle vs hand-derived bytes
def test_golden_v1_int64_string(orc):
    a = np.array([1, 2, 3], np.int64)
    chars, offs = strings_to_column([b"", b"ab", b"xyz"])
    got = orc.codec_encode([("a", "Int64", a, None, None), ("s", "String", chars, offs, None)], 3, version=V1)
    want = (b"\x02" + vu(2) + vu(3) + sb(b"a") + sb(b"Int64") + sb(b"s") + sb(b"String") + vu(3) +
            struct.pack("<3q", 1, 2, 3) + b"\x00" + b"\x02ab" + b"\x03xyz")
    assert got == want


def test_golden_chblock_interleaves_meta_and_data(orc):
    a = np.array([1, 2, 3], np.int64)
    chars, offs = strings_to_column([b"", b"ab", b"xyz"])
    got = orc.codec_encode([("a", "Int64", a, None, None), ("s", "String", chars, offs, None)], 3, version=CHB)
    want = (vu(2) + vu(3) + sb(b"a") + sb(b"Int64") + struct.pack("<3q", 1, 2, 3) + sb(b"s") + sb(b"String") +
            b"\x00\x02ab\x03xyz")
    assert got == want


def test_golden_nullable_decimal_stringv2(orc):
    x = np.array([5, 0, 7], np.int32)
    nm = np.array([0, 1, 0], np.uint8)
    d = np.array([[12345, 0], [-1, -1]], np.int64)  # Decimal(20,2): Int128 limbs
    chars, offs = strings_to_column([b"a", b"bc"])
    got = orc.codec_encode([("x", "Nullable(Int32)", x, None, nm)], 3, version=V1)
    assert got == b"\x02\x01\x03" + sb(b"x") + sb(b"Nullable(Int32)") + b"\x03" + bytes(nm) + x.tobytes()
    got = orc.codec_encode([("d", "Decimal(20,2)", d, None, None), ("s", "StringV2", chars, offs, None)], 2,
                           version=V1)
    want = (b"\x02\x02\x02" + sb(b"d") + sb(b"Decimal(20,2)") + sb(b"s") + sb(b"StringV2") + b"\x02" + d.tobytes() +
            struct.pack("<2Q", 2, 3) + b"a\0bc\0")
    assert got == want


def test_golden_multibyte_varint_and_empty(orc):
    s = bytes(range(200))
    chars, offs = strings_to_column([s])
    got = orc.codec_encode([("s", "String", chars, offs, None)], 1, version=CHB)
    assert got == b"\x01\x01" + sb(b"s") + sb(b"String") + b"\xc8\x01" + s
    # V1 writes nothing for an empty block; CHBlock writes the header
    assert orc.codec_encode([("a", "Int64", np.zeros(0, np.int64), None, None)], 0, version=V1) == b""
    assert orc.codec_encode([("a", "Int64", np.zeros(0, np.int64), None, None)], 0, version=CHB) == \
        b"\x01\x00" + sb(b"a") + sb(b"Int64")


def test_golden_v1_parts(orc):
    a = np.arange(5, dtype=np.int64)
    got = orc.codec_encode([("a", "Int64", a, None, None)], 5, version=V1, part_rows=[2, 0, 3])
    want = b"\x02\x01\x05" + sb(b"a") + sb(b"Int64") + b"\x02" + a[:2].tobytes() + b"\x03" + a[2:].tobytes()
    assert got == want


def test_oracle_string_decode_roundtrip(orc):
    rng = np.random.default_rng(3)
    strs = [bytes(rng.integers(0, 256, rng.integers(0, 300)).astype(np.uint8)) for _ in range(200)]
    chars, offs = strings_to_column(strs)
    pkt = orc.codec_encode([("s", "String", chars, offs, None)], len(strs), version=CHB)
    body = pkt[len(vu(1) + vu(len(strs)) + sb(b"s") + sb(b"String")):]
    c2, o2, used = orc.codec_decode_strings(body, len(strs), chars.size)
    assert used == len(body)
    assert np.array_equal(c2, chars) and np.array_equal(o2, offs)


# ------------------------------------------------------------------ GPU: HIP codec vs oracle
TYPES = [("Int8", np.int8), ("Int16", np.int16), ("Int32", np.int32), ("Int64", np.int64), ("UInt8", np.uint8),
         ("UInt16", np.uint16), ("UInt32", np.uint32), ("UInt64", np.uint64), ("Float32", np.float32),
         ("Float64", np.float64), ("Decimal(9,2)", np.int32), ("Decimal(15,2)", np.int64), ("MyDate", np.uint64),
         ("MyDateTime(6)", np.uint64)]


def make_block(rng, n, max_len=24, long_every=0):
    cols = []
    for tn, dt in TYPES:
        v = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, n, dtype=np.int64, endpoint=True)
        cols.append((f"c_{tn}", tn, v.view(np.uint64).astype(dt) if dt not in (np.float32, np.float64)
                     else rng.standard_normal(n).astype(dt), None, None))
    cols.append(("dec128", "Decimal(30,4)", rng.integers(-2**62, 2**62, (n, 2), dtype=np.int64), None, None))
    nm = (rng.random(n) < 0.3).astype(np.uint8)
    cols.append(("n_i64", "Nullable(Int64)", rng.integers(-100, 100, n, dtype=np.int64), None, nm))
    lens = rng.integers(0, max_len + 1, n)
    if long_every:
        lens[::long_every] = rng.integers(300, 3000, len(lens[::long_every]))
    strs = [bytes(rng.integers(0, 256, L).astype(np.uint8)) for L in lens]
    chars, offs = strings_to_column(strs)
    cols.append(("s", "String", chars, offs, None))
    cols.append(("s2", "StringV2", chars, offs, None))
    nm2 = (rng.random(n) < 0.2).astype(np.uint8)
    cols.append(("ns", "Nullable(String)", chars, offs, nm2))
    return cols


def to_dev(cols, dev):
    import torch
    out = []
    for name, tn, data, offs, nm in cols:
        t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).to(dev)
        out.append((name, tn, t(data), None if offs is None else torch.from_numpy(offs.astype(np.int64)).to(dev),
                    t(nm)))
    return out


def assert_decoded(cols, n, rows, dec):
    assert rows == n and len(dec) == len(cols)
    for (name, tn, data, offs, nm), d in zip(cols, dec):
        assert d["name"] == name and d["type_name"] == tn
        if nm is not None:
            assert np.array_equal(d["nullmap"].cpu().numpy(), nm)
        if offs is not None:
            assert np.array_equal(d["offsets"].cpu().numpy().astype(np.uint64), offs)
            assert d["data"].cpu().numpy().tobytes() == data.tobytes()
        else:
            assert d["data"].cpu().numpy().tobytes() == np.ascontiguousarray(data).tobytes(), name


@pytest.mark.gpu
@pytest.mark.parametrize("version", [CHB, V1])
@pytest.mark.parametrize("n", [0, 1, 7, 1000, 20000])
def test_gpu_encode_matches_oracle(tfa, orc, ctx, dev, version, n):
    rng = np.random.default_rng(100 + n + version)
    cols = make_block(rng, n, long_every=97 if n >= 1000 else 0)
    want = orc.codec_encode(cols, n, version=version)
    pkt = tfa.codec_encode(ctx, to_dev(cols, dev), n, version=version)
    assert pkt.cpu().numpy().tobytes() == want


@pytest.mark.gpu
@pytest.mark.parametrize("version", [CHB, V1])
@pytest.mark.parametrize("n,long_every", [(1, 0), (7, 0), (5000, 0), (5000, 61), (200000, 0)])
def test_gpu_decode_oracle_packets(tfa, orc, ctx, dev, version, n, long_every):
    import torch
    rng = np.random.default_rng(7 + n + long_every)
    cols = make_block(rng, n, long_every=long_every)
    pkt = torch.from_numpy(np.frombuffer(orc.codec_encode(cols, n, version=version), np.uint8).copy()).to(dev)
    rows, dec = tfa.codec_decode(ctx, pkt, version=version)
    assert_decoded(cols, n, rows, dec)


@pytest.mark.gpu
def test_gpu_decode_multipart_v1(tfa, orc, ctx, dev):
    import torch
    rng = np.random.default_rng(11)
    n = 3000
    cols = make_block(rng, n)
    pkt = orc.codec_encode(cols, n, version=V1, part_rows=[1000, 0, 1, 1999])
    rows, dec = tfa.codec_decode(ctx, torch.from_numpy(np.frombuffer(pkt, np.uint8).copy()).to(dev), version=V1)
    assert_decoded(cols, n, rows, dec)


@pytest.mark.gpu
def test_gpu_legacy_strings_many_chunks(tfa, orc, ctx, dev):
    """A String column of ~60 MB: hundreds of 32 KB parse chunks in several resolution groups."""
    import torch
    n = 3_000_000
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 40, n)
    offs = np.cumsum(lens + 1).astype(np.uint64)
    chars = rng.integers(1, 256, int(offs[-1])).astype(np.uint8)
    chars[(offs - 1).astype(np.int64)] = 0
    cols = [("k", "Int64", np.arange(n, dtype=np.int64), None, None), ("s", "String", chars, offs, None)]
    pkt_host = orc.codec_encode(cols, n, version=V1)
    pkt = tfa.codec_encode(ctx, to_dev(cols, dev), n, version=V1)
    assert pkt.cpu().numpy().tobytes() == pkt_host
    rows, dec = tfa.codec_decode(ctx, pkt, version=V1)
    assert_decoded(cols, n, rows, dec)


@pytest.mark.gpu
def test_gpu_decode_rejects_bad_packets(tfa, ctx, dev):
    import torch
    with pytest.raises(tfa.TfgError) as e:  # ZSTD method byte, truncated frame header
        tfa.codec_decode(ctx, torch.tensor([0x90, 1, 0], dtype=torch.uint8, device=dev), version=V1)
    assert e.value.code == -1
    with pytest.raises(tfa.TfgError) as e:  # an unknown method byte
        tfa.codec_decode(ctx, torch.tensor([0x83, 1, 0], dtype=torch.uint8, device=dev), version=V1)
    assert e.value.code == -4
    with pytest.raises(tfa.TfgError) as e:  # LZ4 method byte, truncated frame header
        tfa.codec_decode(ctx, torch.tensor([0x82, 1, 0], dtype=torch.uint8, device=dev), version=V1)
    assert e.value.code == -1
    with pytest.raises(tfa.TfgError):  # truncated String column
        tfa.codec_decode(ctx, torch.tensor(list(b"\x01\x02" + sb(b"s") + sb(b"String") + b"\x05ab"),
                                           dtype=torch.uint8, device=dev), version=CHB)
    with pytest.raises(tfa.TfgError) as e:  # Decimal256 is out of scope
        tfa.codec_decode(ctx, torch.tensor(list(b"\x01\x01" + sb(b"d") + sb(b"Decimal(60,2)") + bytes(32)),
                                           dtype=torch.uint8, device=dev), version=CHB)
    assert e.value.code == -6
