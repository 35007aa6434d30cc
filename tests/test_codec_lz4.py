"""LZ4 MPP packets (§8 f1): CHBlockChunkCodecV1 with CompressionMethod::LZ4.

Format (reference CHBlockChunkCodecV1.cpp:391-429, 555-581; IO/Compression/CompressionInfo.h:
24,53-58): the body of the uncompressed V1 packet (no 0x02 byte) in frames
`0x82 | UInt32 frame bytes (header included) | UInt32 raw bytes | LZ4 block`; the LZ4 block is the
published LZ4 block format (lz4 1.9.x, a third-party dependency the reference links and does not
vendor).  The reference's own LZ4 tests are round trips (gtest_block_chunk_codec.cpp:260-360:
encode(block, LZ4) == encode(str_view of the NONE packet, LZ4), decode == block), so parity is:
  CPU: the oracle (oracle/lz4.c) decodes blocks hand-derived from the format description to the
       bytes the description says, rejects malformed blocks, and round-trips its own encoder;
  GPU: the HIP decoder returns exactly the oracle's bytes for oracle-built packets (one frame per
       packet as the reference writes them, and many frames); the HIP encoder's packets decode to
       the original packet in the oracle and on the GPU; codec_decode of LZ4 packets returns the
       original columns; malformed packets fail with an error, never wrong data.
Compressed bytes themselves are not compared: LZ4 block bytes are an encoder's choice.
"""
import struct

import numpy as np
import pytest

from test_codec import V1, assert_decoded, make_block, to_dev


def frame(block: bytes, raw: int) -> bytes:
    return b"\x82" + struct.pack("<II", len(block) + 9, raw) + block


# hand-derived from the LZ4 block format description: (block, decoded bytes)
HAND = [
    (b"\x50hello", b"hello"),                                       # literals only
    (b"\x1fa\x01\x00\x01\x50bcdef", b"a" * 21 + b"bcdef"),         # offset 1, ml 15+1+4 = 20
    (b"\x34abc\x03\x00\x10z", b"abcabcabcab" + b"z"),              # offset 3 overlap, ml 8
    (b"\xf0\xff\x03" + bytes(range(256)) + bytes(17), bytes(range(256)) + bytes(17)),  # 15+255+3 literals
    (b"\x00", b""),                                                 # empty block
    (b"\x2fxy\x02\x00\xff\x00\x50abcde", b"xy" * 138 + b"abcde"),  # ml 15+255+0+4 = 274
    (b"\x80abcdefgh\x08\x00\x10z", b"abcdefghabcd" + b"z"),      # offset 8 >= ml 4: no overlap
]
MALFORMED = [
    b"",                          # no token
    b"\x50hell",                  # literals past the end
    b"\x14abcd\x00\x00\x00",      # offset 0
    b"\x14abcd\x05\x00\x10z",     # offset beyond the output
    b"\x14abcd\x04\x00",          # ends after a match (the last sequence must be literals)
    b"\xf0\xff",                  # literal length extension runs off the end
]


# ------------------------------------------------------------------ CPU: the oracle, pinned
@pytest.mark.parametrize("block,raw", HAND)
def test_oracle_decodes_hand_derived_blocks(orc, block, raw):
    assert orc.lz4_decompress_block(block, len(raw)) == raw
    assert orc.lz4_decompress_block(block, len(raw) - 1) is None if raw else True  # capacity is enforced


@pytest.mark.parametrize("block", MALFORMED)
def test_oracle_rejects_malformed_blocks(orc, block):
    assert orc.lz4_decompress_block(block, 4096) is None


def payloads(rng):
    yield b""
    yield b"x"
    yield bytes(12)
    yield bytes(13)
    yield bytes(rng.integers(0, 256, 5000, dtype=np.uint8))
    yield bytes(100_000)
    yield (b"abc" * 40_000)[:100_001]
    yield bytes(rng.integers(0, 4, 70_000, dtype=np.uint8))
    yield b"".join(b"key%08d|" % int(i) for i in rng.integers(0, 1000, 20_000))


def test_oracle_block_round_trip(orc):
    rng = np.random.default_rng(3)
    for raw in payloads(rng):
        blk = orc.lz4_compress_block(raw)
        assert orc.lz4_decompress_block(blk, len(raw)) == raw
        if len(raw) > 1000 and raw.count(raw[:1]) == len(raw):
            assert len(blk) < len(raw) // 100


def test_oracle_packet_frames(orc):
    pkt = frame(b"\x50hello", 5) + frame(b"\x30abc", 3)
    assert orc.lz4_packet_decompress(pkt) == b"\x02helloabc"
    assert orc.lz4_packet_decompress(pkt[:-1]) is None
    assert orc.lz4_packet_decompress(b"\x90" + pkt[1:]) is None          # ZSTD method byte
    assert orc.lz4_packet_decompress(frame(b"\x50hello", 6)) is None      # raw size mismatch
    body = b"\x02" + bytes(range(256)) * 300
    for fr in (0, 1000, 65536):
        assert orc.lz4_packet_decompress(orc.lz4_packet_compress(body, fr)) == body
    assert orc.lz4_packet_compress(body, 0)[0] == 0x82


# ------------------------------------------------------------------ GPU: HIP vs oracle
def dev_bytes(b, dev):
    import torch
    return torch.from_numpy(np.frombuffer(b, np.uint8).copy()).to(dev)


def host_bytes(t):
    return t.cpu().numpy().tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("block,raw", HAND)
def test_gpu_decompress_hand_derived(tfa, ctx, dev, block, raw):
    pkt = frame(block, len(raw)) + frame(b"\x50hello", 5)
    assert host_bytes(tfa.codec_decompress(ctx, dev_bytes(pkt, dev))) == b"\x02" + raw + b"hello"


@pytest.mark.gpu
@pytest.mark.parametrize("block", [m for m in MALFORMED if m])
def test_gpu_decompress_rejects_malformed(tfa, ctx, dev, block):
    with pytest.raises(tfa.TfgError):
        tfa.codec_decompress(ctx, dev_bytes(frame(block, 4), dev))


@pytest.mark.gpu
def test_gpu_decompress_rejects_bad_frames(tfa, ctx, dev):
    good = frame(b"\x50hello", 5)
    for bad in (good[:-1], b"\x90" + good[1:], frame(b"\x50hello", 6), frame(b"\x50hello", 4), good + b"\x82\x01"):
        with pytest.raises(tfa.TfgError):
            tfa.codec_decompress(ctx, dev_bytes(bad, dev))
    with pytest.raises(tfa.TfgError):  # a NONE packet is not an LZ4 packet
        tfa.codec_decompress(ctx, dev_bytes(b"\x02hello", dev))


@pytest.mark.gpu
def test_gpu_decompress_rejects_forged_raw_sizes(tfa, ctx, dev):
    # frames of a few bytes that each claim ~4 GiB of raw output: rejected from the headers alone
    # (more than LZ4 can expand a block to, and past DBMS_MAX_COMPRESSED_SIZE), before any output
    # is sized
    for raw in (0xFFFFFFFF, 0x40000001, 5 * 255 + 17):
        with pytest.raises(tfa.TfgError):
            tfa.codec_decompress(ctx, dev_bytes(frame(b"\x50hello", raw) * 64, dev))


@pytest.mark.gpu
@pytest.mark.parametrize("frame_raw", [0, 1000, 65536, 300_000])
def test_gpu_decompress_oracle_packets(tfa, orc, ctx, dev, frame_raw):
    rng = np.random.default_rng(11)
    for raw in payloads(rng):
        if not raw:
            continue
        body = b"\x02" + raw
        lz = orc.lz4_packet_compress(body, frame_raw)
        assert host_bytes(tfa.codec_decompress(ctx, dev_bytes(lz, dev))) == body


@pytest.mark.gpu
def test_gpu_decompress_large_single_frame(tfa, orc, ctx, dev):
    """The reference writes one frame per packet: a 7 MB body in one LZ4 block."""
    rng = np.random.default_rng(12)
    raw = b"".join(b"key%06d,%d;" % (int(a), int(b)) for a, b in rng.integers(0, 5000, (500_000, 2)))
    body = b"\x02" + raw
    lz = orc.lz4_packet_compress(body, 0)
    assert len(lz) < len(body) * 3 // 4
    assert host_bytes(tfa.codec_decompress(ctx, dev_bytes(lz, dev))) == body


@pytest.mark.gpu
def test_gpu_compress_round_trip(tfa, orc, ctx, dev):
    rng = np.random.default_rng(13)
    sizes = []
    for raw in list(payloads(rng)) + [bytes(rng.integers(0, 256, 65536 + 7, dtype=np.uint8)),
                                      bytes(65536), bytes(65536 * 3 - 1), bytes(13) + b"\x01" * 65536]:
        body = b"\x02" + raw
        lz = tfa.codec_compress(ctx, dev_bytes(body, dev))
        got = host_bytes(lz)
        if not raw:
            assert got == b""
            continue
        bound = tfa.lib().tfg_codec_compress_bound(len(body))
        assert len(got) <= bound
        assert got[0] == 0x82
        assert orc.lz4_packet_decompress(got) == body  # the reference-format reader accepts it
        assert host_bytes(tfa.codec_decompress(ctx, lz)) == body
        sizes.append((len(raw), len(got)))
    z = [g for r, g in sizes if r == 100_000][0]
    assert z < 2000, sizes  # long zero runs compress ~250x


@pytest.mark.gpu
def test_gpu_compress_rejects(tfa, ctx, dev):
    with pytest.raises(tfa.TfgError):  # not an uncompressed packet
        tfa.codec_compress(ctx, dev_bytes(b"\x82abc", dev))
    with pytest.raises(tfa.TfgError):  # no such method (NONE is not a compressor)
        tfa.codec_compress(ctx, dev_bytes(b"\x02abc", dev), method=tfa.COMPRESSION_NONE)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 50_000])
def test_gpu_codec_decode_lz4_packets(tfa, orc, ctx, dev, n):
    """decode(header, LZ4 packet) == the Block (CHBlockChunkCodecV1::decode, :567-581): both the
    oracle's one-frame packet and the GPU encoder's packet of the GPU-encoded Block."""
    rng = np.random.default_rng(20 + n)
    cols = make_block(rng, n)
    plain = orc.codec_encode(cols, n, version=V1)
    rows, dec = tfa.codec_decode(ctx, dev_bytes(orc.lz4_packet_compress(plain, 0), dev), version=V1)
    assert_decoded(cols, n, rows, dec)
    gpkt = tfa.codec_encode(ctx, to_dev(cols, dev), n, version=V1)
    lz = tfa.codec_compress(ctx, gpkt)
    assert orc.lz4_packet_decompress(host_bytes(lz)) == plain
    rows, dec = tfa.codec_decode(ctx, lz, version=V1)
    assert_decoded(cols, n, rows, dec)


@pytest.mark.gpu
@pytest.mark.parametrize("frame", [0, 1000, 7000, 65536, 300_000])
def test_gpu_decompress_frame_table_shapes(tfa, orc, ctx, dev, frame):
    """The frame table of a multi-segment packet (the segmented parse, lz4.hip frames_seg_kernel /
    frames_join_kernel, falling back to the serial walk): one frame, frames smaller than the
    parse's per-segment capacity allows, frames of a few KB, 64 KB and larger than a segment."""
    rng = np.random.default_rng(frame + 3)
    raw = b"".join(b"key%06d,%d;" % (int(a), int(b)) for a, b in rng.integers(0, 5000, (120_000, 2)))
    body = b"\x02" + raw
    lz = orc.lz4_packet_compress(body, frame)
    assert host_bytes(tfa.codec_decompress(ctx, dev_bytes(lz, dev))) == body
    # a frame header forged inside the data of a later frame must not confuse the parse: the
    # packet with one byte less is malformed and stays an error
    with pytest.raises(tfa.TfgError):
        tfa.codec_decompress(ctx, dev_bytes(lz[:-1], dev))
