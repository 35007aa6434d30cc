"""The zero-copy exchange (tfg_exchange_slices, tfg_alltoall_counts_n, tfg_string_rebase_offsets;
comm.hip) — the one exchange both front ends call: tfa::MPPExchange::exchange (host/operators.cpp)
and tiflash_amd.exchange.exchange_sides.  Every (peer, plane) slice is sent from where it lies in
the partitioned columns and received into the output column at its row offset (one RCCL group),
replacing the HashPartitionWriter -> MPPTunnelSetWriter packets of the reference
(Flash/Mpp/HashPartitionWriter.cpp:139-204, MPPTunnelSetWriter.cpp:365-400).  A world-1 RCCL
communicator exchanges with itself; the two-rank exchange runs in the C++ suite over TCP
(test_gpu_host_cpp.py) and, over gloo, in test_gpu_multirank.py."""
import ctypes
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Slice(ctypes.Structure):
    _fields_ = [("peer", ctypes.c_int), ("ptr", ctypes.c_void_p), ("bytes", ctypes.c_uint64)]


@pytest.fixture(scope="module")
def comm1(tfa, ctx):
    uid = (ctypes.c_uint8 * 128)()
    tfa.check(tfa.lib().tfg_comm_unique_id(uid, ctypes.c_size_t(128)))
    h = ctypes.c_void_p()
    tfa.check(tfa.lib().tfg_comm_init(ctx.h, 1, 0, uid, ctypes.c_size_t(128), ctypes.byref(h)))
    yield h
    tfa.lib().tfg_comm_destroy(h)


def test_exchange_slices_self(tfa, ctx, dev, comm1):
    """slices of several planes (widths 1..32, empty ones included) land byte-exact at their
    receive offsets; the bytes around them are untouched"""
    rng = np.random.default_rng(3)
    widths = [1, 8, 4, 16, 2, 32, 3]
    rows = [int(rng.choice([0, 1, 7, 1000, 70000])) for _ in widths]
    src = [torch.from_numpy(rng.integers(0, 256, r * w + 5, dtype=np.uint8)).to(dev) for r, w in zip(rows, widths)]
    dst = [torch.full((r * w + 11,), 0xAB, dtype=torch.uint8, device=dev) for r, w in zip(rows, widths)]
    sends = (_Slice * len(widths))(*[_Slice(0, s.data_ptr() + 5, r * w) for s, r, w in zip(src, rows, widths)])
    recvs = (_Slice * len(widths))(*[_Slice(0, d.data_ptr() + 7, r * w) for d, r, w in zip(dst, rows, widths)])
    tfa.check(tfa.lib().tfg_exchange_slices(comm1, len(widths), sends, len(widths), recvs))
    torch.cuda.synchronize()
    for s, d, r, w in zip(src, dst, rows, widths):
        assert torch.equal(d[7:7 + r * w].cpu(), s[5:5 + r * w].cpu())
        assert bool((d[:7] == 0xAB).all()) and bool((d[7 + r * w:] == 0xAB).all())


def test_alltoall_counts_n_self(tfa, ctx, comm1):
    send = (ctypes.c_uint64 * 3)(5, 0, 1 << 40)
    recv = (ctypes.c_uint64 * 3)()
    tfa.check(tfa.lib().tfg_alltoall_counts_n(comm1, 3, send, recv))
    assert list(recv) == [5, 0, 1 << 40]


def test_exchange_slices_rejects_bad_peer(tfa, ctx, dev, comm1):
    buf = torch.empty(8, dtype=torch.uint8, device=dev)
    bad = (_Slice * 1)(_Slice(1, buf.data_ptr(), 8))
    with pytest.raises(tfa.TfgError):
        tfa.check(tfa.lib().tfg_exchange_slices(comm1, 1, bad, 0, None))


def test_string_rebase_offsets(tfa, ctx, dev):
    """end offsets of three sources' String rows, each relative to its own chars -> one column"""
    parts = [[3, 5, 9], [], [1, 2], [4]]
    add, row0, flat, base = [], [0], [], 0
    want = []
    for p in parts:
        add.append(base)
        flat += p
        want += [x + base for x in p]
        row0.append(row0[-1] + len(p))
        base += p[-1] if p else 0
    off = torch.tensor(flat, dtype=torch.int64, device=dev)
    r0 = (ctypes.c_uint64 * len(row0))(*row0)
    ad = (ctypes.c_uint64 * len(add))(*add)
    tfa.check(tfa.lib().tfg_string_rebase_offsets(ctx.h, tfa._p(off), len(parts), r0, ad))
    torch.cuda.synchronize()
    assert off.cpu().tolist() == want


def test_exchange_sides_rccl_world1(tfa, ctx, dev):
    """exchange_sides through RCCL (the bench's N > 1 path) on a world-1 group: counts, then the
    zero-copy slices; every side comes back unchanged"""
    import torch.distributed as dist
    from tiflash_amd.exchange import exchange_sides
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        g = torch.Generator(device="cpu").manual_seed(5)
        a = torch.randint(-2**62, 2**62, (5000,), generator=g).to(dev)
        b = torch.randint(0, 2, (5000,), generator=g).to(torch.uint8).to(dev)
        c = torch.randint(-2**62, 2**62, (5000, 2), generator=g).to(dev)
        d = torch.rand(777, generator=g, dtype=torch.float64).to(dev)
        e = torch.randint(0, 255, (0,), generator=g).to(torch.uint8).to(dev)
        got = exchange_sides([([a, b, c], [0, 5000]), ([d], [0, 777]), ([e], [0, 0])], ctx=ctx)
        for x, y in zip([a, b, c, d, e], got[0] + got[1] + got[2]):
            assert x.dtype == y.dtype and x.shape == y.shape and torch.equal(x, y)
    finally:
        dist.destroy_process_group()
