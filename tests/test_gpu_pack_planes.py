"""The fused exchange's device pack / unpack (tfg_pack_planes / tfg_unpack_planes, comm.hip) — the
layout both exchanges put on the wire: tfa::MPPExchange::exchange (host/operators.cpp) and
tiflash_amd.exchange.exchange_sides.  Peer p's segment = every plane's rows of p in plane order;
unpack concatenates each plane's rows source after source.  Checked byte-exact against the same
layout built with torch slicing (partition-major inputs, as HashPartitionWriter's scatter leaves
them, Flash/Mpp/HashPartitionWriter.cpp:139-204)."""
import ctypes
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pack_ref(planes, widths, rows):
    """planes[p][k]: uint8 [rows[p][k] * widths[k]] tensors (None = zeros)"""
    segs, out = [], []
    for p in range(len(rows)):
        seg = []
        for k, w in enumerate(widths):
            n = rows[p][k] * w
            seg.append(planes[p][k].cpu() if planes[p][k] is not None else torch.zeros(n, dtype=torch.uint8))
        segs.append(sum(x.numel() for x in seg))
        out += seg
    return torch.cat(out + [torch.empty(0, dtype=torch.uint8)]), segs


@pytest.mark.parametrize("nparts,seed", [(1, 0), (4, 1), (8, 2), (3, 3)])
def test_pack_unpack_planes(tfa, ctx, dev, nparts, seed):
    rng = np.random.default_rng(seed)
    widths = [1, 8, 4, 16, 2, 32, 1, 3]
    NP = len(widths)
    rows = [[int(rng.choice([0, 1, 7, 1000, 70000])) for _ in range(NP)] for _ in range(nparts)]
    planes = [[None if (k == 6 and p % 2) else
               torch.from_numpy(rng.integers(0, 256, rows[p][k] * widths[k], dtype=np.uint8)).to(dev)
               for k in range(NP)] for p in range(nparts)]
    want, segs = _pack_ref(planes, widths, rows)
    out = torch.empty(max(want.numel(), 1), dtype=torch.uint8, device=dev)
    ptrs = (ctypes.c_void_p * (nparts * NP))(*[planes[p][k].data_ptr() if planes[p][k] is not None and rows[p][k]
                                               else None for p in range(nparts) for k in range(NP)])
    w_arr = (ctypes.c_int * NP)(*widths)
    r_arr = (ctypes.c_uint64 * (nparts * NP))(*[rows[p][k] for p in range(nparts) for k in range(NP)])
    seg = (ctypes.c_uint64 * nparts)()
    tfa.check(tfa.lib().tfg_pack_planes(ctx.h, nparts, NP, ptrs, w_arr, r_arr, tfa._p(out), seg))
    torch.cuda.synchronize()
    assert list(seg) == segs
    assert torch.equal(out[:want.numel()].cpu(), want)
    # unpack the packed buffer as if each segment came from a different source
    outs = [torch.full((sum(rows[p][k] for p in range(nparts)) * widths[k] + 1,), 0xAB, dtype=torch.uint8, device=dev)
            for k in range(NP)]
    tfa.check(tfa.lib().tfg_unpack_planes(ctx.h, nparts, NP, w_arr, r_arr, tfa._p(out), tfa._ptr_array(outs)))
    torch.cuda.synchronize()
    for k in range(NP):
        exp = torch.cat([(planes[p][k].cpu() if planes[p][k] is not None
                          else torch.zeros(rows[p][k] * widths[k], dtype=torch.uint8)) for p in range(nparts)])
        assert torch.equal(outs[k][:-1].cpu(), exp), k
        assert int(outs[k][-1]) == 0xAB  # nothing past the plane's rows


def test_pack_planes_rejects_bad_args(tfa, ctx, dev):
    w = (ctypes.c_int * 1)(0)
    r = (ctypes.c_uint64 * 1)(1)
    seg = (ctypes.c_uint64 * 1)()
    p = (ctypes.c_void_p * 1)(None)
    out = torch.empty(8, dtype=torch.uint8, device=dev)
    with pytest.raises(tfa.TfgError):
        tfa.check(tfa.lib().tfg_pack_planes(ctx.h, 1, 1, p, w, r, tfa._p(out), seg))


def test_exchange_sides_rccl_world1(tfa, ctx, dev):
    """exchange_sides through RCCL (the bench's N > 1 path) on a world-1 group: the device pack ->
    all_to_all_single -> unpack round trip returns every side unchanged."""
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
