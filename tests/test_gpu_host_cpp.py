"""C++ host operators (tiflash_amd/host: FilterTransformAction, Aggregator, Join,
HashPartitionWriter, MPPExchange, block streams) — tests/cpp/test_host.cpp run as one process.

The C++ test cases mirror the reference's gtests (known answers from tests/golden/) and check
randomized inputs against the CPU restatement; see the file header."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tiflash_amd", "host", "build", "test_host")
HOSTLIB = os.path.join(ROOT, "tiflash_amd", "libtiflash_amd_host.so")


def test_host_library_links():
    """CPU: the host library and the test driver are built and resolve every shared library."""
    assert os.path.exists(HOSTLIB) and os.path.exists(BIN)
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    assert "not found" not in out
    assert "libtiflash_amd_host.so" in out and "libtiflash_amd.so" in out


def test_host_driver_reports_missing_device():
    """CPU: without a GPU the driver fails loudly (exit 2), never falls back to a CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([BIN, ROOT], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "no device" in r.stderr


@pytest.mark.gpu
def test_host_operators_cpp():
    r = subprocess.run([BIN, ROOT], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    print(r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " failed" in r.stdout and "0 failed" in r.stdout


@pytest.mark.gpu
def test_mpp_exchange_two_ranks_cpp():
    """MPPExchange's fused exchange between two processes on one GPU, through the ExchangeTransport
    seam (a host-staged TCP transport in the test driver): fixed-width columns with and without
    null maps and a Decimal(30,2), a String key block, and a case where rank 1 sends no rows.
    Each rank checks that it received partition `rank` of both ranks' inputs."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen([BIN, ROOT, "--exchange-rank", str(r), str(port)], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=180)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    print("\n".join(outs))
    assert [p.returncode for p in procs] == [0, 0], "\n".join(outs)
    assert sum(o.count("[  OK  ] exchange case") for o in outs) == 6
