"""CPU tests of bench.py's cpu_baseline legs for the chain and frame configs: they time the
reference (or the oracle port) over a host copy of the batch and their outputs agree with
the oracle. Small batches; no GPU."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402
from aipstack_amd import synth  # noqa: E402


def test_cpu_baseline_chain_matches_oracle():
    n = 2000
    spec = {"n": n, "seed": synth.SEED_DATA}
    hdr = bench.CHAIN_HDR_STRIDE * n
    host = np.empty(hdr + bench.CHAIN_PAYLOAD * n, dtype=np.uint8)
    synth.fill_host(host, spec["seed"], 0)
    buf = torch.from_numpy(host)
    # make_chains's table, built over a "device" base that is really this host buffer
    rng = np.random.default_rng(spec["seed"])
    split = rng.integers(1, bench.CHAIN_PAYLOAD, n).astype(np.uint64)
    base = 0x7000_0000_0000  # any bias: the baseline translates addr - base + host
    i = np.arange(n, dtype=np.uint64)
    addr = np.empty(3 * n, dtype=np.uint64)
    lens = np.empty(3 * n, dtype=np.uint32)
    addr[0::3] = base + bench.CHAIN_HDR_STRIDE * i
    lens[0::3] = bench.CHAIN_HDR
    addr[1::3] = base + hdr + bench.CHAIN_PAYLOAD * i
    lens[1::3] = split
    addr[2::3] = addr[1::3] + split
    lens[2::3] = bench.CHAIN_PAYLOAD - split
    chain = {"buf": buf, "base": base, "n": n, "addr_host": addr, "len_host": lens,
             "index_host": np.arange(n + 1, dtype=np.uint64) * 3,
             "states_host": rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32),
             "payload": (bench.CHAIN_HDR + bench.CHAIN_PAYLOAD) * n}
    res = bench.cpu_baseline_chain(chain)
    assert res["value"] > 0 and res["cores"] == 1
    assert res["kind"] in ("reference", "port")
    # the baseline's outputs are the oracle's: chain_check compares them
    assert bench.chain_check(chain, _baseline_out(chain)) .startswith("bit-exact")


def _baseline_out(chain):
    # recompute through the same entry point the baseline times (1 thread, 1 pass)
    import ctypes
    host = chain["buf"].numpy()
    out = np.empty(chain["n"], dtype=np.uint16)
    ref = os.path.join(ROOT, "oracle", "_ref", "libref_chksum.so")
    if not os.path.exists(ref):
        pytest.skip("reference build absent: the port path is the oracle itself")
    lib = ctypes.CDLL(ref)
    lib.ref_time_batch_chain.restype = ctypes.c_double
    lib.ref_time_batch_chain.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64] + \
        [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]
    bias = (chain["base"] - host.ctypes.data) % (1 << 64)
    lib.ref_time_batch_chain(3, 1, bias, chain["addr_host"].ctypes.data,
                             chain["len_host"].ctypes.data, chain["index_host"].ctypes.data,
                             chain["states_host"].ctypes.data, chain["n"], out.ctypes.data)
    return out


@pytest.mark.parametrize("layout", ["rx", "tx"])
def test_cpu_baseline_frames(layout):
    spec = {"layout": layout, "n": 3000, "seed": synth.SEED_DATA}
    frames = bench.host_shard(spec)
    res = bench.cpu_baseline_frames(spec, frames)
    assert res["value"] > 0 and res["kind"] == "port" and res["cores"] == 1
    assert res["affinity_cores"] >= 1
