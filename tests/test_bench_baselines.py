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


def test_oracle_check_threaded_reference_and_mismatch():
    """Every rank's own-shard check (bench.oracle_check): the reference's IpChksumInverted over
    several threads (or the oracle port), bit-exact on the right answers, MISMATCH on a
    flipped one."""
    import ctypes
    for layout in ("strided", "csr"):
        if layout == "strided":
            spec = {"layout": "strided", "n": 5000, "plen": 1500, "stride": 1500,
                    "total": 5000 * 1500, "byte_offset": 3 * 5000 * 1500, "offsets": None,
                    "first_packet": 15000}
        else:
            off = synth.mixed_offsets(2 * 4000)
            spec = {"layout": "csr", "n": 4000, "plen": None,
                    "offsets": off[4000:] - off[4000], "byte_offset": int(off[4000]),
                    "first_packet": 4000}
            spec["total"] = int(spec["offsets"][-1])
        host = bench.host_shard(spec)
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
        want = np.empty(spec["n"], dtype=np.uint16)
        if layout == "strided":
            lib.oracle_batch_strided.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32]
            lib.oracle_batch_strided(host.ctypes.data, 1500, 1500, spec["n"], want.ctypes.data, 0)
        else:
            lib.oracle_batch_csr.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.c_void_p, ctypes.c_uint32]
            o = spec["offsets"].astype(np.uint64)
            lib.oracle_batch_csr(host.ctypes.data, o.ctypes.data, spec["n"], want.ctypes.data, 0)
        assert bench.oracle_check(spec, want, threads=4).startswith("bit-exact")
        bad = want.copy()
        bad[123] ^= 1
        assert bench.oracle_check(spec, bad, threads=4) == "MISMATCH"


def test_slots_and_records_checks():
    """The RX2K / C2K parity check (bench.slots_check) and the TXREC one (records_check)."""
    import ctypes
    spec = {"layout": "rxslot", "n": 3000, "seed": synth.SEED_DATA}
    frames = bench.host_shard(spec)
    ring, lens = synth.to_slots(frames, spec["offsets"], 2048)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    want = np.empty(3000, dtype=np.uint8)
    lib.oracle_rx_verify_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]
    o = spec["offsets"].astype(np.uint64)
    lib.oracle_rx_verify_batch(frames.ctypes.data, o.ctypes.data, 3000, want.ctypes.data)
    assert bench.slots_check("rxslot", ring, lens, want).startswith("bit-exact")
    want[7] ^= 1
    assert bench.slots_check("rxslot", ring, lens, want) == "MISMATCH"
    # records: what the device returns, built here from the oracle's fill
    tspec = {"layout": "txrec", "n": 2000, "seed": 77}
    fr = bench.host_shard(tspec)
    filled = fr.copy()
    st = np.empty(2000, dtype=np.uint8)
    lib.oracle_tx_fill_batch.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_uint64, ctypes.c_void_p]
    to = tspec["offsets"].astype(np.uint64)
    lib.oracle_tx_fill_batch(filled.ctypes.data, to.ctypes.data, 2000, st.ctypes.data)
    rec = np.zeros(2000, dtype=np.uint64)
    for i in range(2000):
        s = int(to[i])
        hl = (int(filled[s + 14]) & 15) * 4 if filled[s + 12] == 8 and filled[s + 13] == 0 else 0
        w1 = int(st[i]) << 16
        w0 = 0
        if fr[s + 24] != filled[s + 24] or fr[s + 25] != filled[s + 25] or st[i] in (3, 6, 8, 4):
            if hl:
                w0 |= (int(filled[s + 24]) << 8) | int(filled[s + 25])
                w1 |= 1 << 8
        if st[i] == 6:
            proto = int(filled[s + 23])
            fo = {6: 16, 17: 6, 1: 2}[proto]
            fld = 14 + hl + fo
            w0 |= ((int(filled[s + fld]) << 8) | int(filled[s + fld + 1])) << 16
            w1 |= fld | (1 << 9)
        rec[i] = w0 | (w1 << 32)
    assert bench.records_check(tspec, fr, fr.copy(), rec.view(np.int64)).startswith("bit-exact")
    rec[5] ^= np.uint64(1 << 16)
    assert bench.records_check(tspec, fr, fr.copy(), rec.view(np.int64)) == "MISMATCH"


def test_tx_slots_check():
    """The TX2K parity check (bench.tx_slots_check): filled slots and statuses vs the oracle's
    fill of the ring as it was before the timed fills."""
    import ctypes
    spec = {"layout": "txslot", "n": 2500, "seed": 91}
    frames = bench.host_shard(spec)
    ring, lens = synth.to_slots(frames, spec["offsets"], 2048)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "libchksum_oracle.so"))
    filled = ring.copy()
    st = np.empty(2500, dtype=np.uint8)
    lib.oracle_tx_fill_slotted.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p]
    lib.oracle_tx_fill_slotted(filled.ctypes.data, 2048, lens.ctypes.data, 2500, st.ctypes.data)
    assert not np.array_equal(filled, ring)  # raw frames: the fill changes them
    assert bench.tx_slots_check(ring, lens, filled, st).startswith("bit-exact")
    bad = filled.copy()
    bad[2048 * 7 + 24] ^= 1
    assert bench.tx_slots_check(ring, lens, bad, st) == "MISMATCH"
    assert bench.algorithmic_bytes("txslot", 10, 1000) == 1000 + 90


def test_pmc_traffic_only_for_the_current_kernels(tmp_path, monkeypatch):
    """roofline.traffic comes from profiles/pmc_traffic.json only while the entry's device-code
    digest (the .hip_fatbin of libaipstack_chksum.so) matches the loaded library's; otherwise
    null, the old value under traffic_stale."""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "pmc_traffic.json").write_text(json.dumps({
        "A": {"hbm_bytes_per_launch": 123, "device_code": "abcd" * 4},
        "C": {"hbm_bytes_per_launch": 456, "device_code": "0" * 16},
        "B": {"hbm_bytes_per_launch": 789, "kernel_sources": "f" * 16}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "device_code_digest", lambda lib_path=None: "abcd" * 4)
    assert bench._pmc_traffic("A") == (123, None)
    t, stale = bench._pmc_traffic("C")
    assert t is None and stale["hbm_bytes_per_launch"] == 456
    t, stale = bench._pmc_traffic("B")  # an entry without a device-code digest: stale
    assert t is None and stale["hbm_bytes_per_launch"] == 789
    assert bench._pmc_traffic("A2K") == (None, None)


def test_device_code_digest_reads_the_fatbin():
    """The digest is the .hip_fatbin section's hash: stable for the built library, None for a
    file that is not an ELF with that section."""
    import tempfile
    lib = os.path.join(ROOT, "aipstack_amd", "lib", "libaipstack_chksum.so")
    d = bench.device_code_digest(lib)
    assert d is not None and len(d) == 16 and d == bench.device_code_digest(lib)
    hook = os.path.join(ROOT, "aipstack_amd", "lib", "libaipstack_chksum_hook.so")
    assert bench.device_code_digest(hook) is None  # host-only library: no device code
    with tempfile.NamedTemporaryFile() as f:
        f.write(b"not an elf")
        f.flush()
        assert bench.device_code_digest(f.name) is None


@pytest.mark.parametrize("config", ["A", "C"])
def test_cpu_baseline_carries_the_hook(config):
    """The N=1 line's cpu_baseline gains a `hook` entry: the repo's drop-in
    libaipstack_chksum_hook IpChksumInverted over the same batch, 1 thread and every affinity
    core, labelled as the repo's (not the reference), its outputs equal to the reference
    leg's."""
    import subprocess
    subprocess.run(["make", "-C", os.path.join(ROOT, "tools"), "build/libhook_time.so"],
                   check=True, stdout=subprocess.DEVNULL)
    spec = bench.shard_spec(config, 0, 1, n=4000)
    res, out = bench.cpu_baseline(spec)
    hook = res["hook"]
    assert hook["value"] > 0 and hook["cores"] == 1 and "not the reference" in hook["kind"]
    assert hook["matches_reference"] is True
    if res["affinity_cores"] > 1:
        assert hook["all_cores"]["threads"] == res["affinity_cores"]
