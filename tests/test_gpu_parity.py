"""GPU parity: every batch entry point of libaipstack_chksum.so (through the C-ABI) against
the oracle and the reference's golden vectors -- bit-exact, as required for integer work.

Covers the BASELINE configs at full size (A: 1M x 1500 B, B: 256K x 9000 B, C: 2M mixed
64-1500 B with odd lengths/starts and all-0x00 / all-0xFF / sum=0 mod 0xFFFF packets, D:
a 1M shard of the 8-GPU batch) plus the edge cases the reference contract admits: empty
batches and packets, ragged counts, odd base pointers, len 65535, FINAL flag, seeds.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import aipstack_amd as A
from aipstack_amd import synth
from conftest import ROOT

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    assert A.device_check(0) == A.AIPSTACK_CHKSUM_OK, "device 0 is not gfx950"


def _d(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.cpu().numpy()


class _engine_copy_mode:
    """Engines created inside read registered input in place (zero_copy=1, the default) or
    DMA it first (0: the 2-D slot copies, whole spans); restored on exit."""

    def __init__(self, zero_copy):
        self.zc = int(zero_copy)

    def __enter__(self):
        assert A._lib.load().aipstack_chksum_tune(b"engine_zero_copy", self.zc) == 0

    def __exit__(self, *exc):
        A._lib.load().aipstack_chksum_tune(b"engine_zero_copy", 1)


def test_native_library_loaded_in_process():
    """The in-tree product library is what this process runs, and it was built from the
    sources beside it (its embedded source digest equals the tree's): a stale prebuilt .so
    pushed to the box fails here."""
    from aipstack_amd import _lib
    maps = open("/proc/self/maps").read()
    assert os.path.join("aipstack_amd", "lib", "libaipstack_chksum.so") in maps
    assert _lib.load().aipstack_chksum_source_digest().decode() == _lib.tree_source_digest()


def test_golden_flat_cases_strided_n1(golden):
    """Each reference golden case (start, len) as a 1-packet strided launch."""
    b = golden["blob"]
    db = _d(b)
    cases = golden["flat"]["flat"]
    out = torch.empty(len(cases), dtype=torch.uint16, device=DEV)
    fin = torch.empty(len(cases), dtype=torch.uint16, device=DEV)
    for i, (o, l, _, _) in enumerate(cases):
        A.chksum_batch_strided(db, max(l, 1), l, 1, out=out[i:], byte_offset=o)
        A.chksum_batch_strided(db, max(l, 1), l, 1, out=fin[i:], byte_offset=o, final=True)
    got, gotf = _np(out), _np(fin)
    want = np.array([c[2] for c in cases], dtype=np.uint16)
    wantf = np.array([c[3] for c in cases], dtype=np.uint16)
    bad = np.nonzero((got != want) | (gotf != wantf))[0]
    assert bad.size == 0, [cases[i] for i in bad[:10]]


def test_golden_batch_fixtures_device_generated(golden):
    bc = golden["batch"]
    m = bc["mixed_csr"]
    off = synth.mixed_offsets(m["n"], m["len_seed"])
    buf = torch.empty(int(off[-1]), dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, m["data_seed"])
    doff = _d(off)
    synth.apply_classes_device(buf, doff, m["len_seed"])
    assert _np(A.chksum_batch_csr(buf, doff)).tolist() == m["inverted"]
    for name in ("strided_1500", "strided_9000"):
        c = bc[name]
        buf = torch.empty(c["stride"] * c["n"], dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, c["data_seed"])
        got = _np(A.chksum_batch_strided(buf, c["stride"], c["len"], c["n"]))
        assert got.tolist() == c["inverted"]


def test_device_generator_matches_host():
    buf = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)
    for off in (0, 3, 4096, 12345):
        synth.fill_device(buf, 42, off)
        assert np.array_equal(_np(buf), synth.random_bytes(42, 1 << 20, off))


@pytest.mark.parametrize("cfg,n,plen", [("A", 1 << 20, 1500), ("B", 256 << 10, 9000)])
def test_full_size_strided(oracle, cfg, n, plen):
    buf = torch.empty(n * plen, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, synth.SEED_DATA)
    got = _np(A.chksum_batch_strided(buf, plen, plen, n))
    host = _np(buf)
    want = oracle.batch_strided(host, plen, plen, n)
    assert np.array_equal(got, want), f"config {cfg}: {np.count_nonzero(got != want)} mismatches"
    # idempotence: a second launch gives the same result
    assert np.array_equal(_np(A.chksum_batch_strided(buf, plen, plen, n)), got)
    # FINAL flag = bitwise NOT, packet for packet
    fin = _np(A.chksum_batch_strided(buf, plen, plen, n, final=True))
    assert np.array_equal(fin, ~got)
    # the JUST_WRITTEN hint reads the batch another way: the same sums
    assert np.array_equal(_np(A.chksum_batch_strided(buf, plen, plen, n, just_written=True)), got)


def test_full_size_mixed_csr(oracle):
    n = 2 << 20
    off = synth.mixed_offsets(n)
    buf = torch.empty(int(off[-1]), dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, synth.SEED_DATA)
    doff = _d(off)
    synth.apply_classes_device(buf, doff)
    got = _np(A.chksum_batch_csr(buf, doff))
    host = _np(buf)
    want = oracle.batch_csr(host, off)
    assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} mismatches"
    cls = synth.mixed_classes(n)
    lens = np.diff(off)
    assert np.all(got[cls == 1] == 0x0000)          # all-zero packets
    assert np.all(got[cls == 2] == 0xFFFF)          # nonzero, sum = 0 mod 0xFFFF
    ff = (cls == 0)
    assert np.all(got[ff & (lens % 2 == 0)] == 0xFFFF)  # k * 0xFFFF
    assert np.all(got[ff & (lens % 2 == 1)] == 0xFF00)  # k * 0xFFFF + 0xFF00 tail
    assert np.any(off[:-1] % 2 == 1) and np.any(lens % 2 == 1)


def test_config_d_shard_of_8(oracle):
    """Rank 7's shard of the 8-GPU batch (packets [7M, 8M)) as bench.py builds it."""
    n, plen, rank = 1 << 20, 1500, 7
    buf = torch.empty(n * plen, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, synth.SEED_DATA, rank * n * plen)
    got = _np(A.chksum_batch_strided(buf, plen, plen, n))
    want = oracle.batch_strided(_np(buf), plen, plen, n)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 1000, 4097])
@pytest.mark.parametrize("base", [0, 1, 2, 3, 5, 8, 13])
def test_ragged_counts_and_odd_bases(oracle, n, base):
    plen = 1500 if n % 2 else 1499
    buf = torch.empty(n * plen + 64, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, 9)
    got = _np(A.chksum_batch_strided(buf, plen, plen, n, byte_offset=base))
    want = oracle.batch_strided(_np(buf), plen, plen, n, base_off=base)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("plen", [0, 1, 2, 3, 15, 16, 17, 31, 33, 1023, 1024, 1025, 2032,
                                  2033, 4095, 8999, 9001, 16383, 65534, 65535])
def test_lengths(oracle, plen):
    n = 300
    stride = max(plen, 1) + 7   # overlapping-free, misaligned starts
    buf = torch.empty(n * stride + 64, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, plen + 1)
    got = _np(A.chksum_batch_strided(buf, stride, plen, n, byte_offset=3))
    want = oracle.batch_strided(_np(buf), stride, plen, n, base_off=3)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("plen", [2, 15, 16, 17, 31, 100, 1499, 1500, 2047, 9000, 65535])
def test_slotted_packets(oracle, plen):
    """Packets in fixed slots (stride % 16 == 0, stride != len: one packet per wavefront),
    at every start offset within a 16-byte segment."""
    rng = np.random.default_rng(plen)
    for base in (0, 1, 7, 8, 15):
        for extra in (0, 16, 512):
            stride = ((base % 16 + plen + 15) // 16) * 16 + extra
            if stride == plen:
                stride += 16
            for n in (1, 63, 64, 65, 1000 if plen < 10000 else 100):
                buf = torch.empty(n * stride + 64, dtype=torch.uint8, device=DEV)
                synth.fill_device(buf, int(rng.integers(0, 1 << 30)))
                got = _np(A.chksum_batch_strided(buf, stride, plen, n, byte_offset=base))
                want = oracle.batch_strided(_np(buf), stride, plen, n, base_off=base)
                assert np.array_equal(got, want), (plen, stride, base, n,
                                                   np.nonzero(got != want)[0][:8])


def test_slotted_full_size_ring_slots(oracle):
    """bench.py's A2K: 1M x 1500-byte packets in 2048-byte slots, all 0x00 / all 0xFF
    slots mixed in; FINAL flag."""
    n, plen, stride = 1 << 20, 1500, 2048
    buf = torch.empty(n * stride, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, synth.SEED_DATA)
    v = buf.view(n, stride)
    v[::97, :plen] = 0
    v[5::101, :plen] = 0xFF
    got = _np(A.chksum_batch_strided(buf, stride, plen, n))
    want = oracle.batch_strided(_np(buf), stride, plen, n)
    assert np.array_equal(got, want), np.count_nonzero(got != want)
    i = np.arange(n)
    assert np.all(got[(i % 97 == 0) & (i % 101 != 5)] == 0)      # all-zero packets
    assert np.all(got[i % 101 == 5] == 0xFFFF)                     # all-0xFF, even length
    fin = _np(A.chksum_batch_strided(buf, stride, plen, n, final=True))
    assert np.array_equal(fin, ~want)


def _tune(key, value):
    from aipstack_amd import _lib
    assert _lib.load().aipstack_chksum_tune(key.encode(), value) == A.AIPSTACK_CHKSUM_OK


@pytest.fixture
def stream_mode():
    """Yields a setter for the stream-mode tunable; restores automatic afterwards."""
    yield lambda v: _tune("stream", v)
    _tune("stream", 0)


@pytest.mark.parametrize("su", [2, 4, 8])
@pytest.mark.parametrize("plen", [0, 1, 2, 3, 15, 16, 17, 31, 33, 1023, 1024, 1025, 1500, 2033,
                                  9000, 65535])
def test_stream_mode_back_to_back_strided(oracle, stream_mode, plen, su):
    """stride == len: every chunk is read as one contiguous run (stream mode)."""
    stream_mode(su)
    for n, base in ((1, 0), (63, 3), (65, 1), (300, 13)):
        if plen * n > 64 << 20:
            n = 70
        buf = torch.empty(n * max(plen, 1) + 64, dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, plen + n)
        got = _np(A.chksum_batch_strided(buf, plen, plen, n, byte_offset=base))
        want = oracle.batch_strided(_np(buf), plen, plen, n, base_off=base)
        assert np.array_equal(got, want), (plen, n, base, np.nonzero(got != want)[0][:8])


@pytest.mark.parametrize("su", [-1, 2, 4, 8])
def test_stream_mode_csr_tiny_and_mixed(oracle, stream_mode, su):
    """Back-to-back CSR packets from 0 to 65535 bytes, many per 16-byte segment, odd starts,
    all-0x00 / all-0xFF packets; stream mode (su > 0) and per-packet mode (su = -1)."""
    stream_mode(su)
    rng = np.random.default_rng(17)
    for choice in ([0, 0, 1, 2, 3, 5, 7, 16, 17, 31], [0, 64, 65, 1499, 1500, 9000, 65535],
                   list(range(0, 200))):
        n = 20000 if max(choice) < 10000 else 3000
        lens = rng.choice(choice, size=n)
        off = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        off += 7
        buf = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, n + 5)
        host = _np(buf)
        for j in range(0, n, 13):
            host[off[j]:off[j + 1]] = 0 if j % 2 else 0xFF
        buf = _d(host)
        got = _np(A.chksum_batch_csr(buf, _d(off)))
        want = oracle.batch_csr(host, off)
        assert np.array_equal(got, want), (choice[:3], np.nonzero(got != want)[0][:8])
        fin = _np(A.chksum_batch_csr(buf, _d(off), final=True))
        assert np.array_equal(fin, ~want)


def test_stream_mode_off_matches_on_config_c(stream_mode):
    """Config C through stream mode (2, 4, 8 windows) and per-packet mode: identical."""
    n = 2 << 20
    off = synth.mixed_offsets(n)
    buf = torch.empty(int(off[-1]), dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, synth.SEED_DATA)
    doff = _d(off)
    synth.apply_classes_device(buf, doff)
    outs = []
    for su in (-1, 2, 4, 8):
        stream_mode(su)
        outs.append(_np(A.chksum_batch_csr(buf, doff)))
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])


def test_stream_mode_mixed_chunks(oracle):
    """A CSR batch whose chunks alternate between back to back and not (a decreasing
    offset, a packet over 2^17 bytes): both modes in one launch."""
    rng = np.random.default_rng(23)
    n = 64 * 40
    lens = rng.integers(0, 2000, size=n)
    lens[64 * 3 + 5] = 1 << 17          # too long for stream mode: chunk 3 per packet
    off = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    bad = 64 * 7 + 8
    off[bad + 1] = off[bad] - 10        # decreasing: packet `bad` is empty (E < S)
    buf = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, 29)
    got = _np(A.chksum_batch_csr(buf, _d(off)))
    host = _np(buf)
    want = np.array([oracle.inverted(host, int(off[i]), int(max(off[i + 1] - off[i], 0)))
                     for i in range(n)], dtype=np.uint16)
    assert want[bad] == 0
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]


@pytest.mark.parametrize("chunk", [0, 1, 8, 64])
@pytest.mark.parametrize("gather", [0, -1, 1, 2])
def test_strided_and_csr_in_every_read_form(oracle, gather, chunk):
    """The read forms of back-to-back batches give the same sums, odd starts and lengths
    included: short runs (gather 1, the strided default since round 5; 2 also for CSR), the
    gathered stream (0, round 4) and stream mode with long chunks (-1). chunk_packets forces
    the short-run shape on these small batches (0: the automatic shape)."""
    _tune("gather", gather)
    _tune("chunk_packets", chunk)
    try:
        buf = torch.empty(1 << 22, dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, 31)
        hb = _np(buf)
        for plen in (1, 63, 64, 1500, 1501, 9000):
            n = min(3000, (buf.numel() - 3) // plen)
            got = _np(A.chksum_batch_strided(buf, plen, plen, n, byte_offset=3))
            assert np.array_equal(got, oracle.batch_strided(hb[3:], plen, plen, n)), plen
        rng = np.random.default_rng(32)
        lens = rng.integers(0, 1600, 4000)  # ~3.2 MB of the 4 MiB buffer
        off = np.concatenate([[5], 5 + np.cumsum(lens)]).astype(np.int64)
        assert off[-1] <= buf.numel()
        got = _np(A.chksum_batch_csr(buf, _d(off)))
        assert np.array_equal(got, oracle.batch_csr(hb, off.astype(np.uint64)))
    finally:
        _tune("gather", 1)
        _tune("chunk_packets", 0)


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("plen,n", [(64, 300000), (1500, 270000), (9000, 40000)])
def test_short_runs_large_batches(oracle, plen, n, mode):
    """Back-to-back strided batches large enough for the default short-run shape (one chunk of
    ~12 KiB per wave), at an odd base, against the oracle: stream prefixes through buffer loads
    (tunable short_loads 0) or global loads (1), column runs (2) and segment tables (3)."""
    _tune("short_loads", mode)
    try:
        buf = torch.empty(n * plen + 7, dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, 41 + plen)
        got = _np(A.chksum_batch_strided(buf, plen, plen, n, byte_offset=7, final=True))
        want = oracle.batch_strided(_np(buf)[7:], plen, plen, n, final=True)
        assert np.array_equal(got, want)
        # the JUST_WRITTEN hint (column runs: boundary segments captured from the stream)
        got = _np(A.chksum_batch_strided(buf, plen, plen, n, byte_offset=7, final=True,
                                         just_written=True))
        assert np.array_equal(got, want)
    finally:
        _tune("short_loads", -1)


@pytest.mark.parametrize("chunk", [1, 2, 4, 8, 16, 32])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_short_run_forms_ragged(oracle, mode, chunk):
    """The short-run forms at every chunk size (column runs cap chunks at 16 packets; runs
    over the segment table's 1,536 segments take the per-packet path) on ragged strided and
    CSR batches: lengths 0..3000 with odd starts, empty packets, a batch that ends mid-chunk,
    all-0x00 / all-0xFF packets."""
    _tune("short_loads", mode)
    _tune("chunk_packets", chunk)
    try:
        buf = torch.empty(1 << 23, dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, 51 + chunk)
        buf[1000:5000] = 0
        buf[9000:12000] = 255
        hb = _np(buf)
        rng = np.random.default_rng(60 + chunk + 100 * mode)
        for plen in (0, 1, 15, 16, 17, 1023, 1500, 3001):
            n = min(2999, (buf.numel() - 9) // max(plen, 1))
            want = oracle.batch_strided(hb[9:], plen, plen, n)
            for jw in (False, True):  # (the JUST_WRITTEN hint: column runs capture)
                got = _np(A.chksum_batch_strided(buf, plen, plen, n, byte_offset=9,
                                                 just_written=jw))
                assert np.array_equal(got, want), (plen, jw)
        lens = rng.integers(0, 3000, 5001)
        lens[rng.random(lens.size) < 0.1] = 0
        off = np.concatenate([[3], 3 + np.cumsum(lens)]).astype(np.int64)
        assert off[-1] <= buf.numel()
        got = _np(A.chksum_batch_csr(buf, _d(off), final=True))
        assert np.array_equal(got, oracle.batch_csr(hb, off.astype(np.uint64), final=True))
    finally:
        _tune("short_loads", -1)
        _tune("chunk_packets", 0)


@pytest.mark.parametrize("chunk", [1, 4, 16])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_short_runs_empty_chunks_at_buffer_end(oracle, mode, chunk):
    """A chunk of only empty packets starting on a 16-byte boundary is an empty run (no
    segment): it must issue no load. Here such chunks sit at the end of a 16-aligned buffer
    (ragged CSR batch, then 64 empty packets at offset == numel), in every short-run read form;
    the global-load form (short_loads 1) once clamped its windows to segment nseg - 1 there,
    which wrapped for nseg = 0."""
    _tune("short_loads", mode)
    _tune("chunk_packets", chunk)
    try:
        rng = np.random.default_rng(90 + mode + 10 * chunk)
        lens = rng.integers(0, 1600, 3000)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        size = (int(off[-1]) + 15) & ~15
        off = np.concatenate([off, np.full(64, size, dtype=np.int64)])
        off[-65] = size  # the last real packet runs to the aligned end
        buf = torch.empty(size, dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, 93)
        got = _np(A.chksum_batch_csr(buf, _d(off), final=True))
        want = oracle.batch_csr(_np(buf), off.astype(np.uint64), final=True)
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:8]
        assert np.all(got[-64:] == 0xFFFF)  # ~0: IpChksum of nothing
    finally:
        _tune("short_loads", -1)
        _tune("chunk_packets", 0)


def test_overlapping_and_zero_stride(oracle):
    buf = torch.empty(70000, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, 77)
    for stride, plen in ((1, 1500), (3, 65535), (0, 777), (2, 9000)):
        n = 200
        got = _np(A.chksum_batch_strided(buf, stride, plen, n))
        want = oracle.batch_strided(_np(buf), stride, plen, n)
        assert np.array_equal(got, want), (stride, plen)


@pytest.mark.parametrize("chunk", [1, 4, 8, 16])
def test_gapped_columns_overlapping_and_zero_strides(oracle, chunk):
    """Gapped column runs (strides that are multiples of 16) with strides below 16 x the
    packet's segments -- packets overlapping, the gap negative -- and stride 0 (every packet
    the same bytes), forced onto the column kernel with chunk_packets on a small batch
    (ADVICE round 5), at odd and even bases, against the oracle."""
    _tune("chunk_packets", chunk)
    try:
        buf = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)
        synth.fill_device(buf, 78 + chunk)
        hb = _np(buf)
        for stride, plen in ((16, 1500), (0, 777), (0, 1500), (32, 9000), (48, 100),
                             (1504, 1500), (16, 1), (64, 65535)):
            for base in (0, 5):
                n = 300
                if base + (n - 1) * stride + plen > buf.numel():
                    n = (buf.numel() - base - plen) // max(stride, 1) + 1
                got = _np(A.chksum_batch_strided(buf, stride, plen, n, byte_offset=base))
                want = oracle.batch_strided(hb[base:], stride, plen, n)
                assert np.array_equal(got, want), (stride, plen, base, np.nonzero(got != want)[0][:8])
    finally:
        _tune("chunk_packets", 0)


def test_just_written_hint_every_form(oracle, golden):
    """The AIPSTACK_CHKSUM_JUST_WRITTEN hint changes how a batch is read, never the
    result: gapped strided packets (A2K's form, odd and even starts), ring slots of mixed
    lengths (C2K's form) and chains (the reference fixtures' scatter chains), each against the
    same call without the hint and the oracle."""
    buf = torch.empty(1 << 22, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, 97)
    hb = _np(buf)
    for stride, plen, base in ((2048, 1500, 0), (2048, 1500, 7), (1504, 1500, 3), (64, 33, 1)):
        n = min(1500, (buf.numel() - base - plen) // stride + 1)
        want = oracle.batch_strided(hb[base:], stride, plen, n)
        for jw in (False, True):
            got = _np(A.chksum_batch_strided(buf, stride, plen, n, byte_offset=base,
                                             just_written=jw))
            assert np.array_equal(got, want), (stride, plen, base, jw)
    rng = np.random.default_rng(98)
    lens = rng.integers(0, 2049, 1500).astype(np.uint32)
    ring = torch.empty(1500 * 2048, dtype=torch.uint8, device=DEV)
    synth.fill_device(ring, 99)
    dl = _d(lens.view(np.int32))
    a = _np(A.chksum_batch_slotted(ring, 2048, dl))
    b = _np(A.chksum_batch_slotted(ring, 2048, dl, just_written=True))
    rh = _np(ring)
    want = np.array([oracle.inverted(rh, 2048 * i, int(lens[i])) for i in range(1500)],
                    dtype=np.uint16)
    assert np.array_equal(a, want) and np.array_equal(b, want)
    db = _d(golden["blob"])
    addr, ln, idx, st, want = _chain_tables(golden, db)
    args = (_d(addr.view(np.int64)), _d(ln.view(np.int32)), _d(idx.view(np.int64)),
            _d(st.view(np.int32)))
    got = _np(A.chksum_batch_chain(*args, final=True, just_written=True))
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def test_all_zero_and_all_ff_batches():
    for fill, want in ((0x00, 0x0000), (0xFF, 0xFFFF)):
        buf = torch.full((1500 * 4096,), fill, dtype=torch.uint8, device=DEV)
        got = _np(A.chksum_batch_strided(buf, 1500, 1500, 4096))
        assert np.all(got == want)
        got = _np(A.chksum_batch_strided(buf, 1500, 1499, 4096, byte_offset=1))
        assert np.all(got == (0x0000 if fill == 0 else 0xFF00))  # odd: + 0xFF00 tail


def test_csr_empty_and_long_packets(oracle):
    rng = np.random.default_rng(3)
    n = 50000
    lens = rng.choice([0, 0, 1, 2, 3, 64, 1500, 9000, 65535], size=n,
                      p=[.2, .05, .1, .1, .05, .2, .2, .08, .02])
    off = np.zeros(n + 1, dtype=np.int64)
    off[0] = 1
    np.cumsum(lens, out=off[1:])
    off[1:] += 1
    buf = torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, 5)
    got = _np(A.chksum_batch_csr(buf, _d(off)))
    want = oracle.batch_csr(_np(buf), off)
    assert np.array_equal(got, want)
    assert np.all(got[lens == 0] == 0)
    fin = _np(A.chksum_batch_csr(buf, _d(off), final=True))
    assert np.array_equal(fin, ~want)


def test_seeded_csr(oracle, golden):
    n = 100000
    off = synth.mixed_offsets(n, 11)
    buf = torch.empty(int(off[-1]), dtype=torch.uint8, device=DEV)
    synth.fill_device(buf, 12)
    rng = np.random.default_rng(4)
    states = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    states[::7] = 0xFFFFFFFF
    states[1::7] = 0
    got = _np(A.chksum_batch_seeded_csr(buf, _d(off), _d(states.view(np.int32))))
    want = oracle.batch_seeded_csr(_np(buf), off, states)
    assert np.array_equal(got, want)


def test_seeded_against_reference_accumulate_golden(golden):
    """IpChksumAccumulator header state (exported by the reference) + payload on the GPU."""
    b = golden["blob"]
    cases = golden["chain"]["accumulate"]
    db = _d(b)
    for c in cases:
        po, pl = c["payload"]
        off = _d(np.array([po, po + pl], dtype=np.int64))
        st = _d(np.array([c["state"]], dtype=np.uint32).view(np.int32))
        got = int(_np(A.chksum_batch_seeded_csr(db, off, st))[0])
        assert got == c["chksum"], c


def test_stream_ordering_user_stream(oracle):
    s = torch.cuda.Stream()
    n, plen = 20000, 1500
    buf = torch.empty(n * plen, dtype=torch.uint8, device=DEV)
    with torch.cuda.stream(s):
        synth.fill_device(buf, 31, stream=s)
        out = A.chksum_batch_strided(buf, plen, plen, n, stream=s)
    s.synchronize()
    assert np.array_equal(_np(out), oracle.batch_strided(_np(buf), plen, plen, n))


def test_cpp_capi_program():
    exe = os.path.join(ROOT, "tests", "cpp", "build", "gpu_capi_test")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp"), "gpu"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout


@pytest.mark.parametrize("build", ["engine_fault_test", "engine_fault_test_asan"])
def test_engine_fault_injection_program(build):
    """tests/cpp/engine_fault_test.cpp against an engine built with its test-only fault
    injection (plain and host-side ASan/UBSan builds): per-ticket failures with two failing
    batches in flight, a launch failure part-way, destroy completing a pending Tx fill,
    unregister completing the batches in flight, and _wait not blocking _poll."""
    exe = os.path.join(ROOT, "tests", "cpp", "build", build)
    assert os.path.exists(exe), f"{exe} not built (make -C tests/cpp gpu)"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[:3000] + r.stderr[-1500:]
    assert "OK" in r.stdout


def test_bench_two_ranks_one_gpu():
    """The multi-GPU bench path (one process per GPU, disjoint packet shards, gloo for the
    control plane only) rehearsed with 2 ranks on device 0 (AIPSTACK_BENCH_FORCE_DEVICE):
    torchrun launches bench.py --gpus 2 as the driver does; exactly one JSON line comes
    back, with n_gpus 2, rank 0's shard bit-exact and its CPU baseline present."""
    import json
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, AIPSTACK_BENCH_FORCE_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--steps", "5", "--warmup", "2", "--cpu-reps", "2"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["scaling"] == "weak"
    # every rank checked its own shard; the line says which device each rank ran on, and
    # that here (FORCE_DEVICE) both ranks shared one
    assert d["parity"].startswith("bit-exact (each of 2 rank(s)"), d["parity"]
    assert all(p.startswith("bit-exact") for p in d["per_gpu"]["parity"])
    assert len(d["per_gpu"]["devices"]) == 2 and d["per_gpu"]["arch"] == ["gfx950"] * 2 or \
        all(a.startswith("gfx950") for a in d["per_gpu"]["arch"])
    assert d["per_gpu"]["devices"][0] == d["per_gpu"]["devices"][1]
    assert d["per_gpu"]["distinct_devices"] is False and "note" in d["per_gpu"]
    cpu = d["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["cores"] == 1
    assert cpu["affinity_cores"] >= 1
    per = d["per_gpu"]  # every rank's own rate and kernel time
    assert len(per["GiB_s"]) == 2 and len(per["kernel_us"]) == 2
    assert min(per["GiB_s"]) > 0 and min(per["kernel_us"]) > 0


def test_bench_e2e_tx_two_ranks_one_gpu():
    """bench.py --e2e --config TX under torchrun with 2 ranks (each its own frame shard in
    host memory, filled in place through its engine): one JSON line, rank 0 bit-exact."""
    import json
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, AIPSTACK_BENCH_FORCE_DEVICE="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
           "--e2e", "--config", "TX", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["parity"].startswith("bit-exact (each of 2") and d["value"] > 0
    assert d["metric"].startswith("GiB/s Tx-filled end-to-end")
    assert d["per_gpu"]["distinct_devices"] is False


# ---- host-memory streaming engine ------------------------------------

@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("register", [False, True])
def test_engine_host_strided(oracle, register, zero_copy):
    n, plen = 300000, 1500
    host = synth.random_bytes(21, n * plen + 3)
    with _engine_copy_mode(zero_copy), A.ChksumEngine(0, chunk_bytes=16 << 20, nstreams=3) as eng:
        if register:
            eng.register(host)
        got = eng.strided(host[3:], plen, plen, n) if not register else \
            eng.strided(host, plen, plen, n)
        want = oracle.batch_strided(host, plen, plen, n, base_off=0 if register else 3)
        assert np.array_equal(got, want)
        fin = eng.strided(host, 1501, 1499, 1000, final=True)
        assert np.array_equal(fin, oracle.batch_strided(host, 1501, 1499, 1000, final=True))


@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("register", [False, True])
def test_engine_host_csr(oracle, register, zero_copy):
    buf, off = synth.mixed_batch(400000)
    with _engine_copy_mode(zero_copy), A.ChksumEngine(0, chunk_bytes=8 << 20, nstreams=2) as eng:
        if register:
            eng.register(buf)
        got = eng.csr(buf, off)
        assert np.array_equal(got, oracle.batch_csr(buf, off))


def test_engine_async_submit_poll_wait(oracle):
    """Non-blocking engine: several batches in flight at once (registered and pageable,
    strided and CSR), completed out of submission order by poll and wait; results as the
    synchronous calls give."""
    rng = np.random.default_rng(31)
    a = rng.integers(0, 256, size=300 * 1500, dtype=np.uint8)      # registered, strided
    b_buf, b_off = synth.mixed_batch(5000)                          # pageable, CSR
    c = rng.integers(0, 256, size=4000 * 9000, dtype=np.uint8)      # pageable, big strided
    with A.ChksumEngine(0, chunk_bytes=1 << 20, nstreams=3) as eng:
        eng.register(a)
        ta, oa = eng.submit_strided(a, 1500, 1500, 300)
        tb, ob = eng.submit_csr(b_buf, b_off, final=True)
        tc, oc = eng.submit_strided(c, 9000, 9000, 4000)
        assert len({ta, tb, tc}) == 3
        # the caller is free meanwhile; complete the last one first
        eng.wait(tc)
        spins = 0
        while not eng.poll(tb):
            spins += 1
            assert spins < 10_000_000
        eng.wait(ta)
        assert eng.poll(ta)  # already complete: stays complete
        assert np.array_equal(oa, oracle.batch_strided(a, 1500, 1500, 300))
        assert np.array_equal(ob, oracle.batch_csr(b_buf, b_off, final=True))
        assert np.array_equal(oc, oracle.batch_strided(c, 9000, 9000, 4000))
        with pytest.raises(A.ChksumError):
            eng.wait(10**9)  # never issued


def test_engine_async_frames_in_flight(oracle):
    """Tx fill, Rx verify and a CSR checksum batch in flight together over small pieces
    (1 MiB), completed out of order; the Tx batch's offsets are a temporary the engine's
    completion still reads (kept alive by the wrapper)."""
    tx_buf, tx_off = synth.frames_host(20000, seed=51)
    _corrupt(tx_buf, tx_off, 0.1, 52)
    want_tx = tx_buf.copy()
    want_st = oracle.tx_fill_batch(want_tx, tx_off)
    rx_buf, rx_off = synth.frames_host(15000, seed=53)
    oracle.tx_fill_batch(rx_buf, rx_off)
    _corrupt(rx_buf, rx_off, 0.3, 54)
    want_rx = oracle.rx_verify_batch(rx_buf, rx_off)
    b_buf, b_off = synth.mixed_batch(7000)
    with A.ChksumEngine(0, chunk_bytes=1 << 20, nstreams=2) as eng:
        eng.register(rx_buf)
        tt, st = eng.submit_tx_fill(tx_buf, [int(x) for x in tx_off])
        tr, vr = eng.submit_rx_verify(rx_buf, rx_off)
        tb, ob = eng.submit_csr(b_buf, b_off)
        eng.wait(tb)
        eng.wait(tt)
        while not eng.poll(tr):
            pass
        assert np.array_equal(st, want_st) and np.array_equal(tx_buf, want_tx)
        assert np.array_equal(vr, want_rx)
        assert np.array_equal(ob, oracle.batch_csr(b_buf, b_off))


@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("register", [False, True])
def test_engine_host_rx_verify(oracle, register, zero_copy):
    """Raw frames in host memory (the TAP receive path batched): verdicts as the device
    batch and the frame oracle give, over several engine chunks; also through submit/wait."""
    buf, off = synth.frames_host(60000, seed=41)
    oracle.tx_fill_batch(buf, off)
    _corrupt(buf, off, 0.2, 3)
    want = oracle.rx_verify_batch(buf, off)
    with _engine_copy_mode(zero_copy), A.ChksumEngine(0, chunk_bytes=4 << 20, nstreams=3) as eng:
        if register:
            eng.register(buf)
        got = eng.rx_verify(buf, off)
        assert got.dtype == np.uint8 and np.array_equal(got, want)
        t, out = eng.submit_rx_verify(buf, off)
        eng.wait(t)
        assert np.array_equal(out, want)
        with pytest.raises(A.ChksumError):
            eng.rx_verify(buf, np.array([0, 100, 50], dtype=np.uint64))


@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("register", [False, True])
def test_engine_host_tx_fill(oracle, register, zero_copy):
    """Raw frames in host memory (the TAP send path batched), filled IN PLACE: frames and
    statuses byte-identical to the frame oracle's, over several engine chunks; also through
    submit/wait, on frames whose fields hold garbage."""
    buf, off = synth.frames_host(60000, seed=43)
    _corrupt(buf, off, 0.2, 5)  # garbage in the fields, and some frames not fillable
    orig = buf.copy()
    want = buf.copy()
    want_st = oracle.tx_fill_batch(want, off)
    assert len(set(want_st.tolist())) > 1
    with _engine_copy_mode(zero_copy), A.ChksumEngine(0, chunk_bytes=4 << 20, nstreams=3) as eng:
        if register:
            eng.register(buf)
        st = eng.tx_fill(buf, off)
        assert st.dtype == np.uint8 and np.array_equal(st, want_st)
        assert np.array_equal(buf, want)
        buf[:] = orig
        t, st2 = eng.submit_tx_fill(buf, off)
        eng.wait(t)
        assert np.array_equal(st2, want_st) and np.array_equal(buf, want)
        with pytest.raises(A.ChksumError):
            eng.tx_fill(buf, np.array([0, 100, 50], dtype=np.uint64))


def test_engine_rejects_bad_offsets():
    buf = np.zeros(1 << 20, dtype=np.uint8)
    with A.ChksumEngine(0) as eng:
        with pytest.raises(A.ChksumError):
            eng.csr(buf, np.array([0, 100, 50], dtype=np.uint64))
        with pytest.raises(A.ChksumError):
            eng.csr(buf, np.array([0, 70000], dtype=np.uint64))
        assert eng.csr(buf, np.array([0], dtype=np.uint64)).size == 0
        # int64 offsets / int32 lengths are passed to the C-ABI as views (no copy): a
        # negative entry becomes a huge unsigned value, which the engine rejects
        with pytest.raises((A.ChksumError, ValueError)):
            eng.csr(buf, np.array([0, -100, 200], dtype=np.int64))
        with pytest.raises((A.ChksumError, ValueError)):
            eng.rx_verify(buf, np.array([-64, 0], dtype=np.int64))
        with pytest.raises(A.ChksumError):
            eng.slotted(buf[:2048 * 4], 2048, np.array([60, -1, 60, 60], dtype=np.int32))
        good = np.array([0, 100, 1500], dtype=np.int64)
        assert np.array_equal(eng.csr(buf, good), eng.csr(buf, good.astype(np.uint64)))


# ---- chained scatter-gather batches ---------------------------------

def _chain_tables(golden, db):
    from conftest import chain_to_chunks
    addrs, lens, index, states, want = [], [], [0], [], []
    base = db.data_ptr()
    for c in golden["chain"]["chains"]:
        for o, l in chain_to_chunks(c):
            addrs.append(base + o)
            lens.append(l)
        index.append(len(addrs))
        states.append(c["state"])
        want.append(c["chksum"])
    return (np.array(addrs, dtype=np.uint64), np.array(lens, dtype=np.uint32),
            np.array(index, dtype=np.uint64), np.array(states, dtype=np.uint32),
            np.array(want, dtype=np.uint16))


@pytest.fixture
def chain_short():
    """Setter for the chain_short tunable (chunks of at most this many bytes that share no
    line with their table neighbours first in each group's gathered stream; 0 = table
    order); restores the default (-1: 128) afterwards."""
    yield lambda v: _tune("chain_short", v)
    _tune("chain_short", -1)


@pytest.mark.parametrize("short", [0, 128, 65535])
@pytest.mark.parametrize("su", [0, -1])
def test_chain_golden_reference_cases(golden, stream_mode, chain_short, su, short):
    """All 3,609 reference chain cases (the 512-node 0x00FF KAT, the chain==flat splits,
    scatter chains with states/offsets/tot_len) in ONE GPU batch; with and without the
    stream runs over chunks that lie close together; chunks in table order, short ones
    apart from their neighbours' lines first (the default) and every chunk counted short."""
    stream_mode(su)
    chain_short(short)
    db = _d(golden["blob"])
    addr, ln, idx, st, want = _chain_tables(golden, db)
    got = _np(A.chksum_batch_chain(_d(addr.view(np.int64)), _d(ln.view(np.int32)),
                                   _d(idx.view(np.int64)), _d(st.view(np.int32)), final=True))
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    inv = _np(A.chksum_batch_chain(_d(addr.view(np.int64)), _d(ln.view(np.int32)),
                                   _d(idx.view(np.int64)), _d(st.view(np.int32))))
    assert np.array_equal(inv, ~want)


def test_contract_violations_chain_chunk_over_65535(oracle):
    """A chain chunk longer than 65535 bytes (outside the contract, chksum.h): no load leaves
    the chunks, the chunk is summed as empty (its chain gives the checksum of the others)
    and the sticky CHUNK_LEN bit reports it; in-contract batches set no bit."""
    rng = np.random.default_rng(77)
    host = rng.integers(0, 256, size=300000, dtype=np.uint8)
    db = _d(host)
    base = db.data_ptr()
    A.contract_violations(0, clear=True)
    # chain 0: 3 small chunks; chain 1: small + 70000 B + small; chain 2: 65535 B (legal)
    chunks = [(0, 100), (1000, 33), (2001, 1460),
              (5000, 77), (10000, 70000), (90001, 301),
              (100000, 65535)]
    idx = np.array([0, 3, 6, 7], dtype=np.uint64)
    addr = np.array([base + o for o, _ in chunks], dtype=np.uint64)
    ln = np.array([l for _, l in chunks], dtype=np.uint32)
    st = np.array([0x1234, 0xFFFFFFFF, 7], dtype=np.uint32)
    got = _np(A.chksum_batch_chain(_d(addr.view(np.int64)), _d(ln.view(np.int32)),
                                   _d(idx.view(np.int64)), _d(st.view(np.int32)), final=True))
    want = [oracle.chain(0x1234, host, chunks[0:3]),
            oracle.chain(0xFFFFFFFF, host, [chunks[3], chunks[5]]),  # the long chunk: empty
            oracle.chain(7, host, chunks[6:7])]
    assert got.tolist() == want
    assert A.contract_violations(0, clear=True) == A.VIOLATION_CHUNK_LEN
    assert A.contract_violations(0) == 0
    ok_idx = np.array([0, 3], dtype=np.uint64)
    A.chksum_batch_chain(_d(addr.view(np.int64)), _d(ln.view(np.int32)),
                         _d(ok_idx.view(np.int64)), None, final=True)
    assert A.contract_violations(0) == 0


def test_contract_violations_csr_and_frames(oracle):
    """CSR packets over 65535 bytes (up to 2^26 still summed exactly) and decreasing offsets
    set PACKET_LEN, without faulting; so do over-long frames in Rx verify."""
    host = np.random.default_rng(78).integers(0, 256, size=1 << 20, dtype=np.uint8)
    db = _d(host)
    A.contract_violations(0, clear=True)
    off = np.array([0, 100, 100 + 70000, 100 + 70000 + 1500], dtype=np.uint64)
    got = _np(A.chksum_batch_csr(db, _d(off.view(np.int64))))
    assert got.tolist() == [oracle.inverted(host, int(off[i]), int(off[i + 1] - off[i]))
                            for i in range(3)]
    assert A.contract_violations(0, clear=True) == A.VIOLATION_PACKET_LEN
    dec = np.array([5000, 4000, 6000], dtype=np.uint64)  # packet 0 ends before it starts
    got = _np(A.chksum_batch_csr(db, _d(dec.view(np.int64))))
    assert got[1] == oracle.inverted(host, 4000, 2000)
    assert A.contract_violations(0, clear=True) == A.VIOLATION_PACKET_LEN
    frames, foff = synth.frames_host(100, seed=3)
    big = np.concatenate([frames, host[:80000]])
    foff2 = np.concatenate([foff, [foff[-1] + 80000]]).astype(np.uint64)
    v = _np(A.rx_verify(_d(big), _d(foff2.view(np.int64))))
    assert v[-1] == 0 and np.array_equal(v[:-1], oracle.rx_verify_batch(frames, foff))
    assert A.contract_violations(0, clear=True) & A.VIOLATION_PACKET_LEN
    A.chksum_batch_csr(db, _d(np.array([0, 1500, 3000], dtype=np.int64)))
    assert A.contract_violations(0) == 0


def test_chain_flatten_and_null_states(oracle):
    """Python IpBufRef chains -> flatten_chains -> GPU, vs the host accumulator mirror."""
    rng = np.random.default_rng(8)
    host = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    db = _d(host)
    refs, want = [], []
    for _ in range(5000):
        nodes = None
        for _ in range(int(rng.integers(1, 6))):
            o = int(rng.integers(0, host.size - 2000))
            l = int(rng.choice([0, 1, 2, 3, int(rng.integers(0, 1600))]))
            nodes = A.IpBufNode(host[o:o + l], l, nodes)
        total, nd = 0, nodes
        while nd is not None:
            total += nd.len
            nd = nd.next
        off = int(rng.integers(0, nodes.len + 1))
        ref = A.IpBufRef(nodes, off, total - off)
        refs.append(ref)
        want.append(A.IpChksumAccumulator().getChksum(ref))
    addr, ln, idx = A.flatten_chains(refs, host, db.data_ptr())
    got = _np(A.chksum_batch_chain(_d(addr.view(np.int64)), _d(ln.view(np.int32)),
                                   _d(idx.view(np.int64)), None, final=True))
    assert np.array_equal(got, np.array(want, dtype=np.uint16))


@pytest.mark.parametrize("short", [0, 128])
@pytest.mark.parametrize("su", [0, -1])
def test_chain_tcp_tx_shape(oracle, stream_mode, chain_short, su, short):
    """TCP Tx shape (tcp/IpTcpProto_output.h:1251-1277): pseudo-header state + header node
    + up to 2 send-ring chunks (utils/TcpRingBufferUtils.h:51), 100k segments."""
    stream_mode(su)
    chain_short(short)
    rng = np.random.default_rng(9)
    ring = rng.integers(0, 256, size=1 << 22, dtype=np.uint8)
    hdrs = rng.integers(0, 256, size=100000 * 60, dtype=np.uint8)
    dring, dh = _d(ring), _d(hdrs)
    addrs, lens, idx, states, want = [], [], [0], [], []
    for i in range(100000):
        hl = 20 + 4 * int(rng.integers(0, 11))
        chunks = [(dh.data_ptr() + 60 * i, hl, hdrs[60 * i:60 * i + hl])]
        seg = int(rng.integers(0, 1461))
        start = int(rng.integers(0, ring.size))
        first = min(seg, ring.size - start)
        chunks.append((dring.data_ptr() + start, first, ring[start:start + first]))
        if seg > first:
            chunks.append((dring.data_ptr(), seg - first, ring[:seg - first]))
        st = int(rng.integers(0, 2**20))
        acc = A.IpChksumAccumulator(st)
        nodes = None
        for _, l, h in reversed(chunks):
            nodes = A.IpBufNode(h, l, nodes)
        want.append(acc.getChksum(A.IpBufRef(nodes, 0, sum(c[1] for c in chunks))))
        for a, l, _ in chunks:
            if l:
                addrs.append(a)
                lens.append(l)
        idx.append(len(addrs))
        states.append(st)
    got = _np(A.chksum_batch_chain(_d(np.array(addrs, dtype=np.int64)),
                                   _d(np.array(lens, dtype=np.int32)),
                                   _d(np.array(idx, dtype=np.int64)),
                                   _d(np.array(states, dtype=np.int32)), final=True))
    assert np.array_equal(got, np.array(want, dtype=np.uint16))


@pytest.mark.parametrize("short", [0, 128])
@pytest.mark.parametrize("su", [2, 4, 8, -1])
def test_chain_bench_shape(su, stream_mode, chain_short, short):
    """bench.py's CHAIN layout (20-B header nodes at a 32-B stride + a contiguous payload ring
    split in two chunks per chain): header and payload chunks each stream as one run."""
    stream_mode(su)
    chain_short(short)
    sys.path.insert(0, ROOT)
    import bench
    spec = {"n": 50000, "seed": 77}
    ch = bench.make_chains(spec, torch.device(DEV))
    out = _np(A.chksum_batch_chain(ch["addr"], ch["len"], ch["index"], ch["states"],
                                   final=True))
    assert bench.chain_check(ch, out).startswith("bit-exact")


def _chain_batch(chains, addr_of):
    """chains: list of (state, [(buffer id, offset, length), ...]); addr_of(buffer id, offset)
    gives the device address. Returns the chunk table as device tensors."""
    addrs, lens, idx, states = [], [], [0], []
    for st, chunks in chains:
        for b, o, l in chunks:
            if l:
                addrs.append(addr_of(b, o))
                lens.append(l)
        idx.append(len(addrs))
        states.append(st)
    return (_d(np.array(addrs, dtype=np.uint64).view(np.int64)),
            _d(np.array(lens, dtype=np.uint32).view(np.int32)),
            _d(np.array(idx, dtype=np.uint64).view(np.int64)),
            _d(np.array(states, dtype=np.uint32).view(np.int32)))


def test_chain_many_chunks_exact(oracle):
    """Chains of 70,000 one-byte and two-byte 0xFF chunks (the per-chain sum of chunk sums
    passes 2^32 in a 32-bit accumulator) and a 200,000-chunk mixed chain, next to short
    ones, against the oracle's chain rule (Chksum.h:283-315: end-around carry per chunk)."""
    rng = np.random.default_rng(70000)
    host = rng.integers(0, 256, size=1 << 20, dtype=np.uint8)
    host[:4096] = 0xFF
    db = _d(host)
    chains = [
        (0, [(0, int(rng.integers(0, 4000)), 1) for _ in range(70000)]),
        (0xFFFFFFFF, [(0, int(rng.integers(0, 4000)), 2) for _ in range(70000)]),
        (0x12345, [(0, 7, 3)]),
        (int(rng.integers(0, 2**32)),
         [(0, int(rng.integers(0, (1 << 20) - 1600)), int(rng.choice([0, 1, 2, 3, 1459])))
          for _ in range(200000)]),
        (0, []),
        (0, [(0, 1, 1)] * 65537),
    ]
    addr, ln, idx, st = _chain_batch(chains, lambda b, o: db.data_ptr() + o)
    got = _np(A.chksum_batch_chain(addr, ln, idx, st, final=True))
    # oracle.chain = IpChksumAccumulator(State).getChksum(chain) (the final form)
    want = np.array([oracle.chain(s, host, [(o, l) for _, o, l in ch if l]) for s, ch in chains],
                    dtype=np.uint16)
    assert np.array_equal(got, want), (got, want)


def test_chain_chunks_in_separate_allocations(oracle):
    """Chunks spread over separately allocated device buffers and pinned host memory: only
    the chunks' own 16-byte segments may be read (the address space between allocations
    can be unmapped; a read there faults the GPU)."""
    rng = np.random.default_rng(4242)
    hosts = [rng.integers(0, 256, size=int(sz), dtype=np.uint8)
             for sz in (4096, 100000, 33, 65536 + 17, 5000)]
    devs = [_d(h) for h in hosts[:4]]
    pinned = torch.from_numpy(hosts[4]).pin_memory()  # device-accessible host memory
    ptrs = [t.data_ptr() for t in devs] + [pinned.data_ptr()]
    chains = []
    for i in range(3000):
        chunks = []
        for _ in range(int(rng.integers(1, 6))):
            b = int(rng.integers(0, len(hosts)))
            sz = hosts[b].size
            l = int(rng.integers(0, min(sz, 1600) + 1))
            if rng.random() < 0.2:
                o = sz - l          # ends at the allocation's last byte
            elif rng.random() < 0.2:
                o = 0               # starts at its first byte
            else:
                o = int(rng.integers(0, sz - l + 1))
            chunks.append((b, o, l))
        chains.append((int(rng.integers(0, 2**32)), chunks))
    addr, ln, idx, st = _chain_batch(chains, lambda b, o: ptrs[b] + o)
    got = _np(A.chksum_batch_chain(addr, ln, idx, st, final=True))
    torch.cuda.synchronize()
    want = []
    for state, chunks in chains:
        flat = np.concatenate([hosts[b][o:o + l] for b, o, l in chunks] + [np.zeros(0, np.uint8)])
        # chain == flat with the state seeded (reference property, tests/ip_chksum_test.cpp)
        want.append(oracle.chain(state, flat, [(0, flat.size)] if flat.size else []))
    assert np.array_equal(got, np.array(want, dtype=np.uint16))


def test_chain_back_to_back_pieces_every_form(oracle):
    """Chains whose payload pieces are cut back to back from one buffer -- the layout the
    JUST_WRITTEN chain kernel reads as column runs -- at its limits: 64 KiB - 1
    pieces (runs of 32 of them, 2 MiB), slices of 64 run chunks and no header nodes, header
    nodes in an area of their own, the first piece at its allocation's first byte and the last
    ending at its last byte, in device and in pinned host memory. Both kernels (with and
    without the hint) against the oracle."""
    rng = np.random.default_rng(7070)

    def layout(n, hdr, piece_len):
        # (state, [(0, offset, length), ...]) with headers (if any) first in the blob
        hbytes = 32 * n if hdr else 0
        chains, p = [], hbytes
        for i in range(n):
            ch = [(0, 32 * i, hdr)] if hdr else []
            for ln in piece_len(i):
                ch.append((0, p, ln))
                p += ln
            chains.append((int(rng.integers(0, 2**32)), ch))
        return chains, p

    cases = [
        layout(40, 20, lambda i: [65535, 65535]),
        layout(300, 0, lambda i: [int(rng.integers(1, 3001))]),
        layout(500, 20, lambda i: [int(x) for x in rng.integers(1, 2000, int(rng.integers(0, 4)))]),
        layout(200, int(rng.integers(1, 33)), lambda i: [int(rng.integers(1, 129)), 1460]),
    ]
    for k, (chains, size) in enumerate(cases):
        host = rng.integers(0, 256, size=size, dtype=np.uint8)
        for where in ("device", "pinned"):
            t = _d(host) if where == "device" else torch.from_numpy(host).pin_memory()
            addr, ln, idx, st = _chain_batch(chains, lambda b, o: t.data_ptr() + o)
            want = np.array([oracle.chain(s, host, [(o, l) for _, o, l in ch if l])
                             for s, ch in chains], dtype=np.uint16)
            for jw in (False, True):
                got = _np(A.chksum_batch_chain(addr, ln, idx, st, final=True, just_written=jw))
                assert np.array_equal(got, want), (k, where, jw, np.nonzero(got != want)[0][:8])
            torch.cuda.synchronize()


# ---- frame-level batches: Tx fill / Rx verify ----------------------

def _corrupt(buf, off, frac, seed):
    """Flip one random byte in a fraction of frames (header or payload)."""
    rng = np.random.default_rng(seed)
    n = off.size - 1
    for i in np.nonzero(rng.random(n) < frac)[0]:
        s, e = int(off[i]), int(off[i + 1])
        j = s + int(rng.integers(12, e - s))
        buf[j] ^= np.uint8(1 << int(rng.integers(0, 8)))


@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("su", [0, -1])
@pytest.mark.parametrize("n,maxp", [(200000, 1460), (20000, 9000)])
def test_tx_fill_matches_oracle(oracle, stream_mode, n, maxp, su, split):
    stream_mode(su)
    buf, off = synth.frames_host(n, seed=11, max_payload=maxp)
    dbuf, doff = _d(buf), _d(off)
    st = _np(A.tx_fill(dbuf, doff, split=split))
    want_buf = buf.copy()
    want_st = oracle.tx_fill_batch(want_buf, off)
    assert np.array_equal(st, want_st)
    got_buf = _np(dbuf)
    bad = np.nonzero(got_buf != want_buf)[0]
    assert bad.size == 0, bad[:10]


@pytest.mark.parametrize("su", [0, -1])
@pytest.mark.parametrize("n,maxp", [(200000, 1460), (20000, 9000)])
def test_rx_verify_matches_oracle(oracle, stream_mode, n, maxp, su):
    stream_mode(su)
    buf, off = synth.frames_host(n, seed=12, max_payload=maxp)
    oracle.tx_fill_batch(buf, off)                 # valid frames ...
    rng = np.random.default_rng(1)
    for i in np.nonzero(rng.random(n) < 0.05)[0]:  # ... some UDP without checksum ...
        s = int(off[i])
        if buf[s + 12] == 8 and buf[s + 13] == 0 and buf[s + 23] == 17:
            hl = int(buf[s + 14] & 15) * 4
            buf[s + 14 + hl + 6: s + 14 + hl + 8] = 0
    _corrupt(buf, off, 0.15, 2)                    # ... and 15 % with one flipped bit
    got = _np(A.rx_verify(_d(buf), _d(off)))
    want = oracle.rx_verify_batch(buf, off)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    kinds = set(np.unique(want).tolist())
    assert {0, 2, 3, 5, 6, 7, 8} <= kinds          # the verdicts this mix must reach


@pytest.fixture
def tx_gather():
    """Setter for the tx_gather tunable (0 per-lane header loads, 1 headers captured from
    the stream, -1 automatic); restores automatic afterwards."""
    yield lambda v: _tune("tx_gather", v)
    _tune("tx_gather", -1)


@pytest.mark.parametrize("gather", [-1, 0, 1])
@pytest.mark.parametrize("su", [0, -1])
@pytest.mark.parametrize("n,maxp", [(200000, 1460), (20000, 9000), (4097, 1460)])
def test_tx_fill_records_matches_oracle(oracle, stream_mode, tx_gather, n, maxp, su, gather):
    """The records-only read pass (aipstack_chksum_tx_fill_records, the E2E Tx kernel): the
    frames stay untouched, and the records applied on the host give the oracle's fill and
    statuses -- with its default header capture and with per-lane header loads."""
    stream_mode(su)
    tx_gather(gather)
    buf, off = synth.frames_host(n, seed=21 + n, max_payload=maxp)
    dbuf, doff = _d(buf), _d(off)
    rec = _np(A.tx_fill_records(dbuf, doff))
    assert np.array_equal(_np(dbuf), buf)
    got = buf.copy()
    st = A.apply_tx_records(got, off, rec)
    want = buf.copy()
    want_st = oracle.tx_fill_batch(want, off)
    assert np.array_equal(st, want_st)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


@pytest.mark.parametrize("shift", [0, 5])
def test_tx_fill_records_edge_frames(oracle, shift):
    buf, off = _edge_frames(31 + shift, 3000)
    big = np.zeros(buf.size + shift, dtype=np.uint8)
    big[shift:] = buf
    rec = _np(A.tx_fill_records(_d(big), _d(off + np.uint64(shift))))
    got = buf.copy()
    st = A.apply_tx_records(got, off, rec)
    want = buf.copy()
    want_st = oracle.tx_fill_batch(want, off)
    assert np.array_equal(st, want_st)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


@pytest.mark.parametrize("split", [False, True])
def test_tx_fill_with_captured_headers(oracle, tx_gather, split):
    """In-place fills forced onto the header-capture path (tx_gather = 1): same bytes."""
    tx_gather(1)
    for seed, (n, maxp) in enumerate([(200000, 1460), (3000, 9000)]):
        buf, off = synth.frames_host(n, seed=40 + seed, max_payload=maxp)
        dbuf, doff = _d(buf), _d(off)
        st = _np(A.tx_fill(dbuf, doff, split=split))
        want = buf.copy()
        want_st = oracle.tx_fill_batch(want, off)
        assert np.array_equal(st, want_st) and np.array_equal(_np(dbuf), want)


def test_tx_fill_split_workspace_and_ragged_counts(oracle):
    """Split Tx fill with a caller workspace (reused across calls, larger than needed, at
    an 8-byte-aligned offset of a bigger tensor) at ragged frame counts; idempotent."""
    import torch
    ws = torch.empty(8 * 5000 + 64, dtype=torch.uint8, device="cuda")
    for n in (1, 63, 64, 65, 4097):
        buf, off = synth.frames_host(n, seed=100 + n)
        dbuf, doff = _d(buf), _d(off)
        st = _np(A.tx_fill(dbuf, doff, workspace=ws[8:], split=True))
        want = buf.copy()
        want_st = oracle.tx_fill_batch(want, off)
        assert np.array_equal(st, want_st)
        assert np.array_equal(_np(dbuf), want)
        st2 = _np(A.tx_fill(dbuf, doff, workspace=ws[8:], split=True))  # fill is idempotent
        assert np.array_equal(st2, want_st) and np.array_equal(_np(dbuf), want)
    with pytest.raises(A.ChksumError):
        A.tx_fill(dbuf, doff, workspace=ws[: 8 * n - 8], split=True)


@pytest.mark.parametrize("raw_handle", [False, True])
def test_tx_fill_split_on_a_non_current_stream(oracle, raw_handle):
    """The split fill's temporary workspace stays reserved for the launch stream when that
    is not torch's current stream (a torch Stream, or a raw hipStream_t handle): torch's
    allocator may not reuse it while the passes run. Allocations on the current stream
    meanwhile must not disturb the result."""
    import torch
    s = torch.cuda.Stream()
    buf, off = synth.frames_host(50000, seed=17)
    dbuf, doff = _d(buf), _d(off)
    torch.cuda.synchronize()
    st = A.tx_fill(dbuf, doff, stream=s.cuda_stream if raw_handle else s, split=True)
    junk = [torch.full((8 * 50000,), 0xAB, dtype=torch.uint8, device=DEV) for _ in range(4)]
    s.synchronize()
    torch.cuda.synchronize()
    want = buf.copy()
    want_st = oracle.tx_fill_batch(want, off)
    assert np.array_equal(_np(st), want_st)
    assert np.array_equal(_np(dbuf), want)
    del junk


def test_fill_then_verify_on_gpu():
    buf, off = synth.frames_host(100000, seed=13)
    dbuf, doff = _d(buf), _d(off)
    st = _np(A.tx_fill(dbuf, doff))
    v = _np(A.rx_verify(dbuf, doff))
    assert np.array_equal(st, v)
    assert set(np.unique(v).tolist()) <= {0, 3, 6, 8}


def _capture_group_crossings(off, shift, cpk=32, U=4):
    """Frames whose captured header segments span windows of two different groups of U
    windows in the frames' double-buffered stream (frame_kernels.hip, HeaderCapture: the
    masks of windows w and w + U share mk[w & (U - 1)]). Chunks of cpk frames; the batch
    starts `shift` bytes past a 16-aligned address; kHdrNeed = 97."""
    n = off.size - 1
    count = 0
    for c0 in range(0, n, cpk):
        S = off[c0:min(c0 + cpk, n)].astype(np.int64) + shift
        base = int(S[0]) & ~15
        a0_32 = S & 16
        hb_end = ((a0_32 + (S & 15) + 97 + 31) & ~31) - a0_32
        r0 = ((S & ~15) - base) >> 4
        r1 = r0 + (hb_end >> 4)
        count += int(np.count_nonzero((r0 >> 6) // U != ((r1 - 1) >> 6) // U))
    return count


@pytest.mark.parametrize("maxp", [0, 120, 600, 1460])
def test_frames_header_capture_across_groups(oracle, maxp):
    """the frames' header capture (an exec-setting inline-asm LDS
    store per window) driven through frames whose header segments span the last window of
    one group and the first of the next, in the double-buffered loop, at every byte shift 0-15
    and ragged chunk edges: Rx verdicts, Tx records and the in-place fill against the oracle.
    The test counts those frames and requires some (the case is exercised, not just random)."""
    crossings = 0
    for shift in range(16):
        buf, off = synth.frames_host(2049, seed=7000 + 16 * maxp + shift, max_payload=maxp)
        oracle.tx_fill_batch(buf, off)       # valid frames, then one flipped bit in 10 %
        _corrupt(buf, off, 0.10, shift)
        big = np.zeros(buf.size + shift + 16, dtype=np.uint8)
        big[shift:shift + buf.size] = buf
        dbig = _d(big)
        assert dbig.data_ptr() % 16 == 0
        doff = _d((off + shift).astype(off.dtype))
        crossings += _capture_group_crossings(off, shift)
        got = _np(A.rx_verify(dbig, doff))
        assert np.array_equal(got, oracle.rx_verify_batch(buf, off)), (shift, maxp)
        rec = _np(A.tx_fill_records(dbig, doff))
        filled = buf.copy()
        st = A.apply_tx_records(filled, off, rec)
        want = buf.copy()
        want_st = oracle.tx_fill_batch(want, off)
        assert np.array_equal(st, want_st) and np.array_equal(filled, want), (shift, maxp)
        st2 = _np(A.tx_fill(dbig, doff))
        assert np.array_equal(st2, want_st), (shift, maxp)
        assert np.array_equal(_np(dbig)[shift:shift + buf.size], want), (shift, maxp)
    if maxp >= 600:  # (chunks of 32 short frames stay inside one group of 4 KiB)
        assert crossings > 100, crossings


def _edge_frames(seed, n):
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import frame_cases
    return frame_cases.pack(frame_cases.frames(seed, n))


@pytest.mark.parametrize("su", [0, 2, -1])
@pytest.mark.parametrize("shift", [0, 1, 7, 13])
def test_rx_verify_edge_frames(oracle, stream_mode, shift, su):
    """tests/golden/frame_cases.py: every verdict, IPv4 options, padding, zero-sum L4 data,
    one mutation in 40 % of frames; the whole batch starts `shift` bytes into a buffer."""
    stream_mode(su)
    buf, off = _edge_frames(20251015 + shift, 3000)
    big = np.zeros(buf.size + shift, dtype=np.uint8)
    big[shift:] = buf
    got = _np(A.rx_verify(_d(big), _d(off + np.uint64(shift))))
    want = oracle.rx_verify_batch(buf, off)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    assert np.all(np.bincount(want, minlength=9) > 0)


@pytest.fixture
def tx_store():
    """Setter for the tx_store tunable (0 = 2-byte field stores, 1 = whole sectors, -1 =
    the default); restores the default afterwards."""
    yield lambda v: _tune("tx_store", v)
    _tune("tx_store", -1)


@pytest.mark.parametrize("store", [0, 1])
@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("su", [0, 2, -1])
@pytest.mark.parametrize("shift", [0, 3])
def test_tx_fill_edge_frames(oracle, stream_mode, tx_store, shift, su, split, store):
    stream_mode(su)
    tx_store(store)
    buf, off = _edge_frames(7 + shift, 3000)
    big = np.zeros(buf.size + shift, dtype=np.uint8)
    big[shift:] = buf
    dbig = _d(big)
    st = _np(A.tx_fill(dbig, _d(off + np.uint64(shift)), split=split))
    want = buf.copy()
    want_st = oracle.tx_fill_batch(want, off)
    assert np.array_equal(st, want_st)
    got = _np(dbig)[shift:]
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


# ---- ring slots: one packet / frame per fixed slot, a length per slot ---------------------

@pytest.mark.parametrize("su", [0, 4, -1])
@pytest.mark.parametrize("stride", [64, 1517, 2048, 9216, 65536])
def test_slotted_checksums(oracle, stream_mode, stride, su):
    """aipstack_chksum_batch_slotted: lengths 0..min(stride, 65535) at every slot alignment
    an odd stride gives, slack bytes random; inverted and FINAL; the gathered stream (2 or 4
    windows) and the per-packet wave mode (su = -1)."""
    stream_mode(su)
    rng = np.random.default_rng(stride)
    n = {64: 50000, 1517: 20000, 2048: 20000, 9216: 3000, 65536: 300}[stride]
    cap = min(stride, 65535)
    lens = rng.integers(0, cap + 1, n).astype(np.uint32)
    lens[:8] = [0, 1, 2, cap, cap - 1, 15, 16, 17][:8] if cap > 17 else lens[:8]
    ring = synth.random_bytes(stride + 7, n * stride + 16)
    for base in (0, 3):
        view = ring[base:base + n * stride]
        dring = _d(ring)
        got = _np(A.chksum_batch_slotted(dring[base:base + n * stride], stride,
                                         _d(lens.view(np.int32))))
        assert np.array_equal(got, oracle.batch_slotted(np.ascontiguousarray(view), stride, lens))
    fin = _np(A.chksum_batch_slotted(_d(ring[:n * stride]), stride, _d(lens.view(np.int32)),
                                     final=True))
    assert np.array_equal(fin, oracle.batch_slotted(ring[:n * stride], stride, lens, final=True))


@pytest.mark.parametrize("chunk", [0, 8, 16, 64])
def test_gathered_stream_chunk_edges(oracle, chunk):
    """The gathered stream on ring slots at the edges of its chunks: 16-slot chunks whose
    streams hold 1023, 1024 and 1025 segments, a multiple of 64 plus one, empty slots at a
    chunk's end (the last prefix is the stream's total) and in its middle, one segment per
    slot, and 2000-byte slots; in 8-, 16- and 64-slot chunks, slots starting at 0, 5 and 15
    within a segment."""
    stride = 2048
    rows = [
        [1024] * 16,                       # T = 1024
        [1024] * 15 + [1040],              # T = 1025
        [1023] * 16,                       # T = 1024 with a partial last segment per slot
        [1024] * 15 + [1008],              # T = 1023
        [16 * 61 + 1] + [1024] * 15,       # T = 1024, first slot ends past a block edge
        [1500] * 10 + [0] * 6,             # empty slots at the end: cs = T
        [0, 0, 2000] + [0] * 5 + [64] * 8,  # empty slots first and in the middle
        [1] * 16,                          # one segment each
        [2000] * 16,                       # T = 2000
    ]
    lens = np.array([x for r in rows for x in r] * 5, dtype=np.uint32)
    n = len(lens)
    _tune("chunk_packets", chunk)
    try:
        for base in (0, 5, 15):
            ring = synth.random_bytes(stride + base, n * stride + 32)
            view = np.ascontiguousarray(ring[base:base + n * stride])
            dring = _d(ring)
            got = _np(A.chksum_batch_slotted(dring[base:base + n * stride], stride,
                                             _d(lens.view(np.int32))))
            want = oracle.batch_slotted(view, stride, lens)
            assert np.array_equal(got, want), (base, np.nonzero(got != want)[0][:8])
    finally:
        _tune("chunk_packets", 0)


@pytest.fixture
def slot_windows():
    """Setter for the slot_windows tunable (1 = slot windows, 0 = the gathered stream);
    restores the default afterwards."""
    yield lambda v: _tune("slot_windows", v)
    _tune("slot_windows", 0)


@pytest.mark.parametrize("chunk", [0, 1, 8, 16, 64])
@pytest.mark.parametrize("stride", [64, 1517, 2048, 9216, 65536])
def test_slot_windows(oracle, slot_windows, stride, chunk):
    """Slot windows (sum_slot_windows, tunable slot_windows = 1): each packet read on its own
    through a descriptor of exactly its segments, two windows per slot up front, further
    windows for longer packets; lengths 0..min(stride, 65535) at the alignments an odd stride
    and a shifted base give, random slack; the same form on fixed lengths at a gap
    (aipstack_chksum_batch_strided with stride != length, overlapping strides included) and on
    CSR packets; every chunk size."""
    slot_windows(1)
    _tune("chunk_packets", chunk)
    try:
        rng = np.random.default_rng(stride + chunk)
        n = {64: 20000, 1517: 8000, 2048: 8000, 9216: 1500, 65536: 200}[stride]
        cap = min(stride, 65535)
        lens = rng.integers(0, cap + 1, n).astype(np.uint32)
        lens[:8] = [0, 1, 2, cap, cap - 1, 15, 16, 17][:8] if cap > 17 else lens[:8]
        ring = synth.random_bytes(stride + 11, n * stride + 16)
        ring[: 2 * stride] = 0xFF
        dring = _d(ring)
        for base in (0, 5):
            view = ring[base:base + n * stride]
            got = _np(A.chksum_batch_slotted(dring[base:base + n * stride], stride,
                                             _d(lens.view(np.int32)), final=(base == 5)))
            assert np.array_equal(got, oracle.batch_slotted(np.ascontiguousarray(view), stride,
                                                            lens, final=(base == 5)))
        plen = min(stride - 1, 1500) if stride > 1 else 1
        for st, ln in ((stride, plen), (7, 1500), (1, 3000)):
            m = min(n, (ring.size - 16 - ln) // max(st, 1))
            got = _np(A.chksum_batch_strided(dring, st, ln, m, byte_offset=3))
            assert np.array_equal(got, oracle.batch_strided(ring[3:], st, ln, m)), (st, ln)
    finally:
        _tune("chunk_packets", 0)


def test_slot_windows_full_size(oracle, slot_windows):
    """Slot windows on 1 M config-C packets in 2048-B slots and config A's packets in
    2048-B slots (A2K), whole batches against the oracle."""
    slot_windows(1)
    n = 1 << 20
    buf, off = synth.mixed_batch(n)
    ring, lens = synth.to_slots(buf, off, 2048)
    got = _np(A.chksum_batch_slotted(_d(ring), 2048, _d(lens.view(np.int32))))
    assert np.array_equal(got, oracle.batch_slotted(ring, 2048, lens))
    del ring, buf
    b = torch.empty(n * 2048, dtype=torch.uint8, device=DEV)
    synth.fill_device(b, 97)
    got = _np(A.chksum_batch_strided(b, 2048, 1500, n))
    assert np.array_equal(got, oracle.batch_strided(_np(b), 2048, 1500, n))


def test_slotted_full_size_1m(oracle):
    """1 M config-C packets (64-1500 B, odd lengths, all-0x00/0xFF/sum-0 classes) in 2048-B
    ring slots, and 1 M raw frames in 2048-B slots through Rx verify: whole batch vs oracle."""
    n = 1 << 20
    buf, off = synth.mixed_batch(n)
    ring, lens = synth.to_slots(buf, off, 2048)
    got = _np(A.chksum_batch_slotted(_d(ring), 2048, _d(lens.view(np.int32))))
    assert np.array_equal(got, oracle.batch_slotted(ring, 2048, lens))
    del ring, buf
    fr, foff = synth.frames_host(n, seed=71, max_payload=1460)
    oracle.tx_fill_batch(fr, foff)
    _corrupt(fr, foff, 0.1, 3)
    fring, flens = synth.to_slots(fr, foff, 2048)
    v = _np(A.rx_verify_slotted(_d(fring), 2048, _d(flens.view(np.int32))))
    want = oracle.rx_verify_slotted(fring, 2048, flens)
    assert np.array_equal(v, want), np.nonzero(v != want)[0][:10]
    assert np.array_equal(want, oracle.rx_verify_batch(fr, foff))  # same verdicts as CSR


@pytest.mark.parametrize("gather", [1, 2])
@pytest.mark.parametrize("su", [0, -1])
def test_tx_fill_sector_stores_every_alignment(oracle, stream_mode, tx_gather, tx_store, su,
                                              gather):
    """The in-place fill's sector stores (tx_store = 1): the batch starts at each of the 32
    byte offsets of a sector, so both fields' sectors meet every position (inside the frame,
    straddling its start, a field at byte 31); short frames keep 2-byte stores; the bytes
    around the fields, and the frames' neighbours, are rewritten unchanged."""
    stream_mode(su)
    tx_gather(gather)
    tx_store(1)
    buf, off = _edge_frames(5150, 2000)
    for shift in range(32):
        big = synth.random_bytes(shift + 1, buf.size + shift + 64)
        big[shift:shift + buf.size] = buf
        dbig = _d(big)
        st = _np(A.tx_fill(dbig, _d(off + np.uint64(shift)), split=False))
        want = big.copy()
        want_st = oracle.tx_fill_batch(want[shift:shift + buf.size], off)
        assert np.array_equal(st, want_st), shift
        got = _np(dbig)
        assert np.array_equal(got, want), (shift, np.nonzero(got != want)[0][:10])


@pytest.mark.parametrize("store,split", [(0, False), (1, False), (2, False), (0, True)])
@pytest.mark.parametrize("base", [0, 8, 21, 128])
@pytest.mark.parametrize("stride", [1601, 2048])
def test_slotted_tx_fill_store_forms(oracle, tx_store, stride, base, store, split):
    """The send ring's fill forms: one pass with 2-byte, sector or whole-line field stores
    (line stores where the slots lie on the 128-byte grid: stride 2048 at base 0 or 128, else
    the 2-byte stores), and the split slotted fill (aipstack_chksum_tx_fill_slotted_split), at
    slot starts of every alignment an odd stride or a shifted base gives; filled, untouched and
    slack bytes all as the oracle's."""
    tx_store(store)
    buf, off = synth.frames_host(20000, seed=stride + base, max_payload=1460)
    ring, lens = synth.to_slots(buf, off, stride, slack_seed=base + 1)
    big = synth.random_bytes(base + 5, ring.size + base + 16)
    big[base:base + ring.size] = ring
    dbig = _d(big)
    st = _np(A.tx_fill_slotted(dbig[base:base + ring.size], stride, _d(lens.view(np.int32)),
                               split=split))
    want = big.copy()
    want_st = oracle.tx_fill_slotted(want[base:base + ring.size], stride, lens)
    assert np.array_equal(st, want_st)
    got = _np(dbig)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def test_slotted_frame_stride_limit(oracle):
    """The frame batches on slots take slot_stride <= AIPSTACK_CHKSUM_MAX_SLOT_STRIDE (their
    64-frame header window spans at most 4 MiB): 65536 works, 65537 is _EINVAL for every
    slotted frame entry point."""
    import torch
    from aipstack_amd import _lib
    lib = _lib.load()
    buf, off = synth.frames_host(70, seed=3, max_payload=1460)
    ring, lens = synth.to_slots(buf, off, 65536)
    want = ring.copy()
    want_st = oracle.tx_fill_slotted(want, 65536, lens)
    dring = _d(ring)
    st = _np(A.tx_fill_slotted(dring, 65536, _d(lens.view(np.int32))))
    assert np.array_equal(st, want_st) and np.array_equal(_np(dring), want)
    v = _np(A.rx_verify_slotted(dring, 65536, _d(lens.view(np.int32))))
    assert np.array_equal(v, oracle.rx_verify_slotted(want, 65536, lens))
    big = torch.zeros(70 * 65537, dtype=torch.uint8, device=DEV)
    dl = _d(np.full(70, 60, dtype=np.int32))
    out = torch.empty(70, dtype=torch.uint8, device=DEV)
    rec = torch.empty(70, dtype=torch.int64, device=DEV)
    ws = torch.empty(8 * 70, dtype=torch.uint8, device=DEV)
    s = 0
    for st in (lib.aipstack_chksum_rx_verify_slotted(big.data_ptr(), 65537, dl.data_ptr(), 70,
                                                      out.data_ptr(), s),
               lib.aipstack_chksum_tx_fill_slotted(big.data_ptr(), 65537, dl.data_ptr(), 70,
                                                   out.data_ptr(), s),
               lib.aipstack_chksum_tx_fill_records_slotted(big.data_ptr(), 65537, dl.data_ptr(),
                                                           70, rec.data_ptr(), s),
               lib.aipstack_chksum_tx_fill_slotted_split(big.data_ptr(), 65537, dl.data_ptr(), 70,
                                                         out.data_ptr(), ws.data_ptr(), 8 * 70, s)):
        assert st == A.AIPSTACK_CHKSUM_EINVAL


@pytest.mark.parametrize("stride", [1600, 2048, 4096])
def test_slotted_frames_tx_fill_and_records(oracle, stride):
    buf, off = synth.frames_host(30000, seed=stride, max_payload=1460)
    ring, lens = synth.to_slots(buf, off, stride)
    dl = _d(lens.view(np.int32))
    want = ring.copy()
    want_st = oracle.tx_fill_slotted(want, stride, lens)
    rec = _np(A.tx_fill_records_slotted(_d(ring), stride, dl))
    got = ring.copy()
    st = A.apply_tx_records(got, A.slots_to_offsets(lens.size, stride), rec)
    assert np.array_equal(st, want_st) and np.array_equal(got, want)
    dring = _d(ring)
    st2 = _np(A.tx_fill_slotted(dring, stride, dl))
    assert np.array_equal(st2, want_st)
    assert np.array_equal(_np(dring), want)  # fields written, slack untouched
    v = _np(A.rx_verify_slotted(dring, stride, dl))
    assert np.array_equal(v, oracle.rx_verify_slotted(want, stride, lens))


@pytest.mark.parametrize("stride", [128, 256, 2048])
def test_slotted_tx_line_stores_edge_frames(oracle, tx_store, stride):
    """Line stores (tx_store = 2) on the edge-case frames (tests/golden/frame_cases.py: IPv4
    options putting the L4 field past byte 127, short frames with slack in their first line,
    non-IP frames, bad headers) in slots of 128, 256 and 2048 bytes: statuses, fields and
    every other byte, slack included, exactly as the oracle's fill leaves them."""
    tx_store(2)
    buf, off = _edge_frames(91 + stride, 3000)
    keep = np.diff(off) <= stride
    idx = np.nonzero(keep)[0]
    parts = [buf[off[i]:off[i + 1]] for i in idx]
    off2 = np.concatenate([[0], np.cumsum([p.size for p in parts])]).astype(np.int64)
    buf2 = np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)
    ring, lens = synth.to_slots(buf2, off2, stride, slack_seed=stride)
    want = ring.copy()
    want_st = oracle.tx_fill_slotted(want, stride, lens)
    dr = _d(ring)
    st = _np(A.tx_fill_slotted(dr, stride, _d(lens.view(np.int32))))
    assert np.array_equal(st, want_st)
    got = _np(dr)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


@pytest.mark.parametrize("shift", [0, 5])
def test_slotted_edge_frames(oracle, shift):
    buf, off = _edge_frames(77 + shift, 3000)
    ring, lens = synth.to_slots(buf, off, 1600)
    big = np.zeros(ring.size + shift, dtype=np.uint8)
    big[shift:] = ring
    d = _d(big)
    v = _np(A.rx_verify_slotted(d[shift:], 1600, _d(lens.view(np.int32))))
    assert np.array_equal(v, oracle.rx_verify_slotted(ring, 1600, lens))
    assert np.array_equal(v, oracle.rx_verify_batch(buf, off))


def test_slotted_length_over_slot_is_clamped_and_reported(oracle):
    n, stride = 1000, 512
    ring = synth.random_bytes(5, n * stride)
    lens = np.full(n, 300, dtype=np.uint32)
    lens[7] = 600    # > the slot
    lens[9] = 70000  # > the slot and > 65535
    A.contract_violations(0, clear=True)
    got = _np(A.chksum_batch_slotted(_d(ring), stride, _d(lens.view(np.int32))))
    clamped = np.minimum(lens, stride)
    assert np.array_equal(got, oracle.batch_slotted(ring, stride, clamped))
    assert A.contract_violations(0, clear=True) == A.VIOLATION_PACKET_LEN
    A.rx_verify_slotted(_d(ring), stride, _d(lens.view(np.int32)))
    assert A.contract_violations(0, clear=True) == A.VIOLATION_PACKET_LEN


@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("register", [False, True])
def test_engine_slotted(oracle, register, zero_copy):
    """The engine's ring-slot calls from host memory: checksums, Rx verify, Tx fill in place
    (slack bytes untouched), several pieces per batch; bad lengths rejected up front. Both
    copy modes of registered input (read in place, or DMA'd first)."""
    with _engine_copy_mode(zero_copy), A.ChksumEngine(0, chunk_bytes=4 << 20, nstreams=3) as eng:
        buf, off = synth.mixed_batch(40000)
        ring, lens = synth.to_slots(buf, off, 2048)
        if register:
            eng.register(ring)
        assert np.array_equal(eng.slotted(ring, 2048, lens), oracle.batch_slotted(ring, 2048, lens))
        fr, foff = synth.frames_host(30000, seed=72, max_payload=1460)
        fring, flens = synth.to_slots(fr, foff, 2048)
        if register:
            eng.register(fring)
        want = fring.copy()
        want_st = oracle.tx_fill_slotted(want, 2048, flens)
        st = eng.tx_fill_slotted(fring, 2048, flens)
        assert np.array_equal(st, want_st) and np.array_equal(fring, want)
        v = eng.rx_verify_slotted(fring, 2048, flens)
        assert np.array_equal(v, oracle.rx_verify_slotted(fring, 2048, flens))
        bad = flens.copy()
        bad[3] = 2049
        with pytest.raises(A.ChksumError):
            eng.rx_verify_slotted(fring, 2048, bad)
        t, out = eng.submit_slotted(ring, 2048, lens)
        eng.wait(t)
        assert np.array_equal(out, oracle.batch_slotted(ring, 2048, lens))


@pytest.mark.parametrize("zero_copy", [0, 1])
@pytest.mark.parametrize("register", [False, True])
def test_engine_slotted_moves_only_used_slot_prefix(oracle, register, zero_copy):
    """Ring-slot pieces cross PCIe as 2-D copies of each slot's first bytes (the piece's longest
    frame, rounded up to 64): a batch of long frames leaves its bytes in the device staging,
    then batches of short frames (<= 60 / <= 100 B: 64- and 128-byte rows, below the
    112-byte header window) run on the same slots -- the bytes past each row are stale, and
    the results must still be the oracle's."""
    stride = 2048
    with _engine_copy_mode(zero_copy), A.ChksumEngine(0, chunk_bytes=1 << 20, nstreams=2) as eng:
        # (max payload, seed, length cap): capped lengths cut frames short in their slots
        for maxp, seed, cap in ((1460, 3, None), (6, 4, 60), (46, 5, 100), (1460, 6, None),
                                (0, 7, 64), (20, 8, None)):
            fr, foff = synth.frames_host(3000, seed=seed, max_payload=maxp)
            ring, lens = synth.to_slots(fr, foff, stride, slack_seed=seed)
            if cap is not None:
                lens = np.minimum(lens, cap).astype(np.uint32)
            if register:
                eng.register(ring)
            want = ring.copy()
            want_st = oracle.tx_fill_slotted(want, stride, lens)
            assert np.array_equal(eng.tx_fill_slotted(ring, stride, lens), want_st)
            assert np.array_equal(ring, want)
            assert np.array_equal(eng.rx_verify_slotted(ring, stride, lens),
                                  oracle.rx_verify_slotted(ring, stride, lens))
            assert np.array_equal(eng.slotted(ring, stride, lens),
                                  oracle.batch_slotted(ring, stride, lens))
            zero = np.zeros_like(lens)  # every frame empty: nothing crosses PCIe
            assert np.array_equal(eng.slotted(ring, stride, zero),
                                  oracle.batch_slotted(ring, stride, zero))
            if register:
                eng.unregister(ring)


@pytest.mark.parametrize("zero_copy", [1, 0])
@pytest.mark.parametrize("register", [False, True])
def test_engine_ring_receive_loop(oracle, register, zero_copy):
    """A TAP-style receive/send ring driven through the engine's tickets
    (tap/linux/TapDeviceLinux.cpp:156-178: one frame per slot, its length beside it): 8
    regions of 2,048 slots x 2,048 B, several batches in flight; a region is refilled only
    after its previous ticket completed (wait, or poll when it is done), so every wrap reuses
    slots the GPU has finished with. Rx batches (a tenth of the frames corrupted) are checked
    against the oracle's verdicts, Tx batches (filled in place) against the oracle's fill."""
    stride, per, regions = 2048, 2048, 8
    ring = np.zeros(regions * per * stride, dtype=np.uint8)
    raw, soff = synth.frames_host(per * 5, seed=91, max_payload=1460)  # fields zero
    filled = raw.copy()
    oracle.tx_fill_batch(filled, soff)  # what a sender put on the wire
    rng = np.random.default_rng(17)
    with _engine_copy_mode(zero_copy), A.ChksumEngine(0, chunk_bytes=2 << 20, nstreams=3) as eng:
        if register:
            eng.register(ring)
        pending = [None] * regions  # region -> (ticket, kind, out, want)
        done = 0

        def finish(r, block):
            nonlocal done
            t, kind, out, want = pending[r]
            if block:
                eng.wait(t)
            elif not eng.poll(t):
                return False
            region = ring[r * per * stride:(r + 1) * per * stride]
            if kind == "rx":
                assert np.array_equal(out, want), f"region {r}: Rx verdicts differ"
            else:
                want_st, want_bytes = want
                assert np.array_equal(out, want_st), f"region {r}: Tx statuses differ"
                assert np.array_equal(region, want_bytes), f"region {r}: Tx fields differ"
            pending[r] = None
            done += 1
            return True

        for b in range(5 * regions):
            r = b % regions
            if pending[r] is not None:
                finish(r, block=True)
            for q in range(regions):  # complete whatever finished meanwhile, out of order
                if pending[q] is not None:
                    finish(q, block=False)
            # the "read()"s of this region: frames of the source batch, at random rotations
            k = int(rng.integers(0, per * 4))
            fb, fo = (raw if b % 3 == 2 else filled), soff[k:k + per + 1]
            region = ring[r * per * stride:(r + 1) * per * stride]
            slots, lens = synth.to_slots(fb[int(fo[0]):int(fo[-1])], fo - fo[0], stride,
                                         slack_seed=b)
            region[:] = slots
            if b % 3 == 2:
                want_bytes = region.copy()
                want_st = oracle.tx_fill_slotted(want_bytes, stride, lens)
                t, out = eng.submit_tx_fill_slotted(region, stride, lens)
                pending[r] = (t, "tx", out, (want_st, want_bytes))
            else:
                for i in np.nonzero(rng.random(per) < 0.1)[0]:
                    j = int(i) * stride + int(rng.integers(12, int(lens[i])))
                    region[j] ^= np.uint8(1 << int(rng.integers(0, 8)))
                want = oracle.rx_verify_slotted(region, stride, lens)
                t, out = eng.submit_rx_verify_slotted(region, stride, lens)
                pending[r] = (t, "rx", out, want)
        for r in range(regions):
            if pending[r] is not None:
                finish(r, block=True)
        assert done == 5 * regions
        if register:
            eng.unregister(ring)


# ---- several engines in one process (engine group) ----------------------------------------

@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0]])
@pytest.mark.parametrize("register", [False, True])
def test_engine_group(oracle, devices, register):
    """aipstack_chksum_engine_group_*: one process, one engine per listed device (all device 0
    on this box), the batch split into disjoint ranges of about equal bytes, one host thread
    per engine; every result against the oracle, every engine's status 0."""
    with A.ChksumEngineGroup(devices, chunk_bytes=8 << 20, nstreams=2) as grp:
        n = 300000
        buf, off = synth.mixed_batch(n)
        if register:
            grp.register(buf)
        assert np.array_equal(grp.csr(buf, off), oracle.batch_csr(buf, off))
        assert grp.last_status == [0] * len(devices)
        sb = synth.random_bytes(3, 100000 * 1500)
        assert np.array_equal(grp.strided(sb, 1500, 1500, 100000, final=True),
                              oracle.batch_strided(sb, 1500, 1500, 100000, final=True))
        fr, foff = synth.frames_host(200000, seed=81, max_payload=1460)
        if register:
            grp.register(fr)
        want = fr.copy()
        want_st = oracle.tx_fill_batch(want, foff)
        st = grp.tx_fill(fr, foff)
        assert np.array_equal(st, want_st) and np.array_equal(fr, want)
        _corrupt(fr, foff, 0.1, 4)
        assert np.array_equal(grp.rx_verify(fr, foff), oracle.rx_verify_batch(fr, foff))
        if register:
            grp.unregister(fr)
            grp.unregister(buf)
        # fewer packets than engines: the idle engines report 0
        one = grp.csr(buf, off[:2])
        assert one[0] == oracle.batch_csr(buf, off[:2])[0]
        bad = off[:4].copy()
        bad[2] = bad[1] - 1
        with pytest.raises(A.ChksumError):
            grp.csr(buf, bad)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
@pytest.mark.parametrize("register", [False, True])
def test_engine_group_ring_slots(oracle, devices, register):
    """The engine group on a ring of 2048-B slots: contiguous runs of slots per engine;
    checksums, Rx verify and Tx fill in place against the oracle; a length over the slot
    rejected before any engine starts (the ring unchanged)."""
    with A.ChksumEngineGroup(devices, chunk_bytes=4 << 20, nstreams=2) as grp:
        fr, foff = synth.frames_host(60000, seed=83, max_payload=1460)
        ring, lens = synth.to_slots(fr, foff, 2048)
        if register:
            grp.register(ring)
        want = ring.copy()
        want_st = oracle.tx_fill_slotted(want, 2048, lens)
        assert np.array_equal(grp.tx_fill_slotted(ring, 2048, lens), want_st)
        assert np.array_equal(ring, want) and grp.last_status == [0] * len(devices)
        assert np.array_equal(grp.rx_verify_slotted(ring, 2048, lens),
                              oracle.rx_verify_slotted(ring, 2048, lens))
        assert np.array_equal(grp.slotted(ring, 2048, lens, final=True),
                              oracle.batch_slotted(ring, 2048, lens, final=True))
        bad = lens.copy()
        bad[-1] = 2049
        before = ring.copy()
        with pytest.raises(A.ChksumError):
            grp.tx_fill_slotted(ring, 2048, bad)
        assert np.array_equal(ring, before)
        if register:
            grp.unregister(ring)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_engine_group_async_tickets(oracle, devices):
    """Group tickets (aipstack_chksum_engine_group_submit_* / _poll / _wait): large batches
    split over every engine (pageable ones submitted by the devices' worker threads, registered
    ones on the calling thread), small ones whole on one engine in turn; several tickets in
    flight, completed out of order, every result against the oracle; a registered region is
    read in place by every engine; each engine reports its locality."""
    with A.ChksumEngineGroup(devices, chunk_bytes=4 << 20, nstreams=2) as grp:
        loc = grp.locality()
        assert len(loc) == len(devices) and all(c >= 0 for _, c in loc)
        assert len({l for l in loc}) == 1  # one device, one locality
        big, boff = synth.mixed_batch(200000)                      # ~160 MB: split
        fr, foff = synth.frames_host(100000, seed=91, max_payload=1460)
        reg, roff = synth.mixed_batch(60000)                       # registered
        grp.register(reg)
        assert grp.region_mapped(reg)
        small = [synth.frames_host(64, seed=300 + i, max_payload=1460) for i in range(2 * len(devices))]
        t_big, o_big = grp.submit_csr(big, boff, final=True)
        want_fr = fr.copy()
        want_st = oracle.tx_fill_batch(want_fr, foff)
        t_tx, st_tx = grp.submit_tx_fill(fr, foff)
        t_reg, o_reg = grp.submit_csr(reg, roff)
        t_small = [grp.submit_rx_verify(b, o) for b, o in small]
        for (t, out), (b, o) in zip(reversed(t_small), reversed(small)):
            grp.wait(t)
            assert np.array_equal(out, oracle.rx_verify_batch(b, o))
        while not grp.poll(t_reg):
            pass
        assert np.array_equal(o_reg, oracle.batch_csr(reg, roff))
        grp.wait(t_tx)
        assert np.array_equal(st_tx, want_st) and np.array_equal(fr, want_fr)
        assert grp.last_status == [0] * len(devices)
        grp.wait(t_big)
        assert np.array_equal(o_big, oracle.batch_csr(big, boff, final=True))
        grp.wait(t_big)  # completing a ticket again is a no-op
        ring, lens = synth.to_slots(*synth.frames_host(20000, seed=92, max_payload=1460), 2048)
        want = ring.copy()
        want_st = oracle.tx_fill_slotted(want, 2048, lens)
        t, st = grp.submit_tx_fill_slotted(ring, 2048, lens)
        t2, v = grp.submit_rx_verify_slotted(want, 2048, lens)
        grp.wait(t2)
        grp.wait(t)
        assert np.array_equal(st, want_st) and np.array_equal(ring, want)
        assert np.array_equal(v, oracle.rx_verify_slotted(want, 2048, lens))
        grp.unregister(reg)


def _need_devices(k):
    have = torch.cuda.device_count()
    if have < k:
        pytest.skip(f"needs {k} or more GPUs, this box shows {have}: the distinct-device path "
                    "is rehearsed on device 0 alone by the tests above")
    return have


def test_engine_group_distinct_devices(oracle):
    """The engine group over every visible device, each a distinct GPU (VERDICT round 4, item
    5): a registered region is mapped for every device's kernels (zero copy on each device's
    own mapping); synchronous and ticketed batches split over all of them are bit-exact; every
    device reports status 0 and its own locality. Skips below two GPUs."""
    n_dev = _need_devices(2)
    devices = list(range(n_dev))
    with A.ChksumEngineGroup(devices, chunk_bytes=8 << 20, nstreams=2) as grp:
        assert grp.size == n_dev and len(grp.locality()) == n_dev
        n = 60000 * n_dev  # ~48 MB per device: split over every device (>= 4 MiB each)
        buf, off = synth.mixed_batch(n)
        grp.register(buf)
        assert grp.region_mapped(buf), "a device's kernels cannot read the registered region"
        assert np.array_equal(grp.csr(buf, off), oracle.batch_csr(buf, off))
        assert grp.last_status == [0] * n_dev
        t, o = grp.submit_csr(buf, off, final=True)
        sb = synth.random_bytes(5, 40000 * n_dev * 1500)  # pageable: the devices' workers stage
        t2, o2 = grp.submit_strided(sb, 1500, 1500, 40000 * n_dev)
        grp.wait(t2)
        assert np.array_equal(o2, oracle.batch_strided(sb, 1500, 1500, 40000 * n_dev))
        while not grp.poll(t):
            pass
        assert np.array_equal(o, oracle.batch_csr(buf, off, final=True))
        assert grp.last_status == [0] * n_dev
        fr, foff = synth.frames_host(50000 * n_dev, seed=85, max_payload=1460)
        want = fr.copy()
        want_st = oracle.tx_fill_batch(want, foff)
        assert np.array_equal(grp.tx_fill(fr, foff), want_st) and np.array_equal(fr, want)
        grp.unregister(buf)


def test_engine_group_distinct_devices_one_failing():
    """The fault program's group cases (one device's piece made to fail; a wait and a poll of
    that ticket from two threads) on devices 0 and 1. Skips below two GPUs."""
    _need_devices(2)
    exe = os.path.join(ROOT, "tests", "cpp", "build", "engine_fault_test")
    assert os.path.exists(exe), f"{exe} not built (make -C tests/cpp gpu)"
    env = dict(os.environ, AIPSTACK_FAULT_GROUP_DEVICES="0,1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_bench_torchrun_distinct_devices():
    """bench.py under torchrun with one rank per visible GPU, as the driver launches it: every
    rank on its own device (per_gpu.distinct_devices), every shard bit-exact. Skips below two
    GPUs (test_bench_two_ranks_one_gpu rehearses the flow on one)."""
    import json
    import socket
    n_dev = _need_devices(2)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k != "AIPSTACK_BENCH_FORCE_DEVICE"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(n_dev), "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py",
           "--gpus", str(n_dev), "--steps", "5", "--warmup", "2", "--cpu-reps", "1",
           "--no-ceiling"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip()][-1])
    assert d["n_gpus"] == n_dev and d["parity"].startswith(f"bit-exact (each of {n_dev}")
    assert d["per_gpu"]["distinct_devices"] is True, d["per_gpu"]["devices"]
    assert len(set(d["per_gpu"]["devices"])) == n_dev


def test_engine_slotted_frame_stride_limit():
    """The engine's and the group's frame submits on slots reject slot_stride > 65536 before
    any work; the checksum form has no such limit."""
    ring = np.zeros(4 * 65537, dtype=np.uint8)
    lens = np.full(4, 60, dtype=np.uint32)
    with A.ChksumEngine(0, chunk_bytes=1 << 20) as eng:
        with pytest.raises(A.ChksumError):
            eng.rx_verify_slotted(ring, 65537, lens)
        with pytest.raises(A.ChksumError):
            eng.tx_fill_slotted(ring, 65537, lens)
        assert eng.slotted(ring, 65537, lens).shape == (4,)
    with A.ChksumEngineGroup([0, 0], chunk_bytes=1 << 20) as grp:
        with pytest.raises(A.ChksumError):
            grp.rx_verify_slotted(ring, 65537, lens)


def test_engine_group_submit_check_failures_leave_no_ticket():
    """A group submit whose argument checks fail returns _EINVAL before anything starts and
    sets *ticket = 0 (chksum.h, section 4): decreasing CSR offsets, a packet over 65535 bytes,
    a slot length over the stride, a frame slot stride over 65536."""
    from aipstack_amd import _lib
    lib = _lib.load()
    buf = np.zeros(1 << 20, dtype=np.uint8)
    out16 = np.zeros(4, dtype=np.uint16)
    out8 = np.zeros(4, dtype=np.uint8)
    p = lambda a: a.ctypes.data  # noqa: E731
    with A.ChksumEngineGroup([0, 0], chunk_bytes=1 << 20) as grp:
        t = ctypes.c_uint64(123)
        bad = np.array([0, 100, 50], dtype=np.uint64)
        assert lib.aipstack_chksum_engine_group_submit_csr(
            grp._h, p(buf), p(bad), 2, p(out16), 0, ctypes.byref(t)) == A.AIPSTACK_CHKSUM_EINVAL
        assert t.value == 0
        t.value = 123
        long = np.array([0, 70000], dtype=np.uint64)
        assert lib.aipstack_chksum_engine_group_submit_rx_verify(
            grp._h, p(buf), p(long), 1, p(out8), ctypes.byref(t)) == A.AIPSTACK_CHKSUM_EINVAL
        assert t.value == 0
        t.value = 123
        lens = np.array([60, 2049], dtype=np.uint32)
        assert lib.aipstack_chksum_engine_group_submit_slotted(
            grp._h, p(buf), 2048, p(lens), 2, p(out16), 0, ctypes.byref(t)) == A.AIPSTACK_CHKSUM_EINVAL
        assert t.value == 0
        t.value = 123
        lens = np.array([60, 60], dtype=np.uint32)
        assert lib.aipstack_chksum_engine_group_submit_tx_fill_slotted(
            grp._h, p(buf), 65537, p(lens), 2, p(out8), ctypes.byref(t)) == A.AIPSTACK_CHKSUM_EINVAL
        assert t.value == 0
        t.value = 123
        assert lib.aipstack_chksum_engine_group_submit_strided(
            grp._h, p(buf), 1500, 70000, 2, p(out16), 0, ctypes.byref(t)) == A.AIPSTACK_CHKSUM_EINVAL
        assert t.value == 0
        # a good batch still goes through afterwards
        good = np.array([0, 1500, 3000], dtype=np.uint64)
        assert np.array_equal(grp.csr(buf, good), np.zeros(2, dtype=np.uint16))


def test_bench_e2e_engine_group_line():
    """bench.py --e2e --engines 3 (all on device 0 here): one JSON line, bit-exact, the
    engines and their devices named."""
    import json
    env = dict(os.environ, AIPSTACK_BENCH_FORCE_DEVICE="0")
    r = subprocess.run([sys.executable, "bench.py", "--e2e", "--engines", "3", "--config", "C",
                        "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip()][-1])
    assert d["parity"].startswith("bit-exact") and d["value"] > 0
    assert d["config"]["engines"] == 3 and d["config"]["engine_devices"] == [0, 0, 0]


@pytest.mark.parametrize("config,pageable,engines", [("RX2K", False, 0), ("C2K", True, 0),
                                                     ("RX2K", False, 2), ("TX2K", False, 0),
                                                     ("TX2K", True, 2)])
def test_bench_e2e_ring_slots_line(config, pageable, engines):
    """bench.py --e2e on a receive ring (RX2K / C2K, 2048-B slots; also through an engine group
    of 2 on the one device): one JSON line, bit-exact against the oracle over every slot; the
    value counts frame bytes, not slot bytes."""
    import json
    cmd = [sys.executable, "bench.py", "--e2e", "--config", config, "--steps", "2", "--warmup", "1"]
    if pageable:
        cmd.append("--e2e-pageable")
    if engines:
        cmd += ["--engines", str(engines)]
    env = dict(os.environ, AIPSTACK_BENCH_FORCE_DEVICE="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip()][-1])
    assert d["parity"].startswith("bit-exact") and d["value"] > 0
    assert d["config"]["slot_stride"] == 2048
    assert d["metric"].startswith({"RX2K": "GiB/s Rx-verified", "TX2K": "GiB/s Tx-filled"}.get(
        config, "GiB/s checksummed"))


@pytest.mark.parametrize("config,split", [("TX2K", False), ("TX2K", True), ("TX", True)])
def test_bench_tx_fill_lines(config, split):
    """bench.py --config TX2K (a send ring filled in place on the device) and TX, in the
    default one-pass form and with --tx-split (read pass + scatter pass): one JSON line,
    every frame filled as the oracle fills it, the form named in the config."""
    import json
    r = subprocess.run([sys.executable, "bench.py", "--config", config, "--steps", "5",
                        "--warmup", "5", "--no-cpu-baseline", "--no-ceiling"]
                       + (["--tx-split"] if split else []), cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.strip()][-1])
    assert d["parity"].startswith("bit-exact") and d["roofline"]["frac"] > 0
    if config == "TX2K":
        assert d["config"]["slot_stride"] == 2048
    assert d["config"]["tx_fill"].startswith("split" if split else "in-place")


# ---- frame decisions pinned by the reference's own call sites (tests/golden/frame_ref.py) ---

@pytest.fixture(scope="module")
def frame_ref_sets():
    from conftest import load_frame_ref_sets
    return load_frame_ref_sets()


@pytest.mark.parametrize("su", [0, -1])
@pytest.mark.parametrize("name", ["edge", "mix", "mix_filled"])
def test_rx_verify_matches_reference_call_sites(frame_ref_sets, stream_mode, name, su):
    """GPU Rx verdicts against the verdicts composed from the reference's compiled call
    sites (ref_cs_ip4_rx, _tcp_rx, _udp_rx, _icmp) recorded in frame_ref_cases.json."""
    stream_mode(su)
    doc, sets, fr = frame_ref_sets
    buf, off = sets[name]
    want = np.array([fr.verdict(buf[int(off[i]):int(off[i + 1])], r)
                     for i, r in enumerate(doc[name])], dtype=np.uint8)
    got = _np(A.rx_verify(_d(buf), _d(off)))
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


@pytest.mark.parametrize("how", ["one_pass", "split", "records"])
@pytest.mark.parametrize("name", ["edge", "mix", "mix_filled"])
def test_tx_fill_matches_reference_call_sites(frame_ref_sets, name, how):
    """GPU Tx field values against the reference send side's values (ref_cs_ip4_rx with the
    field 0, ref_cs_tcp_rx / _udp_tx / _icmp over the zeroed datagram): every written field
    is the reference's, and no other byte changes."""
    doc, sets, fr = frame_ref_sets
    buf, off = sets[name]
    want = buf.copy()
    for i, r in enumerate(doc[name]):
        s0 = int(off[i])
        for at, v in fr.fill_fields(buf[s0:int(off[i + 1])], r):
            want[s0 + at], want[s0 + at + 1] = v >> 8, v & 0xFF
    if how == "records":
        got = buf.copy()
        A.apply_tx_records(got, off, _np(A.tx_fill_records(_d(buf), _d(off))))
    else:
        dbuf = _d(buf)
        A.tx_fill(dbuf, _d(off), split=how == "split")
        got = _np(dbuf)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


# ---- hipGraph capture: the batch entry points never allocate or synchronise ----------------

def test_batches_captured_in_a_graph_and_replayed(oracle):
    """Strided, CSR, Rx verify and the split Tx fill captured once into one HIP graph
    (torch.cuda.CUDAGraph) and replayed over new bytes written into the same buffers: every
    replay matches the oracle (the calls are graph-capturable)."""
    n, plen = 4096, 1500
    sbuf = torch.empty(n * plen, dtype=torch.uint8, device=DEV)
    hbuf, off = synth.mixed_batch(3000)
    cbuf = torch.empty(hbuf.size, dtype=torch.uint8, device=DEV)
    coff = _d(off)
    fr, foff = synth.frames_host(2000, seed=5)
    rbuf = torch.empty(fr.size, dtype=torch.uint8, device=DEV)
    tbuf = torch.empty(fr.size, dtype=torch.uint8, device=DEV)
    dfoff = _d(foff)
    ws = torch.empty(8 * 2000, dtype=torch.uint8, device=DEV)
    s_out = torch.empty(n, dtype=torch.uint16, device=DEV)
    c_out = torch.empty(3000, dtype=torch.uint16, device=DEV)
    r_out = torch.empty(2000, dtype=torch.uint8, device=DEV)
    t_out = torch.empty(2000, dtype=torch.uint8, device=DEV)

    def step():
        A.chksum_batch_strided(sbuf, plen, plen, n, out=s_out)
        A.chksum_batch_csr(cbuf, coff, out=c_out, final=True)
        A.rx_verify(rbuf, dfoff, out=r_out)
        A.tx_fill(tbuf, dfoff, out=t_out, workspace=ws, split=True)

    step()  # warm-up outside the capture (the library caches the device's CU count)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for rep in range(3):
        rng = np.random.default_rng(100 + rep)
        sh = rng.integers(0, 256, n * plen, dtype=np.uint8)
        ch = rng.integers(0, 256, hbuf.size, dtype=np.uint8)
        rx = fr.copy()
        oracle.tx_fill_batch(rx, foff)
        _corrupt_rx = rng.random(2000) < 0.2
        for i in np.nonzero(_corrupt_rx)[0]:
            rx[int(foff[i]) + int(rng.integers(14, int(foff[i + 1] - foff[i])))] ^= 0x10
        tx = fr.copy()
        sbuf.copy_(torch.from_numpy(sh))
        cbuf.copy_(torch.from_numpy(ch))
        rbuf.copy_(torch.from_numpy(rx))
        tbuf.copy_(torch.from_numpy(tx))
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(_np(s_out), oracle.batch_strided(sh, plen, plen, n))
        assert np.array_equal(_np(c_out), oracle.batch_csr(ch, off, final=True))
        assert np.array_equal(_np(r_out), oracle.rx_verify_batch(rx, foff))
        want_st = oracle.tx_fill_batch(tx, foff)
        assert np.array_equal(_np(t_out), want_st)
        assert np.array_equal(_np(tbuf), tx)


# ---- batch shapes: every packets-per-chunk size on every kernel family ---------------------

@pytest.fixture
def chunk_packets():
    """Yields a setter for the chunk-size tunable; restores automatic afterwards."""
    yield lambda v: _tune("chunk_packets", v)
    _tune("chunk_packets", 0)


@pytest.mark.parametrize("cpk", [1, 2, 8, 32, 64])
def test_every_chunk_size_on_every_kernel(oracle, chunk_packets, cpk):
    """Forced packets per chunk (the small-batch shapes of DESIGN 6.7, and 64): strided
    back-to-back and slotted, CSR, seeded CSR, chains, Rx verify and both Tx fills stay
    bit-exact at a ragged count that leaves a partial last chunk."""
    chunk_packets(cpk)
    n = 3001
    # strided, back to back (stream mode) and in 2 KiB slots (wave mode)
    for stride in (1500, 2048):
        host = synth.random_bytes(60 + stride, n * stride + 5)
        d = _d(host)
        got = _np(A.chksum_batch_strided(d, stride, 1500, n, byte_offset=5))
        assert np.array_equal(got, oracle.batch_strided(host, stride, 1500, n, base_off=5))
    # CSR and seeded CSR (config C's construction)
    hbuf, off = synth.mixed_batch(n)
    dbuf, doff = _d(hbuf), _d(off)
    assert np.array_equal(_np(A.chksum_batch_csr(dbuf, doff, final=True)),
                          oracle.batch_csr(hbuf, off, final=True))
    states = np.random.default_rng(cpk).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = _np(A.chksum_batch_seeded_csr(dbuf, doff, _d(states.view(np.int32))))
    assert np.array_equal(got, oracle.batch_seeded_csr(hbuf, off, states))
    # chains: header node + 1-2 payload pieces of one buffer, some empty chains
    rng = np.random.default_rng(100 + cpk)
    addrs, lens, idx, sts, want = [], [], [0], [], []
    for i in range(n):
        chunks = []
        if i % 17 != 0:
            for _ in range(int(rng.integers(1, 4))):
                o = int(rng.integers(0, hbuf.size - 1600))
                chunks.append((o, int(rng.integers(0, 1500))))
        st = int(rng.integers(0, 2**32))
        flat = np.concatenate([hbuf[o:o + l] for o, l in chunks] + [np.zeros(0, np.uint8)])
        want.append(oracle.chain(st, flat, [(0, flat.size)] if flat.size else []))
        for o, l in chunks:
            if l:
                addrs.append(dbuf.data_ptr() + o)
                lens.append(l)
        idx.append(len(addrs))
        sts.append(st)
    got = _np(A.chksum_batch_chain(_d(np.array(addrs, dtype=np.int64)),
                                   _d(np.array(lens, dtype=np.int32)),
                                   _d(np.array(idx, dtype=np.int64)),
                                   _d(np.array(sts, dtype=np.uint32).view(np.int32)), final=True))
    assert np.array_equal(got, np.array(want, dtype=np.uint16))
    # frames: Rx verify on filled + corrupted frames, Tx fill both ways
    fr, foff = synth.frames_host(n, seed=70 + cpk)
    rx = fr.copy()
    oracle.tx_fill_batch(rx, foff)
    _corrupt(rx, foff, 0.2, cpk)
    assert np.array_equal(_np(A.rx_verify(_d(rx), _d(foff))), oracle.rx_verify_batch(rx, foff))
    for split in (False, True):
        d = _d(fr)
        st = _np(A.tx_fill(d, _d(foff), split=split))
        want_fr = fr.copy()
        assert np.array_equal(st, oracle.tx_fill_batch(want_fr, foff))
        assert np.array_equal(_np(d), want_fr)


@pytest.mark.parametrize("n", [1, 63, 65, 2047, 2049, 65535, 65537, 4095 * 64, 4096 * 64 + 1])
def test_batch_sizes_at_shape_boundaries(oracle, n):
    """Automatic shapes at the batch sizes where the chunk size or the regime changes
    (256 CUs: 2048 / 65536 packets, 4096 chunks of 64), CSR and strided."""
    hbuf, off = synth.mixed_batch(n)
    assert np.array_equal(_np(A.chksum_batch_csr(_d(hbuf), _d(off))), oracle.batch_csr(hbuf, off))
    host = synth.random_bytes(n, n * 1500)
    assert np.array_equal(_np(A.chksum_batch_strided(_d(host), 1500, 1500, n)),
                          oracle.batch_strided(host, 1500, 1500, n))


# ---- chain fill: the Tx call sites' checksum written into the header node ------------------

def test_chain_fill_tcp_tx_shape(oracle):
    """tcp/IpTcpProto_output.h:1251-1277: pseudo-header State + 20-60 B TCP header node (its
    checksum field at offset 16 reading 0) + 1-2 send-ring chunks; chain_fill stores each
    checksum big-endian into its header and returns the same values as the chained batch."""
    import torch
    rng = np.random.default_rng(77)
    n = 50000
    ring = rng.integers(0, 256, size=1 << 21, dtype=np.uint8)
    hdrs = rng.integers(0, 256, size=n * 64, dtype=np.uint8)
    hl = 20 + 4 * rng.integers(0, 11, n)
    for i in range(n):
        hdrs[64 * i + 16: 64 * i + 18] = 0            # the checksum field reads 0
    dring, dh = _d(ring), _d(hdrs)
    addrs, lens, idx, states, fields = [], [], [0], [], []
    for i in range(n):
        addrs.append(dh.data_ptr() + 64 * i)
        lens.append(int(hl[i]))
        seg = int(rng.integers(0, 1461))
        start = int(rng.integers(0, ring.size))
        first = min(seg, ring.size - start)
        if first:
            addrs.append(dring.data_ptr() + start)
            lens.append(first)
        if seg > first:
            addrs.append(dring.data_ptr())
            lens.append(seg - first)
        idx.append(len(addrs))
        states.append(int(rng.integers(0, 2**20)))
        fields.append(dh.data_ptr() + 64 * i + 16)
    args = (_d(np.array(addrs, dtype=np.int64)), _d(np.array(lens, dtype=np.int32)),
            _d(np.array(idx, dtype=np.int64)), _d(np.array(states, dtype=np.int32)))
    want = _np(A.chksum_batch_chain(*args, final=True))
    got = _np(A.chksum_chain_fill(*args, _d(np.array(fields, dtype=np.int64))))
    torch.cuda.synchronize()
    assert np.array_equal(got, want)
    filled = _np(dh)
    expect = hdrs.copy()
    for i in range(n):
        expect[64 * i + 16] = want[i] >> 8
        expect[64 * i + 17] = want[i] & 0xFF
    assert np.array_equal(filled, expect)
    # and the filled header now verifies: the chain sums to 0xFFFF, IpChksum == 0
    again = _np(A.chksum_batch_chain(*args, final=True))
    assert np.all(again == 0)


def test_chain_fill_udp_zero_as_ffff_and_skipped_fields():
    """udp/IpUdpProto.h:176-178: a computed 0 goes out as 0xFFFF (flag), else as 0; a field
    address of 0 stores nothing; odd field addresses."""
    import torch
    n = 64
    buf = torch.zeros(4096, dtype=torch.uint8, device=DEV)
    base = buf.data_ptr()
    # chain i: 8 zero bytes at 33 + 40 i (a UDP header, checksum field at +6) with state
    # 0xFFFF -> sum 0xFFFF -> final checksum 0
    addr = torch.tensor([base + 33 + 40 * i for i in range(n)], dtype=torch.int64, device=DEV)
    ln = torch.full((n,), 8, dtype=torch.int32, device=DEV)
    idx = torch.arange(n + 1, dtype=torch.int64, device=DEV)
    st = torch.full((n,), 0xFFFF, dtype=torch.int32, device=DEV)
    fields = torch.tensor([base + 33 + 40 * i + 6 if i % 5 else 0 for i in range(n)],
                          dtype=torch.int64, device=DEV)
    out = _np(A.chksum_chain_fill(addr, ln, idx, st, fields))
    assert np.all(out == 0)
    assert int(buf.sum().item()) == 0  # 0 written as 0x0000
    out = _np(A.chksum_chain_fill(addr, ln, idx, st, fields, zero_as_ffff=True))
    torch.cuda.synchronize()
    assert np.all(out == 0xFFFF)
    h = _np(buf)
    for i in range(n):
        f = 33 + 40 * i + 6
        assert (h[f], h[f + 1]) == ((0xFF, 0xFF) if i % 5 else (0, 0)), i


@pytest.mark.parametrize("args", [["-r", "4", "256"], ["-g", "2", "-r", "4", "256"],
                                  ["-s", "-r", "4", "64", "256"],
                                  ["-s", "-g", "2", "-r", "4", "64"]])
def test_ring_loop_program(args):
    """tools/ring_loop from C++ over the C-ABI: the registered receive ring (ring mode), and
    the descriptor-driven loop (-s): frames read() one per slot from a SOCK_SEQPACKET
    socketpair into a registered ring and Rx-verified, frames Tx-filled in a send ring and
    write()n to a second socketpair whose consumer compares each with the oracle's fill; with
    one engine and with an engine group (-g 2). Every verdict and every sent frame exact."""
    import json
    exe = os.path.join(ROOT, "tools", "build", "ring_loop")
    assert os.path.exists(exe), f"{exe} not built (make -C tools)"
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines and all(d["parity"].startswith("bit-exact") for d in lines), lines
