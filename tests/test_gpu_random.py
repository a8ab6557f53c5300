"""Randomised GPU parity: seeded scenarios that draw the batch shape, the lengths, the
alignment and the byte classes at random for every entry point, each against the oracle
(bit-exact). The fixed-shape tests in test_gpu_parity.py pin the BASELINE configs and the
reference's cases; these widen the inputs the way a stack would mix them: packets of 0 to
65535 bytes at any byte address, long runs of 0x00 / 0xFF, strided batches whose stride
exceeds the length, ring slots of any size, chains of up to 9 chunks anywhere in memory
(separate allocations included), seeded states, frames of every class with corruptions.
"""
import numpy as np
import pytest

import aipstack_amd as A
from aipstack_amd import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda"
SCENARIOS = 100


def _d(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _np(t):
    return t.cpu().numpy()


def _tune(key, value):
    from aipstack_amd import _lib
    assert _lib.load().aipstack_chksum_tune(key.encode(), value) == A.AIPSTACK_CHKSUM_OK


def _blob(rng, nbytes):
    """Random bytes with runs of 0x00 and 0xFF (the reference's zero rule and its all-ones
    known answer) and runs of one repeated word."""
    b = rng.integers(0, 256, size=nbytes, dtype=np.uint8)
    for _ in range(int(rng.integers(1, 12))):
        s = int(rng.integers(0, nbytes))
        e = min(nbytes, s + int(rng.integers(1, 70000)))
        b[s:e] = rng.choice([0x00, 0xFF, int(rng.integers(0, 256))])
    return b


def _lengths(rng, n, cap=65535):
    """A mixture: empty, tiny (odd included), Ethernet-sized, jumbo, and a few near the cap."""
    kind = rng.integers(0, 100, size=n)
    lens = np.where(kind < 5, 0,
           np.where(kind < 25, rng.integers(1, 64, size=n),
           np.where(kind < 85, rng.integers(64, 1515, size=n),
           np.where(kind < 98, rng.integers(1515, 9001, size=n),
                    rng.integers(max(cap - 600, 0), cap + 1, size=n)))))
    return np.minimum(lens, cap).astype(np.int64)


@pytest.mark.parametrize("seed", range(SCENARIOS))
def test_random_packet_batches(oracle, seed):
    rng = np.random.default_rng(1000 + seed)
    # ---- CSR (+ seeded): packets back to back from an odd or even base
    n = int(rng.integers(1, 2500))
    lens = _lengths(rng, n)
    base = int(rng.integers(0, 64))
    off = np.concatenate([[0], np.cumsum(lens)]) + base
    blob = _blob(rng, int(off[-1]) + 64)
    db = _d(blob)
    final = bool(rng.integers(0, 2))
    got = _np(A.chksum_batch_csr(db, _d(off), final=final))
    assert np.array_equal(got, oracle.batch_csr(blob, off, final=final)), seed
    states = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    got = _np(A.chksum_batch_seeded_csr(db, _d(off), _d(states.view(np.int32))))
    assert np.array_equal(got, oracle.batch_seeded_csr(blob, off, states)), seed
    # ---- strided: stride >= length, any byte offset
    length = int(_lengths(rng, 1)[0])
    stride = max(1, length + int(rng.integers(0, 3)) * int(rng.integers(1, 4097)))
    ns = int(rng.integers(1, max(2, min(3000, (blob.size - 64) // max(stride, 1)))))
    bo = int(rng.integers(0, 64))
    if bo + (ns - 1) * stride + length <= blob.size:
        got = _np(A.chksum_batch_strided(db, stride, length, ns, byte_offset=bo, final=final))
        want = oracle.batch_strided(blob, stride, length, ns, final=final, base_off=bo)
        assert np.array_equal(got, want), (seed, stride, length, ns, bo)
    # ---- ring slots of any stride
    slot = int(rng.choice([64, 100, 1536, 2048, 4096, 9216, 65536]))
    nsl = int(rng.integers(1, max(2, min(3000, (blob.size // slot)))))
    sl = np.minimum(_lengths(rng, nsl, cap=min(slot, 65535)), min(slot, 65535)).astype(np.uint32)
    if nsl * slot <= blob.size:
        ring = blob[:nsl * slot]
        got = _np(A.chksum_batch_slotted(_d(ring), slot, _d(sl.view(np.int32)), final=final))
        assert np.array_equal(got, oracle.batch_slotted(ring, slot, sl, final=final)), (seed, slot)


@pytest.mark.parametrize("seed", range(SCENARIOS))
def test_random_chains(oracle, seed):
    """Chains of 0-9 chunks of 0-3000 bytes (a few up to 65535) anywhere in two separate
    device allocations, with or without states, inverted or final."""
    rng = np.random.default_rng(2000 + seed)
    b1 = _blob(rng, 1 << 20)
    b2 = _blob(rng, 300000)
    d1, d2 = _d(b1), _d(b2)
    n = int(rng.integers(1, 1500))
    addr, clen, index, per_chain = [], [], [0], []
    for _ in range(n):
        chunks = []
        for _ in range(int(rng.integers(0, 10))):
            big = rng.random() < 0.02
            ln = int(rng.integers(0, 65536 if big else 3001))
            if rng.random() < 0.3:
                ln = min(ln, b2.size)
                o = int(rng.integers(0, b2.size - ln + 1))
                addr.append(d2.data_ptr() + o)
                chunks.append((2, o, ln))
            else:
                o = int(rng.integers(0, b1.size - ln + 1))
                addr.append(d1.data_ptr() + o)
                chunks.append((1, o, ln))
            clen.append(ln)
        per_chain.append(chunks)
        index.append(len(addr))
    use_states = bool(rng.integers(0, 2))
    states = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    final = bool(rng.integers(0, 2))
    got = _np(A.chksum_batch_chain(
        _d(np.array(addr, dtype=np.uint64).view(np.int64)) if addr else torch.zeros(1, dtype=torch.int64, device=DEV),
        _d(np.array(clen, dtype=np.uint32).view(np.int32)) if clen else torch.zeros(1, dtype=torch.int32, device=DEV),
        _d(np.array(index, dtype=np.uint64).view(np.int64)),
        _d(states.view(np.int32)) if use_states else None, final=final))
    # the oracle walks one chain at a time over one host array: both blobs side by side
    host = np.concatenate([b1, b2])
    for i, chunks in enumerate(per_chain):
        flat = [((o if which == 1 else b1.size + o), ln) for which, o, ln in chunks]
        want = oracle.chain(int(states[i]) if use_states else 0, host, flat)
        if not final:
            want = (~want) & 0xFFFF
        assert got[i] == want, (seed, i, chunks)


@pytest.mark.parametrize("seed", range(SCENARIOS // 2))
def test_random_tx_chains(oracle, seed):
    """TCP-Tx-shaped chains (tcp/IpTcpProto_output.h:1251-1277): a header node in a header
    area, then payload pieces cut back to back from one send buffer -- the layout the chain
    kernel reads as column runs under AIPSTACK_CHKSUM_JUST_WRITTEN (chksum_chain_kernel COLS)
    -- with short and empty pieces, long pieces (up to 65535), headers that are not lone
    short chunks, chains without a header or without payload, and now and then a piece taken
    from elsewhere (the slice falls back to the gathered stream). With and without the hint,
    through the chained batch and the chain fill, against the oracle."""
    rng = np.random.default_rng(4000 + seed)
    n = int(rng.integers(1, 2000))
    hstride = int(rng.choice([20, 24, 32, 40, 64]))
    hbytes = hstride * n + 256
    pieces, total = [], 0
    for i in range(n):
        k = int(rng.integers(0, 5))
        ps = []
        for _ in range(k):
            r = rng.random()
            ln = (int(rng.integers(0, 3)) if r < 0.05 else int(rng.integers(1, 129)) if r < 0.25
                  else int(rng.integers(20000, 65536)) if r < 0.27 else int(rng.integers(129, 1500)))
            ps.append(ln)
            total += ln
        pieces.append(ps)
    blob = _blob(rng, hbytes + total + 4096)
    hoff = int(rng.integers(0, 16))
    poff = hbytes + int(rng.integers(0, 16))
    d = _d(blob)
    base = d.data_ptr()
    addr, clen, index, flat_all = [], [], [0], []
    p = poff
    for i in range(n):
        flat = []
        if rng.random() < 0.95:  # the header node (sometimes long, sometimes elsewhere)
            hl = int(rng.integers(1, hstride + 1)) if rng.random() < 0.97 else int(rng.integers(129, 400))
            ho = hoff + hstride * i if hl <= hstride else int(rng.integers(0, hbytes - hl))
            addr.append(base + ho); clen.append(hl); flat.append((ho, hl))
        for ln in pieces[i]:
            if rng.random() < 0.01:  # a piece from elsewhere: not back to back
                o = int(rng.integers(0, blob.size - ln))
                addr.append(base + o); clen.append(ln); flat.append((o, ln))
            else:
                addr.append(base + p); clen.append(ln); flat.append((p, ln))
            p += ln
        index.append(len(addr))
        flat_all.append(flat)
    states = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    want = np.array([oracle.chain(int(states[i]), blob, flat_all[i]) for i in range(n)],
                    dtype=np.uint16)
    da = _d(np.array(addr or [0], dtype=np.uint64).view(np.int64))
    dl = _d(np.array(clen or [0], dtype=np.uint32).view(np.int32))
    di = _d(np.array(index, dtype=np.uint64).view(np.int64))
    ds = _d(states.view(np.int32))
    for jw in (False, True):
        got = _np(A.chksum_batch_chain(da, dl, di, ds, final=True, just_written=jw))
        assert np.array_equal(got, want), (seed, jw, np.nonzero(got != want)[0][:8])
    # the chain fill (fields in a separate buffer, zero before the fill)
    fbuf = torch.zeros(2 * n, dtype=torch.uint8, device=DEV)
    fields = _d((fbuf.data_ptr() + 2 * np.arange(n, dtype=np.uint64)).view(np.int64))
    got = _np(A.chksum_chain_fill(da, dl, di, ds, fields, just_written=True))
    assert np.array_equal(got, want), (seed, np.nonzero(got != want)[0][:8])
    stored = _np(fbuf).reshape(n, 2)
    assert np.array_equal(stored[:, 0].astype(np.uint16) << 8 | stored[:, 1], want)


@pytest.mark.parametrize("seed", range(SCENARIOS // 2))
def test_random_frames(oracle, seed):
    """Frame batches of random size and payload cap, Tx-filled on the GPU (one pass and
    split) and in ring slots, then corrupted and Rx-verified, all against the frame oracle."""
    rng = np.random.default_rng(3000 + seed)
    n = int(rng.integers(1, 6000))
    fr, off = synth.frames_host(n, seed=4000 + seed, max_payload=int(rng.choice([0, 46, 600, 1460, 8000])))
    want = fr.copy()
    want_st = oracle.tx_fill_batch(want, off)
    # in-place field stores: 2-byte (0), whole sectors (1), whole lines (2: ring slots on the
    # 128-byte grid; elsewhere the 2-byte stores)
    store = int(rng.integers(0, 3))
    _tune("tx_store", store)
    try:
        for split in (False, True):
            d = _d(fr)
            st = _np(A.tx_fill(d, _d(off), split=split))
            assert np.array_equal(st, want_st) and np.array_equal(_np(d), want), (seed, split)
    finally:
        _tune("tx_store", -1)
    # corrupt a random fraction of the filled frames, then verify
    bad = want.copy()
    for i in np.nonzero(rng.random(n) < 0.2)[0]:
        s, e = int(off[i]), int(off[i + 1])
        if e - s > 12:
            j = s + int(rng.integers(12, e - s))
            bad[j] ^= np.uint8(1 << int(rng.integers(0, 8)))
    got = _np(A.rx_verify(_d(bad), _d(off)))
    assert np.array_equal(got, oracle.rx_verify_batch(bad, off)), seed
    # the same frames in ring slots (lengths capped at random: cut frames included)
    stride = int(rng.choice([2048, 4096, 9216, 16384]))
    if int(np.diff(off).max()) <= stride:
        ring, lens = synth.to_slots(bad, off, stride, slack_seed=seed)
        if rng.random() < 0.3:
            lens = np.minimum(lens, rng.integers(0, stride, size=lens.size)).astype(np.uint32)
        got = _np(A.rx_verify_slotted(_d(ring), stride, _d(lens.view(np.int32))))
        assert np.array_equal(got, oracle.rx_verify_slotted(ring, stride, lens)), (seed, stride)
        dr = _d(ring)
        split = bool(rng.integers(0, 2))
        _tune("tx_store", store)
        try:
            st = _np(A.tx_fill_slotted(dr, stride, _d(lens.view(np.int32)), split=split))
        finally:
            _tune("tx_store", -1)
        wr = ring.copy()
        assert np.array_equal(st, oracle.tx_fill_slotted(wr, stride, lens)), (seed, stride, split)
        assert np.array_equal(_np(dr), wr), (seed, stride, split)
