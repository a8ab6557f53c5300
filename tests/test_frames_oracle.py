"""Frame-level oracle (oracle/frame_oracle.c) on the CPU.

The checksum arithmetic under it is pinned by the golden vectors; here its frame logic is
cross-checked against the independent host mirror of the reference interface
(aipstack_amd.IpChksumAccumulator / IpBufRef, itself checked against the reference's
golden chains), and every verdict is exercised by constructed corruptions."""
import numpy as np
import pytest

import aipstack_amd as A
from aipstack_amd import synth

RX = {v: k for k, v in A.RX_VERDICTS.items()}


def be16(b, o):
    return (int(b[o]) << 8) | int(b[o + 1])


@pytest.fixture(scope="module")
def frames():
    buf, off = synth.frames_host(4000, seed=5, max_payload=1600)
    return buf, off


def test_synth_frames_mix(frames):
    buf, off = frames
    lens = np.diff(off)
    assert lens.min() >= 60 and np.any(off[:-1] % 2 == 1)
    eth = np.array([be16(buf, int(o) + 12) for o in off[:-1]])
    assert 0.02 < np.mean(eth == 0x0806) < 0.07
    protos = np.array([buf[int(o) + 23] for o in off[:-1]])[eth == 0x0800]
    for p, lo in ((6, 0.4), (17, 0.2), (1, 0.05), (47, 0.02)):
        assert np.mean(protos == p) > lo


def test_fill_then_verify_accepts_everything(frames, oracle):
    buf, off = frames[0].copy(), frames[1]
    st = oracle.tx_fill_batch(buf, off)
    v = oracle.rx_verify_batch(buf, off)
    ok = {RX["NOT_IP4"], RX["ACCEPT"], RX["ACCEPT_OTHER"], RX["FRAGMENT"]}
    assert set(np.unique(v)) <= ok
    assert np.array_equal(st, v)     # statuses of the fill = verdicts of the check
    assert np.count_nonzero(v == RX["ACCEPT"]) > 3000


def _mirror_l4(b, ip, hl, total, proto):
    """Expected L4 checksum via the host mirror of IpChksumAccumulator (pseudo-header
    words + IpBufRef over the datagram with the checksum field zeroed)."""
    dg = bytearray(b[ip + hl: ip + total])
    if proto == 17:
        dg = dg[:be16(dg, 4)]
    fld = {6: 16, 17: 6, 1: 2}[proto]
    dg[fld:fld + 2] = b"\0\0"
    acc = A.IpChksumAccumulator()
    if proto in (6, 17):
        acc.addWord32((int(b[ip + 12]) << 24) | (int(b[ip + 13]) << 16) | be16(b, ip + 14))
        acc.addWord32((int(b[ip + 16]) << 24) | (int(b[ip + 17]) << 16) | be16(b, ip + 18))
        acc.addWord16(proto)
        acc.addWord16(len(dg))
    c = acc.getChksum(A.IpBufRef(A.IpBufNode(bytes(dg), len(dg)), 0, len(dg)))
    return 0xFFFF if (proto == 17 and c == 0) else c


def test_fill_matches_host_mirror(frames, oracle):
    buf, off = frames[0].copy(), frames[1]
    st = oracle.tx_fill_batch(buf, off)
    checked = 0
    for i in range(0, 4000, 3):
        if st[i] != RX["ACCEPT"]:
            continue
        ip = int(off[i]) + 14
        hl = int(buf[ip] & 15) * 4
        total = be16(buf, ip + 2)
        proto = int(buf[ip + 9])
        fld = ip + hl + {6: 16, 17: 6, 1: 2}[proto]
        assert be16(buf, fld) == _mirror_l4(buf, ip, hl, total, proto), i
        hdr = bytearray(buf[ip: ip + hl])
        hdr[10:12] = b"\0\0"
        assert be16(buf, ip + 10) == A.IpChksum(bytes(hdr))
        checked += 1
    assert checked > 900


def _one(frame_bytes, oracle):
    b = np.frombuffer(bytes(frame_bytes), dtype=np.uint8).copy()
    return oracle.lib.oracle_rx_verify(b.ctypes.data, b.size)


@pytest.mark.parametrize("mutate,verdict", [
    (lambda f, ip: f.__setitem__(slice(12, 14), b"\x86\xdd"), "NOT_IP4"),
    (lambda f, ip: f.__setitem__(ip, 0x65), "DROP_IP_MALFORMED"),          # version 6
    (lambda f, ip: f.__setitem__(ip, 0x44), "DROP_IP_MALFORMED"),          # IHL 4
    (lambda f, ip: f.__setitem__(ip + 2, 0xFF), "DROP_IP_MALFORMED"),      # total_len > frame
    (lambda f, ip: f.__setitem__(ip + 8, f[ip + 8] ^ 1), "DROP_IP_CHKSUM"),  # TTL bit
    (lambda f, ip: f.__setitem__(ip + 13, f[ip + 13] ^ 0x80), "DROP_IP_CHKSUM"),
    (lambda f, ip: f.__setitem__(len(f) - 1 if f[ip + 3] + 14 >= len(f) else ip + 40,
                                 f[ip + 40] ^ 0x10), "DROP_L4_CHKSUM"),
])
def test_constructed_corruptions(frames, oracle, mutate, verdict):
    buf, off = frames[0].copy(), frames[1]
    st = oracle.tx_fill_batch(buf, off)
    # a TCP frame with IHL 5 and >= 40 bytes of datagram
    for i in range(4000):
        f0 = int(off[i])
        ip = f0 + 14
        if st[i] == RX["ACCEPT"] and buf[ip] == 0x45 and buf[ip + 9] == 6 and be16(buf, ip + 2) >= 60:
            break
    fr = bytearray(buf[f0:int(off[i + 1])])
    assert _one(fr, oracle) == RX["ACCEPT"]
    mutate(fr, 14)
    assert _one(fr, oracle) == RX[verdict]


def test_udp_zero_checksum_and_short_frames(frames, oracle):
    buf, off = frames[0].copy(), frames[1]
    st = oracle.tx_fill_batch(buf, off)
    for i in range(4000):
        ip = int(off[i]) + 14
        if st[i] == RX["ACCEPT"] and buf[ip + 9] == 17:
            break
    fr = bytearray(buf[int(off[i]):int(off[i + 1])])
    hl = (fr[14] & 15) * 4
    fr[14 + hl + 6: 14 + hl + 8] = b"\0\0"
    assert _one(fr, oracle) == RX["ACCEPT_NO_CHKSUM"]
    fr[14 + hl + 4: 14 + hl + 6] = b"\0\x07"                       # UDP length 7 < 8
    assert _one(fr, oracle) == RX["DROP_L4_MALFORMED"]
    assert _one(b"\x00" * 13, oracle) == RX["NOT_IP4"]
    assert _one(bytes(12) + b"\x08\x00" + bytes(10), oracle) == RX["DROP_IP_MALFORMED"]


# ---- edge-case frames (tests/golden/frame_cases.py) ------------------------------------

def _edge_frames():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import frame_cases
    return frame_cases


def test_edge_frames_cover_every_verdict(oracle):
    fc = _edge_frames()
    buf, off = fc.pack(fc.frames())
    v = oracle.rx_verify_batch(buf, off)
    counts = np.bincount(v, minlength=9)
    assert np.all(counts > 0), counts.tolist()


def test_edge_frames_zero_sum_checksums_verify(oracle):
    """L4 data whose sum is 0 mod 0xFFFF: the computed checksum is 0x0000; a field of
    0xFFFF (the other zero) verifies too (Chksum.h:245-250 folds both to 0xFFFF)."""
    fc = _edge_frames()
    frs = fc.frames(seed=99, n=4000)
    hits = {0: 0, 0xFFFF: 0}
    for fr in frs:
        b = np.frombuffer(fr, dtype=np.uint8)
        if oracle.rx_verify_batch(b.copy(), np.array([0, len(fr)], dtype=np.uint64))[0] != RX["ACCEPT"]:
            continue
        if fr[23] not in (1, 6):
            continue
        l4 = 14 + (fr[14] & 15) * 4
        co = l4 + (16 if fr[23] == 6 else 2)
        c = be16(fr, co)
        if c not in hits:
            continue
        hits[c] += 1
        alt = bytearray(fr)
        alt[co:co + 2] = (c ^ 0xFFFF).to_bytes(2, "big")
        a = np.frombuffer(bytes(alt), dtype=np.uint8).copy()
        assert oracle.rx_verify_batch(a, np.array([0, len(fr)], dtype=np.uint64))[0] == RX["ACCEPT"]
    assert hits[0] > 5 and hits[0xFFFF] > 5, hits


def test_edge_frames_fill_then_verify(oracle):
    fc = _edge_frames()
    buf, off = fc.pack(fc.frames())
    st = oracle.tx_fill_batch(buf, off)
    v = oracle.rx_verify_batch(buf, off)
    filled = st == RX["ACCEPT"]
    assert filled.sum() > 1000
    assert np.all(v[filled] == RX["ACCEPT"])
    # statuses other than ACCEPT are exactly the verdicts that stop before an L4 sum
    assert np.all(st[~filled] == v[~filled])


# ---- the frame decisions pinned by the reference's own call sites -------------------------
# tests/golden/frame_ref_cases.json: per frame, the answers of the reference stack's checksum
# call sequences compiled against its Chksum.h/Buf.h (ref_cs_ip4_rx / _tcp_rx / _udp_rx /
# _udp_tx / _icmp), composed by tests/golden/frame_ref.py. The C frame oracle must give the
# same verdicts and write the same field values.

@pytest.fixture(scope="module")
def frame_ref_sets():
    from conftest import load_frame_ref_sets
    return load_frame_ref_sets()


@pytest.mark.parametrize("name", ["edge", "mix", "mix_filled"])
def test_frame_oracle_verdicts_match_reference_call_sites(frame_ref_sets, oracle, name):
    doc, sets, fr = frame_ref_sets
    buf, off = sets[name]
    recs = doc[name]
    assert len(recs) == off.size - 1
    want = np.array([fr.verdict(buf[int(off[i]):int(off[i + 1])], r) for i, r in enumerate(recs)],
                    dtype=np.uint8)
    got = oracle.rx_verify_batch(buf, off)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    if name != "mix":
        assert set(np.unique(want).tolist()) >= {2, 5, 6, 8}


@pytest.mark.parametrize("name", ["edge", "mix", "mix_filled"])
def test_frame_oracle_fill_matches_reference_call_sites(frame_ref_sets, oracle, name):
    doc, sets, fr = frame_ref_sets
    buf, off = sets[name]
    filled = buf.copy()
    oracle.tx_fill_batch(filled, off)
    nfields = 0
    want = buf.copy()
    for i, r in enumerate(doc[name]):
        s = int(off[i])
        for at, v in fr.fill_fields(buf[s:int(off[i + 1])], r):
            want[s + at], want[s + at + 1] = v >> 8, v & 0xFF
            nfields += 1
    assert nfields > len(doc[name])  # most frames get both fields
    assert np.array_equal(filled, want), np.nonzero(filled != want)[0][:10]
